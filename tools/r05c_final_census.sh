#!/bin/bash
# round-5 GPU step: ILV bytes at 1080p, then the census measurement refresh at the session's build
set -u
bash tools/r05c_ilv_pmc.sh || exit 1
bash tools/refresh_profiles.sh r05c "$(cat gpurun_out/REV 2>/dev/null || echo unknown)" || exit 1
echo final-census-done
