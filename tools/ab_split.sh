#!/bin/bash
# GPU box: interleaved A/B of the split single census frame (sgm_api.cpp split_steps) against
# the one-launch schedule, by SGM_SPLIT value ("auto" = unset, 0 = off, or a fraction).
#   bash tools/ab_split.sh CONFIGS ROUNDS value1 value2 ...
set -u
CF=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = auto ]; then unset SGM_SPLIT; else export SGM_SPLIT=$v; fi
    timeout -k 10 300 python tools/single_frame.py --configs $CF --reps 20 2>/dev/null \
      | grep '^{' | sed "s/^{/{\"split\": \"$v\", /" >> gpurun_out/ab_split.jsonl || exit 1
  done
done
unset SGM_SPLIT
