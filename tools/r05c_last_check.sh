#!/bin/bash
# round-5 GPU step: smoke + the default bench line on the final tree (the library as the driver
# will load it)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05c_smoke_last.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r05c_bench_last.log 2>&1 || exit 1
grep '^{' gpurun_out/r05c_bench_last.log > gpurun_out/r05c_bench_last.json
echo last-check-done
