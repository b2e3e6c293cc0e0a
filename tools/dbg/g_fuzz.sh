set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
SGM_FUZZ_CASES=${N:-600} timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fuzz.log 2>&1; rc=$?
tail -5 gpurun_out/t_fuzz.log
exit $rc
