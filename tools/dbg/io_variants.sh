set -u
export TMPDIR=/tmp
env | grep -i -E "sdma|hsa_|hip_|gpu_|roc" | sort
for v in "SGM_IO_PRIO=0" "SGM_IO_PRIO=1" "SGM_IO_PRIO=1 HSA_ENABLE_SDMA=1" "SGM_IO_PRIO=0 HSA_ENABLE_SDMA=1"; do
  env $v SGM_IO_TRACE=1 timeout -k 10 300 python bench.py --steps 6 --no-cpu-baseline --host-io > gpurun_out/b_host.log 2>&1 || { tail gpurun_out/b_host.log; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/b_host.log) $(grep 'sgm io' gpurun_out/b_host.log | tail -1 | cut -c1-60)"
done
