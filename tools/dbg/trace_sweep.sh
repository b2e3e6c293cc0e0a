set -u
for k in 2 4 8; do
  SGM_PERSIST=$k SGM_TRACE=gpurun_out/trace_$k.bin timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr_$k.log 2>&1 || exit $?
  SGM_PRIO=1 SGM_PERSIST=$k SGM_TRACE=gpurun_out/trace_p$k.bin timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr_p$k.log 2>&1 || exit $?
done
