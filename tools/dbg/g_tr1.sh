set -u
mkdir -p gpurun_out/tr1
for D in 128 256; do
TRACE_D=$D SGM_TRACE=gpurun_out/tr1/s$D.%d timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr1_$D.log 2>&1 || { tail gpurun_out/tr1_$D.log; exit 1; }
ls gpurun_out/tr1
python tools/dbg/trace_analyze.py $(ls gpurun_out/tr1/s$D.* | tail -1)
done
rm -rf gpurun_out/tr1
