# SGM_TRACE timelines of the single-frame path launch at D = 512 (and 256 for scale)
set -u
mkdir -p gpurun_out/tr5
for D in 512 256; do
TRACE_D=$D SGM_TRACE=gpurun_out/tr5/s$D.%d timeout -k 10 200 python tools/dbg/trace_run.py > gpurun_out/tr5_$D.log 2>&1 || { tail gpurun_out/tr5_$D.log; exit 1; }
python tools/dbg/trace_analyze.py $(ls gpurun_out/tr5/s$D.* | tail -1)
done
rm -rf gpurun_out/tr5
