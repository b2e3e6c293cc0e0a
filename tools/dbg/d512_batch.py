"""A/B of the batch schemes (SGM_UPWTA=1/0) on several geometries, N frames, interleaved."""
import os, sys
sys.path.insert(0, "/root/repo")
import numpy as np, torch
import __graft_entry__ as ge
pkg = ge.load_package()
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
cases = [tuple(int(v) for v in c.split("x")) for c in os.environ.get("CASES", "1080x1920x256").split(",")]
n = int(os.environ.get("NF", "32"))
for (H, W, D) in cases:
    eng = pkg.Engine(0, pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
    fr = [synth.stereo_pair(H, W, 0, D, seed=i, with_truth=False) for i in range(4)]
    dl = [torch.from_numpy(fr[i % 4][0]).cuda() for i in range(n)]; dr = [torch.from_numpy(fr[i % 4][1]).cuda() for i in range(n)]
    outs = torch.empty((n, H, W), dtype=torch.int16, device="cuda"); st = torch.cuda.Stream()
    args = ([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], W, H, W, [outs[i].data_ptr() for i in range(n)], W, st.cuda_stream)
    for rnd in range(2):
        for up in ("1", "0"):
            os.environ["SGM_UPWTA"] = up
            eng.match_device_batch(*args); st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.set_profiling(True)
            e0.record(st); eng.match_device_batch(*args); e1.record(st); st.synchronize()
            stg = eng.stage_times(); eng.set_profiling(False)
            print(H, W, D, "upwta", up, round(e0.elapsed_time(e1) / n, 3), "ms/frame", [(a, round(b, 3)) for a, b, _ in stg], flush=True)
    eng.close()
