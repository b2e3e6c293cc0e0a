"""OCV-mode batch throughput: sgm_match_device_batch of N frames with 1..4 stream lanes."""
import os, sys
sys.path.insert(0, "/root/repo")
import torch
import __graft_entry__ as ge
pkg = ge.load_package()
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
cases = [("C1", pkg.MODE_OCV_SGBM5, 480, 640, {}),
         ("1080p SGBM D128", pkg.MODE_OCV_SGBM5, 1080, 1920, dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)),
         ("1080p HH D128", pkg.MODE_OCV_HH8, 1080, 1920, dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0))]
n = 12
for name, mode, h, w, kw in cases:
    p = pkg.default_params(mode, **kw)
    eng = pkg.Engine(0, p)
    fr = [synth.stereo_pair(h, w, max(p.min_disparity, 0), p.num_disparities, seed=i, with_truth=False) for i in range(4)]
    dl = [torch.from_numpy(fr[i % 4][0]).cuda() for i in range(n)]; dr = [torch.from_numpy(fr[i % 4][1]).cuda() for i in range(n)]
    outs = torch.empty((n, h, w), dtype=torch.int16, device="cuda"); st = torch.cuda.Stream()
    args = ([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, w, [outs[i].data_ptr() for i in range(n)], w, st.cuda_stream)
    for lanes in ("1", "2", "3", "4"):
        os.environ["SGM_OCV_STREAMS"] = lanes
        eng.match_device_batch(*args); st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            eng.match_device_batch(*args)
        e1.record(st); st.synchronize()
        print(f"{name:18s} lanes {lanes}: {e0.elapsed_time(e1) / (3 * n):.3f} ms/frame", flush=True)
    eng.close()
