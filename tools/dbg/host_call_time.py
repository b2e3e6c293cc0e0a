"""Host-side time per sgm_match_device call (no sync) vs GPU time per frame."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import __graft_entry__ as ge
pkg = ge.load_package()
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
h, w = 1080, 1920
p = pkg.default_params(pkg.MODE_OCV_SGBM5, num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)
eng = pkg.Engine(0, p)
l, r, _ = synth.stereo_pair(h, w, 0, 128, seed=3)
dl, dr = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
out = torch.empty((h, w), dtype=torch.int16, device="cuda")
st = torch.cuda.Stream()
run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), w, h, w, out.data_ptr(), w, st.cuda_stream)
run(); st.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    calls = []
    for _ in range(10):
        a = time.perf_counter(); run(); calls.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    st.synchronize()
    t2 = time.perf_counter()
    print(f"issue {1e3*(t1-t0)/10:.3f} ms/call (max {1e3*max(calls):.3f}) total {1e3*(t2-t0)/10:.3f} ms/frame", flush=True)
