"""SGM_TRACE timeline of the fused launch (paths of group k + WTA of group k-1 + census):
runs a 4-frame C3 batch (the dump keeps the last traced launch = the fused one) and prints
per-kind block counts, durations and concurrency over the launch."""
import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import __graft_entry__ as ge
from conftest import _load
pkg = ge.load_package()
synth = _load("sgm_synth", ge.PKG_DIR + "/synth.py")
eng = pkg.Engine(0)
W, H, D = 1920, 1080, 256
eng.set_params(pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
frames = [synth.stereo_pair(H, W, 0, D, seed=1 + i) for i in range(4)]
dl = [torch.from_numpy(f[0]).cuda() for f in frames]
dr = [torch.from_numpy(f[1]).cuda() for f in frames]
out = torch.empty((4, H, W), dtype=torch.int16, device="cuda")
st = torch.cuda.Stream()
for rep in range(3):
    eng.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], W, H, W,
                           [out[i].data_ptr() for i in range(4)], W, st.cuda_stream)
    st.synchronize()
a = np.fromfile(os.environ["SGM_TRACE"], np.uint64).reshape(-1, 4)
a = a[a[:, 3] > 0]
kind = (a[:, 0] >> np.uint64(62)).astype(int)
t0 = a[:, 2].astype(np.int64); t1 = a[:, 3].astype(np.int64)
T0 = t0.min()
s0 = (t0 - T0) / 100.0; s1 = (t1 - T0) / 100.0
span = s1.max()
print(f"records {len(a)} span {span:.1f} us")
names = {0: "paths", 1: "wta", 2: "census"}
for k in range(3):
    m = kind == k
    if m.any():
        d = s1[m] - s0[m]
        print(f"  {names[k]:6s}: waves {m.sum():5d}  start [{s0[m].min():7.1f}, {s0[m].max():7.1f}]  end max {s1[m].max():7.1f}"
              f"  dur mean {d.mean():7.1f} p50 {np.median(d):7.1f} max {d.max():7.1f} us  busy {d.sum():.0f} wave-us")
if (kind == 0).any():
    it = a[kind == 0, 0].astype(np.int64)
    dirs = (it >> 24) & 0xF
    for dd in range(8):
        m = dirs == dd
        if m.any():
            d = (s1[kind == 0] - s0[kind == 0])[m]
            print(f"    dir {dd}: waves {m.sum():5d} dur mean {d.mean():7.1f} max {d.max():7.1f}")
ts = np.linspace(0, span, 21)
for k in range(3):
    conc = [int(((s0 <= t) & (s1 > t) & (kind == k)).sum()) for t in ts]
    print(f"  concurrent {names[k]:6s} waves at 0..100% (5% steps):", conc)
