"""SGM_TRACE timelines of a 6-frame C3 batch in the up+WTA scheme: per traced launch, block
counts and durations by kind (up+WTA / row sweeps / horizontal / census) and the span."""
import os, sys, glob
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import __graft_entry__ as ge
from conftest import _load
pkg = ge.load_package()
synth = _load("sgm_synth", ge.PKG_DIR + "/synth.py")
eng = pkg.Engine(0)
W, H, D = 1920, 1080, int(os.environ.get("TD", "256"))
eng.set_params(pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
N = 6
frames = [synth.stereo_pair(H, W, 0, D, seed=1 + i, with_truth=False) for i in range(N)]
dl = [torch.from_numpy(f[0]).cuda() for f in frames]
dr = [torch.from_numpy(f[1]).cuda() for f in frames]
out = torch.empty((N, H, W), dtype=torch.int16, device="cuda")
st = torch.cuda.Stream()
for rep in range(2):
    eng.match_device_batch([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], W, H, W,
                           [out[i].data_ptr() for i in range(N)], W, st.cuda_stream)
    st.synchronize()
pat = os.environ["SGM_TRACE"]
files = sorted(glob.glob(pat.replace("%d", "*")), key=lambda f: int(f.rsplit(".", 1)[-1]))
for fn in files[-4:]:
    a = np.fromfile(fn, np.uint64).reshape(-1, 4)
    a = a[a[:, 3] > 0]
    kind = (a[:, 0] >> np.uint64(62)).astype(int)
    item = (a[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    d = (item >> 24) & 0xFF
    t0 = a[:, 2].astype(np.int64); t1 = a[:, 3].astype(np.int64)
    T0 = t0.min(); s0 = (t0 - T0) / 100.0; s1 = (t1 - T0) / 100.0   # us
    print(f"== {fn}: span {s1.max():.0f} us, {len(a)} waves")
    for name, m in [("up+wta", (kind == 0) & (d == 8)), ("rows", (kind == 0) & (d < 6)),
                    ("horiz", (kind == 0) & ((d == 6) | (d == 7))), ("census", kind == 2)]:
        if m.sum() == 0: continue
        dur = s1[m] - s0[m]
        print(f"  {name:7s} waves {m.sum():6d} start {s0[m].min():7.0f}-{s0[m].max():7.0f} end max {s1[m].max():7.0f} "
              f"dur mean {dur.mean():7.1f} max {dur.max():7.1f}")

# occupancy over time of the steady launch (second-to-last traced file is the k=ng-1 launch;
# take the one with the most up+WTA waves and census blocks: a steady launch)
best = None
for fn in files:
    a = np.fromfile(fn, np.uint64).reshape(-1, 4)
    a = a[a[:, 3] > 0]
    kind = (a[:, 0] >> np.uint64(62)).astype(int)
    d = ((a[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.int64) >> 24) & 0xFF
    if ((kind == 0) & (d == 8)).sum() > 0 and (kind == 2).sum() > 0:
        best = fn
if best:
    a = np.fromfile(best, np.uint64).reshape(-1, 4)
    a = a[a[:, 3] > 0]
    kind = (a[:, 0] >> np.uint64(62)).astype(int)
    d = ((a[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.int64) >> 24) & 0xFF
    t0 = a[:, 2].astype(np.int64); t1 = a[:, 3].astype(np.int64)
    T0 = t0.min(); s0 = (t0 - T0) / 100.0; s1 = (t1 - T0) / 100.0
    span = s1.max()
    print(f"== occupancy of {best} (span {span:.0f} us): active waves per 100 us [up+wta rows horiz census]")
    for b in np.arange(0, span, 100):
        act = (s0 < b + 100) & (s1 > b)
        print(f"  {b:6.0f} {int((act & (kind == 0) & (d == 8)).sum()):5d} {int((act & (kind == 0) & (d < 6)).sum()):5d} "
              f"{int((act & (kind == 0) & (d >= 6) & (d < 8)).sum()):5d} {int((act & (kind == 2)).sum()):5d}")
