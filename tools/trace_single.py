"""SGM_TRACE timeline of a single-frame census paths launch (sgm_match_device: census ->
paths8 -> WTA): per-direction wave durations and the number of resident path waves over the
launch, to see whether a frame is throughput-bound or ends in a partly-filled tail (DESIGN
§8.3, C5).

    SGM_TRACE=gpurun_out/tr.bin python tools/trace_single.py --config c5
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

CFG = {"c2": (1920, 1080, 128), "c3": (1920, 1080, 256), "c5": (4096, 3000, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    W, H, D = CFG[a.config]
    eng = pkg.Engine(0, pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, subpixel=1, lr_check=1, median=0))
    l, r, _ = synth.stereo_pair(H, W, 0, D, seed=5, with_truth=False)
    dl, dr = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    out = torch.empty((H, W), dtype=torch.int16, device="cuda")
    st = torch.cuda.Stream()
    for _ in range(2):
        eng.match_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, st.cuda_stream)
        st.synchronize()
    eng.close()
    t = np.fromfile(os.environ["SGM_TRACE"], np.uint64).reshape(-1, 4)
    t = t[t[:, 3] > 0]
    s0 = t[:, 2].astype(np.int64)
    s1 = t[:, 3].astype(np.int64)
    T0 = s0.min()
    s0 = (s0 - T0) / 100.0                       # 100 MHz timestamps -> us
    s1 = (s1 - T0) / 100.0
    span = s1.max()
    it = (t[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    dirs = (it >> 24) & 0xF
    dur = s1 - s0
    print(f"{a.config}: {len(t)} path waves, span {span:.1f} us, busy {dur.sum():.0f} wave-us "
          f"(mean resident {dur.sum() / span:.0f} waves)")
    for d in range(8):
        m = dirs == d
        if m.any():
            print(f"  dir {d}: waves {m.sum():5d}  start max {s0[m].max():8.1f}  end max {s1[m].max():8.1f}  "
                  f"dur mean {dur[m].mean():8.1f} max {dur[m].max():8.1f} us")
    ts = np.linspace(0, span, 21)[:-1] + span / 40
    conc = [int(((s0 <= x) & (s1 > x)).sum()) for x in ts]
    print("  resident waves at 2.5, 7.5, ... 97.5 % of the span:", conc)


if __name__ == "__main__":
    main()
