"""GPU timings of the OpenCV-SGBM restatement modes (the reference's own matcher,
matcherOpenCVSGBM.cpp) beside the CPU restatement on the same inputs, device buffers,
HIP events around each match. Prints one JSON line per case.

    python tools/ocv_modes_bench.py [--reps 10]
Cases: C1 (640x480, node defaults: minD 9, D 64, block 15, MODE_SGBM 5 paths + median +
speckle) and 1920x1080 D=128 in MODE_SGBM / MODE_HH.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU restatement (1 thread)")
    ap.add_argument("--case", default="", help="run only the cases whose name contains this")
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    orc = ge._load_file("sgm_oracle", os.path.join(ROOT, "oracle", "sgm_oracle.py")) if a.cpu else None
    cases = [
        ("C1 640x480 node defaults MODE_SGBM", 480, 640, pkg.MODE_OCV_SGBM5, {}),
        ("1920x1080 D=128 MODE_SGBM block 5", 1080, 1920, pkg.MODE_OCV_SGBM5,
         dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)),
        ("1920x1080 D=128 MODE_HH block 5", 1080, 1920, pkg.MODE_OCV_HH8,
         dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)),
    ]
    eng = pkg.Engine(0)
    st = torch.cuda.Stream()
    for name, h, w, mode, kw in cases:
        if a.case not in name:
            continue
        p = pkg.default_params(mode, **kw)
        eng.set_params(p)
        left, right, _ = synth.stereo_pair(h, w, max(p.min_disparity, 0), p.num_disparities, seed=3)
        dl = torch.from_numpy(left).cuda()
        dr = torch.from_numpy(right).cuda()
        out = torch.empty((h, w), dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), w, h, w, out.data_ptr(), w, st.cuda_stream)
            run()
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                run()
            e1.record(st)
            st.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        rec = {"case": name, "gpu_ms_per_frame": round(ms, 3), "gpu_pairs_per_s": round(1000.0 / ms, 1)}
        if orc is not None:
            d = {k: v for k, v in p.as_dict().items() if k != "mode"}
            op = orc.make_params(mode, **d)
            orc.set_threads(1)
            t0 = time.perf_counter()
            ref = orc.match(op, left, right)
            rec["cpu_ms_per_frame_1thread"] = round((time.perf_counter() - t0) * 1e3, 1)
            rec["bit_exact"] = bool(np.array_equal(out.cpu().numpy(), ref))
        print(json.dumps(rec), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
