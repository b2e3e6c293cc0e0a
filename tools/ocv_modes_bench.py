"""GPU timings of the OpenCV-SGBM restatement modes (the reference's own matcher,
matcherOpenCVSGBM.cpp) beside the CPU restatement on the same inputs, device buffers,
HIP events around each match. Prints one JSON line per case.

    python tools/ocv_modes_bench.py [--reps 10]
Cases: C1 (640x480, node defaults: minD 9, D 64, block 15, MODE_SGBM 5 paths + median +
speckle), 1920x1080 D=128 in MODE_SGBM / MODE_HH, and the reference's shipped SGBM launch
config (launch/stereo_matcher.launch:37-48 at the capture size of stereo_capture.launch:14-15:
2448x2048, minD 147, D 480, block 21, cap 7, uniqueness 2, speckle 1000/4, P1 200, P2 400)
in MODE_SGBM / MODE_HH, gated (int16 volumes unless a cost leaves int16) and with the static
int32 volumes (SGM_OCV_GATE=0), and the processing launch's SGBM search
(launch/stereo_processing.launch:65-66: minD 0, D 752, the rest of stereo_matcher.launch:39-47) at
the same size: D > 512, so full int16 volumes (no deficits), 64-bit path offsets and a 64-lane
line whose lanes carry 16 values (752 % 32 = 16). Per case: per-stage HIP-event times with each stage's
algorithmic bytes and fraction of the 8 TB/s HBM peak (the dominant stage is `roofline`).
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
        # 12 MP frames (C5's size) with D <= 256: where the fused vertical WTA and the packed row
        # WTA meet (ocv_vwta_on)
        ("12MP 4096x3000 D=128 MODE_SGBM block 5", 3000, 4096, pkg.MODE_OCV_SGBM5,
         dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)),
        ("12MP 4096x3000 D=256 MODE_HH block 5", 3000, 4096, pkg.MODE_OCV_HH8,
         dict(num_disparities=256, min_disparity=0, block_size=5, speckle_window_size=0)),
        # 128 < D <= 256 in the other shapes (the path lines' width for that range, ocv_lanes_per_line)
        ("12MP 4096x3000 D=256 MODE_SGBM block 5", 3000, 4096, pkg.MODE_OCV_SGBM5,
         dict(num_disparities=256, min_disparity=0, block_size=5, speckle_window_size=0)),
        ("1920x1080 D=256 MODE_SGBM block 5", 1080, 1920, pkg.MODE_OCV_SGBM5,
         dict(num_disparities=256, min_disparity=0, block_size=5, speckle_window_size=0)),
        ("1920x1080 D=256 MODE_HH block 5", 1080, 1920, pkg.MODE_OCV_HH8,
         dict(num_disparities=256, min_disparity=0, block_size=5, speckle_window_size=0)),
    ]
    ref_kw = dict(min_disparity=147, num_disparities=480, block_size=21, uniqueness_ratio=2, speckle_window_size=1000,
                  speckle_range=4, prefilter_cap=7, p1=200, p2=400)
    for gate in ("1", "0"):
        for mname, mode in (("MODE_SGBM", pkg.MODE_OCV_SGBM5), ("MODE_HH", pkg.MODE_OCV_HH8)):
            tag = "gated" if gate == "1" else "int32 volumes"
            cases.append((f"refcfg 2448x2048 minD 147 D 480 block 21 {mname} ({tag})", 2048, 2448, mode,
                          dict(ref_kw, _gate=gate)))
    for mname, mode in (("MODE_SGBM", pkg.MODE_OCV_SGBM5), ("MODE_HH", pkg.MODE_OCV_HH8)):
        cases.append((f"proccfg 2448x2048 minD 0 D 752 block 21 {mname}", 2048, 2448, mode,
                      dict(ref_kw, min_disparity=0, num_disparities=752)))
    # 12 MP at D = 480: 10.4 GB int16 volumes, 64-lane lines of 8 values past the 32-bit buffer range
    # (the rebased packed path kernel, REBK)
    cases.append(("12MP 4096x3000 D=480 MODE_SGBM block 5", 3000, 4096, pkg.MODE_OCV_SGBM5,
                  dict(num_disparities=480, min_disparity=0, block_size=5, speckle_window_size=0)))
    eng = pkg.Engine(0)
    st = torch.cuda.Stream()
    for name, h, w, mode, kw in cases:
        if a.case not in name:
            continue
        kw = dict(kw)
        os.environ["SGM_OCV_GATE"] = kw.pop("_gate", "1")
        p = pkg.default_params(mode, **kw)
        eng.set_params(p)
        left, right, _ = synth.stereo_pair(h, w, max(p.min_disparity, 0), p.num_disparities, seed=3)
        dl = torch.from_numpy(left).cuda()
        dr = torch.from_numpy(right).cuda()
        out = torch.empty((h, w), dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), w, h, w, out.data_ptr(), w, st.cuda_stream)
            for _ in range(3):           # warm-up (first launches of each kernel variant)
                run()
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                run()
            e1.record(st)
            st.synchronize()
            eng.set_profiling(True)          # per-stage HIP events, a separate pass
            for _ in range(a.reps):
                run()
            st.synchronize()
            stages = eng.stage_times()
            eng.set_profiling(False)
        ms = e0.elapsed_time(e1) / a.reps
        rec = {"case": name, "gpu_ms_per_frame": round(ms, 3), "gpu_pairs_per_s": round(1000.0 / ms, 1)}
        rec["stages"] = [{"name": n, "avg_ms": round(t, 4), "alg_bytes": b, "GBps": round(b / (t * 1e-3) / 1e9, 1),
                          "frac": round(b / (t * 1e-3) / 8e12, 3)} for n, t, b in stages]
        if stages:
            dom = max(stages, key=lambda s_: s_[1])
            rec["roofline"] = {"bound": "hbm", "kernel": dom[0], "achieved": round(dom[2] / (dom[1] * 1e-3) / 1e9, 1),
                               "peak": 8000.0, "unit": "GB/s", "frac": round(dom[2] / (dom[1] * 1e-3) / 8e12, 4),
                               "avg_launch_ms": round(dom[1], 4), "algorithmic_bytes_per_launch": dom[2]}
        if orc is not None and h * w <= 1920 * 1080:
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
