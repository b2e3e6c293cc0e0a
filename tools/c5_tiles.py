"""C5 (4096x3000, D=512, census 8-path + subpixel + LR) single-frame timings on the visible
devices: full frame on one device, row bands in overlap mode (halo 128) and in exact mode
(boundary-row exchange). Host buffers in and out (PCIe included in every figure), median of
`--reps` after one warm-up call. Prints one JSON line.

    python tools/c5_tiles.py [--bands 8] [--reps 3] [--devices 0,1,...]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--devices", default="")
    ap.add_argument("--height", type=int, default=3000)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--disparities", type=int, default=512)
    a = ap.parse_args()
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    h, w, D = a.height, a.width, a.disparities
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=5, with_truth=False)
    devs = [int(d) for d in a.devices.split(",")] if a.devices else list(range(pkg.device_count()))
    eng = pkg.Engine(devs[0], pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
    t_full, full = timed(lambda: eng.match(left, right), a.reps)
    t_ovl, ovl = timed(lambda: eng.match_tiled(left, right, a.bands, 128, devices=devs), a.reps)
    t_ex, ex = timed(lambda: eng.match_tiled_exact(left, right, a.bands, devices=devs), a.reps)
    print(json.dumps({
        "workload": f"C5: {w}x{h} D={D} census9x7 8-path + subpixel + LR, one frame",
        "devices": devs, "bands": a.bands,
        "ms_full_frame_1dev": round(t_full, 2),
        "ms_tiled_overlap_halo128": round(t_ovl, 2),
        "ms_tiled_exact": round(t_ex, 2),
        "overlap_disagreement_frac": float((ovl != full).mean()),
        "exact_disagreement_px": int((ex != full).sum()),
        "note": "host buffers in/out (PCIe included); bands dealt round-robin over the devices",
    }))
    eng.close()


if __name__ == "__main__":
    main()
