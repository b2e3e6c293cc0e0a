"""Latency of the host-buffer calls a ROS node makes, beside the
device-resident time of the same frame: per configuration
  * sgm_match (the C-ABI: host images in, int16 disparity out, synchronous), median of reps;
  * MatcherCore::forwardMatch through plugin_core_test (the AbstractStereoMatcher adapter's
    core: parameters set, sgm_match_f32 into the adapter's persistent, page-locked output),
    median of reps, and the same with an unregistered (pageable) output;
  * sgm_match_device on resident buffers (HIP events), for the PCIe + host-work share.
Prints one JSON line per configuration.

    python tools/host_calls.py [--reps 20]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    core = os.path.join(ge.PKG_DIR, "lib", "plugin_core_test")
    cases = [("C1 node defaults, MODE_SGBM 640x480 minD 9 D 64 block 15", pkg.MODE_OCV_SGBM5, 480, 640, 64, 9, 15),
             ("1920x1080 MODE_SGBM D 128 block 5 (node's other params)", pkg.MODE_OCV_SGBM5, 1080, 1920, 128, 0, 5),
             ("C3 census 1920x1080 D 256", pkg.MODE_CENSUS8, 1080, 1920, 256, 0, 5),
             ("C3 census 1920x1080 D 256, no speckle filter (BASELINE C3)", pkg.MODE_CENSUS8, 1080, 1920, 256, 0, 5)]
    for name, mode, h, w, D, minD, block in cases:
        spk = 0 if "no speckle" in name else 100
        left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=3, with_truth=False)
        # the adapter's parameter set (node defaults besides D / minD / block)
        p = pkg.default_params(mode, num_disparities=D, min_disparity=minD, block_size=block, uniqueness_ratio=15,
                               speckle_window_size=spk, speckle_range=4, prefilter_cap=31, p1=200, p2=400)
        eng = pkg.Engine(0, p)
        eng.match(left, right)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            eng.match(left, right)
            ts.append((time.perf_counter() - t0) * 1e3)
        dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
        out = torch.empty((h, w), dtype=torch.int16, device="cuda")
        st = torch.cuda.Stream()
        run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), w, h, w, out.data_ptr(), w, st.cuda_stream)
        run(); st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            run()
        e1.record(st); st.synchronize()
        eng.close()
        rec = {"case": name, "sgm_match_ms_median": round(statistics.median(ts), 3),
               "sgm_match_ms_min": round(min(ts), 3),
               "device_resident_ms": round(e0.elapsed_time(e1) / a.reps, 3)}
        with tempfile.TemporaryDirectory() as td:
            lf, rf = os.path.join(td, "l.raw"), os.path.join(td, "r.raw")
            left.tofile(lf); right.tofile(rf)
            for reg, key in ((1, "forwardMatch"), (0, "forwardMatch_pageable")):
                r = subprocess.run([core, "time", lf, rf, str(w), str(h), str(mode), str(D), str(minD), str(block),
                                    str(a.reps), str(spk), str(reg)], capture_output=True, text=True, timeout=300)
                if r.returncode == 0:
                    c = json.loads(r.stdout.strip().splitlines()[-1])
                    rec[key + "_ms_median"] = c["ms_median"]
                    rec[key + "_ms_min"] = c["ms_min"]
                else:
                    rec[key + "_error"] = r.stderr[-300:]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
