"""Single-frame latency of the census engine (BASELINE configs[1] is one 1920x1080 D=128 frame;
the node matches one frame per callback, generate_disparity.cpp:334-368): sgm_match_device on
resident buffers, each call alone (stream synchronised before the next: what one callback
sees), and back to back (HIP events over the reps). One JSON line per config.

    python tools/single_frame.py [--reps 30] [--configs c2,c3]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

CFG = {"c2": (1920, 1080, 128, 0, 0), "c3": (1920, 1080, 256, 1, 1), "c5": (4096, 3000, 512, 1, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--configs", default="c2,c3")
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    for name in a.configs.split(","):
        W, H, D, sub, lr = CFG[name]
        p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, subpixel=sub, lr_check=lr, median=0)
        eng = pkg.Engine(0, p)
        l, r, _ = synth.stereo_pair(H, W, 0, D, seed=5, with_truth=False)
        dl, dr = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
        out = torch.empty((H, W), dtype=torch.int16, device="cuda")
        st = torch.cuda.Stream()
        run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, st.cuda_stream)
        run(); run(); st.synchronize()
        eng.set_profiling(True)
        for _ in range(5):
            run()
        stages = {n: round(ms, 4) for n, ms, _ in eng.stage_times()}
        eng.set_profiling(False)
        alone = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            run()
            st.synchronize()
            alone.append((time.perf_counter() - t0) * 1e3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            run()
        e1.record(st)
        st.synchronize()
        eng.close()
        print(json.dumps({"config": name, "W": W, "H": H, "D": D,
                          "alone_ms_median": round(statistics.median(alone), 4), "alone_ms_min": round(min(alone), 4),
                          "back_to_back_ms": round(e0.elapsed_time(e1) / a.reps, 4),
                          "stages_ms": stages}), flush=True)


if __name__ == "__main__":
    main()
