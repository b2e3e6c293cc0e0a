"""OCV-mode batch throughput: sgm_match_device_batch of N frames with 1..4 stream lanes.

    python tools/ocv_batch_bench.py            # C1, 1080p MODE_SGBM / MODE_HH, lanes 1..4
    python tools/ocv_batch_bench.py --refcfg   # the shipped 2448x2048 D=480 block-21 config,
                                               # 4 lanes, extra lanes freed after each call
                                               # (default) or kept (SGM_OCV_KEEP_LANES=1),
                                               # back-to-back calls, interleaved rounds
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--refcfg", action="store_true")
ap.add_argument("--rounds", type=int, default=2)
a = ap.parse_args()
pkg = ge.load_package()
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))


def setup(mode, h, w, kw, n):
    p = pkg.default_params(mode, **kw)
    eng = pkg.Engine(0, p)
    fr = [synth.stereo_pair(h, w, max(p.min_disparity, 0), p.num_disparities, seed=i, with_truth=False)
          for i in range(min(n, 4))]
    dl = [torch.from_numpy(fr[i % len(fr)][0]).cuda() for i in range(n)]
    dr = [torch.from_numpy(fr[i % len(fr)][1]).cuda() for i in range(n)]
    outs = torch.empty((n, h, w), dtype=torch.int16, device="cuda")
    st = torch.cuda.Stream()
    args = ([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], w, h, w, [outs[i].data_ptr() for i in range(n)],
            w, st.cuda_stream)
    return eng, args, st, (dl, dr, outs)


def time_calls(eng, args, st, calls, n):
    eng.match_device_batch(*args)
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(calls):
        eng.match_device_batch(*args)
    e1.record(st)
    st.synchronize()
    return e0.elapsed_time(e1) / (calls * n)


if a.refcfg:
    n = 8
    kw = dict(min_disparity=147, num_disparities=480, block_size=21, uniqueness_ratio=2, speckle_window_size=1000,
              speckle_range=4, prefilter_cap=7, p1=200, p2=400)
    eng, args, st, keep_alive = setup(pkg.MODE_OCV_SGBM5, 2048, 2448, kw, n)
    os.environ["SGM_OCV_STREAMS"] = "4"
    for r in range(a.rounds):
        for keep in ("0", "1"):
            os.environ["SGM_OCV_KEEP_LANES"] = keep
            ms = time_calls(eng, args, st, 3, n)
            print(json.dumps({"case": "refcfg 2448x2048 minD 147 D 480 block 21 MODE_SGBM, batch of 8, 4 lanes",
                              "round": r, "lanes_kept": keep == "1", "ms_per_frame": round(ms, 3)}), flush=True)
    eng.close()
else:
    cases = [("C1", pkg.MODE_OCV_SGBM5, 480, 640, {}),
             ("1080p SGBM D128", pkg.MODE_OCV_SGBM5, 1080, 1920,
              dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0)),
             ("1080p HH D128", pkg.MODE_OCV_HH8, 1080, 1920,
              dict(num_disparities=128, min_disparity=0, block_size=5, speckle_window_size=0))]
    n = 12
    for name, mode, h, w, kw in cases:
        eng, args, st, keep_alive = setup(mode, h, w, kw, n)
        for lanes in ("1", "2", "3", "4"):
            os.environ["SGM_OCV_STREAMS"] = lanes
            print(f"{name:18s} lanes {lanes}: {time_calls(eng, args, st, 3, n):.3f} ms/frame", flush=True)
        eng.close()
