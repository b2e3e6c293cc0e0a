"""Interleaved A/B of the node's host-buffer calls across library builds:
per round and per build, `sgm_match` (Python ctypes, host images in, int16 out) and
MatcherCore::forwardMatch through plugin_core_test (sgm_match_f32 into the adapter's
registered output, and into a pageable one) on the C3 census frame without post filters and
on the 1080p MODE_SGBM frame, beside the device-resident time of the same build. One JSON
line per (round, build, case).

    python tools/host_ab.py [--rounds 3] [--reps 30] NAME=path/to/libsgm_hip.so ...

Each build runs in child processes (own HIP context): the Python calls load it through
SGM_HIP_LIB, plugin_core_test through LD_LIBRARY_PATH (its RUNPATH is $ORIGIN).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

CASES = [("C3 census 1920x1080 D 256, no post filters", 2, 256, 0, 5, 0),
         ("1920x1080 MODE_SGBM D 128 block 5, speckle 100", 0, 128, 0, 5, 100)]

CHILD = r"""
import json, statistics, sys, time, numpy as np, torch
sys.path.insert(0, {root!r})
import __graft_entry__ as ge
pkg = ge.load_package()
left = np.fromfile({lf!r}, np.uint8).reshape({h}, {w}); right = np.fromfile({rf!r}, np.uint8).reshape({h}, {w})
p = pkg.default_params({mode}, num_disparities={D}, min_disparity={minD}, block_size={block}, uniqueness_ratio=15,
                       speckle_window_size={spk}, speckle_range=4, prefilter_cap=31, p1=200, p2=400)
eng = pkg.Engine(0, p)
eng.match(left, right)
ts = []
for _ in range({reps}):
    t0 = time.perf_counter(); eng.match(left, right); ts.append((time.perf_counter() - t0) * 1e3)
dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
out = torch.empty(({h}, {w}), dtype=torch.int16, device="cuda")
st = torch.cuda.Stream()
run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), {w}, {h}, {w}, out.data_ptr(), {w}, st.cuda_stream)
run(); st.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range({reps}):
    run()
e1.record(st); st.synchronize()
print(json.dumps({{"sgm_match_ms_median": round(statistics.median(ts), 4), "device_resident_ms": round(e0.elapsed_time(e1) / {reps}, 4)}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("builds", nargs="+", help="NAME=path/to/libsgm_hip.so")
    a = ap.parse_args()
    builds = [b.split("=", 1) for b in a.builds]
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    core = os.path.join(ge.PKG_DIR, "lib", "plugin_core_test")
    h, w = 1080, 1920
    with tempfile.TemporaryDirectory() as td:
        frames = {}
        for D in sorted({c[2] for c in CASES}):
            left, right, _ = synth.stereo_pair(h, w, 0, D, seed=3, with_truth=False)
            lf, rf = os.path.join(td, f"l{D}.raw"), os.path.join(td, f"r{D}.raw")
            left.tofile(lf)
            right.tofile(rf)
            frames[D] = (lf, rf)
        for rnd in range(a.rounds):
            for name, lib in builds:
                lib = os.path.abspath(lib)
                env = dict(os.environ, SGM_HIP_LIB=lib,
                           LD_LIBRARY_PATH=os.path.dirname(lib) + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
                for case, mode, D, minD, block, spk in CASES:
                    lf, rf = frames[D]
                    rec = {"round": rnd, "build": name, "case": case}
                    code = CHILD.format(root=ROOT, lf=lf, rf=rf, h=h, w=w, mode=mode, D=D, minD=minD, block=block,
                                        spk=spk, reps=a.reps)
                    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                                       env=env)
                    if r.returncode == 0:
                        rec.update(json.loads(r.stdout.strip().splitlines()[-1]))
                    else:
                        rec["error"] = r.stderr[-300:]
                    for reg, key in ((1, "forwardMatch"), (0, "forwardMatch_pageable")):
                        r = subprocess.run([core, "time", lf, rf, str(w), str(h), str(mode), str(D), str(minD),
                                            str(block), str(a.reps), str(spk), str(reg)], capture_output=True,
                                           text=True, timeout=300, env=env)
                        if r.returncode == 0:
                            rec[key + "_ms_median"] = json.loads(r.stdout.strip().splitlines()[-1])["ms_median"]
                        else:
                            rec[key + "_error"] = r.stderr[-300:]
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
