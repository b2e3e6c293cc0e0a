"""DESIGN §8.2 prototype A/B (VERDICT r4 "do this" #2): the shared-cost top-down strip sweep
(k_strip3_proto, timing-only, experiment build) against the same three directions of the
production paths kernel, on one 1920x1080 frame's census codes (C2 D=128, C3 D=256).

    bash tools/build_variant.sh strip3 "-DSGM_EXPERIMENT_BUILD" "census_sgm.hip sgm_api.cpp"
    SGM_HIP_LIB=i3dr_stereo_camera-ros_amd/lib/variants/strip3/libsgm_hip.so python tools/strip3_ab.py

One JSON line per (config, strip shape, round): ms of the three top-down directions in the
production kernel (three u8 volumes), of the prototype (one u16 partial-sum volume), and of the
whole eight-direction single-frame paths launch for scale.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shapes", default="32:8,48:8,48:4,64:8,64:16", help="ncol:G pairs (strip = ncol - 2G)")
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    lib = pkg.load_library()
    if not hasattr(lib, "sgm_exp_strip3"):
        sys.exit("needs the experiment build (SGM_HIP_LIB=.../variants/strip3/libsgm_hip.so)")
    lib.sgm_exp_strip3.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    W, H = 1920, 1080
    for cfg, D, sub in (("C2", 128, 0), ("C3", 256, 1)):
        left, right, _ = synth.stereo_pair(H, W, 0, D, seed=3, with_truth=False)
        p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=0, p1=10, p2=120,
                               uniqueness_ratio=5, subpixel=sub, lr_check=sub, median=0, speckle_window_size=0)
        eng = pkg.Engine(0, p)
        dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
        torch.cuda.synchronize()
        for rnd in range(a.rounds):
            for shape in a.shapes.split(","):
                ncol, G = (int(v) for v in shape.split(":"))
                ms = (ctypes.c_float * 3)()
                rc = lib.sgm_exp_strip3(eng.h, dl.data_ptr(), dr.data_ptr(), W, H, ncol, G, a.reps, ms)
                rec = {"config": cfg, "D": D, "round": rnd, "ncol": ncol, "G": G, "strip_cols": ncol - 2 * G, "rc": rc,
                       "down3_paths16_ms": round(ms[0], 4), "strip3_proto_ms": round(ms[1], 4),
                       "all8_paths16_ms": round(ms[2], 4)}
                if rc == 0 and ms[0] > 0:
                    rec["proto_vs_down3"] = round(ms[1] / ms[0], 3)
                print(json.dumps(rec), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
