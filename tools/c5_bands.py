"""C5 (4096x3000, D=512 census 8-path + subpixel + LR, one frame) on paper for 8 GPUs from
1-GPU measurements:

  * full frame, device-resident (sgm_match_device, per-stage HIP events) and a pipelined
    batch of C5 frames (the throughput form);
  * overlap mode: one band of 375 + 2 x 128 halo rows alone, device-resident;
  * exact mode: every band step alone (SGM_TILE_TIMES: each launch synchronised before and
    after, its device time recorded), 8 bands on this one device;

then the critical path of each mode on 8 GPUs (one band per GPU) from those durations, with
the boundary-row exchange priced at an assumed xGMI rate (--xgmi-gbs, one link, one
direction). Prints one JSON line.

    python tools/c5_bands.py [--bands 8] [--halo 128] [--xgmi-gbs 50]
"""
import argparse
import collections
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def device_frame(pkg, torch, eng, left, right, reps=5):
    """ms per frame and per-stage ms of sgm_match_device on resident buffers."""
    h, w = left.shape
    dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
    out = torch.empty((h, w), dtype=torch.int16, device="cuda")
    st = torch.cuda.Stream()
    run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), w, h, w, out.data_ptr(), w, st.cuda_stream)
    run(); st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        run()
    e1.record(st); st.synchronize()
    eng.set_profiling(True)
    for _ in range(reps):
        run()
    st.synchronize()
    stages = {n: round(t, 4) for n, t, _ in eng.stage_times()}
    eng.set_profiling(False)
    return round(e0.elapsed_time(e1) / reps, 3), stages, out.cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--halo", type=int, default=128)
    ap.add_argument("--xgmi-gbs", type=float, default=50.0)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    H, W, D, nb = 3000, 4096, 512, a.bands
    left, right, _ = synth.stereo_pair(H, W, 0, D, seed=5, with_truth=False)
    p = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D)
    eng = pkg.Engine(0, p)
    res = {"workload": f"C5: {W}x{H} D={D} census9x7 8-path + subpixel + LR, one frame", "bands": nb}
    full_ms, full_st, full = device_frame(pkg, torch, eng, left, right)
    res["full_frame_1gpu"] = {"ms": full_ms, "stages": full_st, "device_resident": True}
    # pipelined batch of C5 frames (throughput form)
    dl = [torch.from_numpy(left).cuda() for _ in range(a.batch)]
    dr = [torch.from_numpy(right).cuda() for _ in range(a.batch)]
    outs = torch.empty((a.batch, H, W), dtype=torch.int16, device="cuda")
    st = torch.cuda.Stream()
    args = ([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], W, H, W, [outs[i].data_ptr() for i in range(a.batch)],
            W, st.cuda_stream)
    eng.match_device_batch(*args); st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); eng.match_device_batch(*args); e1.record(st); st.synchronize()
    res["batch_1gpu"] = {"frames": a.batch, "ms_per_frame": round(e0.elapsed_time(e1) / a.batch, 3),
                         "bit_exact_vs_single": bool(np.array_equal(outs[0].cpu().numpy(), full))}
    # overlap mode: an interior band with its halos, alone
    hb = H // nb + 2 * a.halo
    ov_ms, ov_st, _ = device_frame(pkg, torch, eng, np.ascontiguousarray(left[:hb]), np.ascontiguousarray(right[:hb]))
    res["overlap_band_1gpu"] = {"rows": hb, "ms": ov_ms, "stages": ov_st}
    # exact mode: each band step alone
    tf = tempfile.NamedTemporaryFile(delete=False, suffix=".txt").name
    os.environ["SGM_TILE_TIMES"] = tf
    ex = eng.match_tiled_exact(left, right, nb, devices=[0])
    del os.environ["SGM_TILE_TIMES"]
    res["exact_equals_full"] = bool(np.array_equal(ex, full))
    t = collections.defaultdict(dict)
    for line in open(tf):
        b, kind, ms = line.split()
        t[kind][int(b)] = float(ms)
    os.unlink(tf)
    res["exact_band_steps_ms"] = {k: {str(b): round(v, 4) for b, v in sorted(d.items())} for k, d in t.items()}
    # 8-GPU critical paths (one band per GPU; the primary gathers, filters, copies out)
    width1 = W - D + 1
    seam_bytes = 3 * width1 * D                   # three directions' boundary rows per seam
    xgmi_ms = seam_bytes / (a.xgmi_gbs * 1e9) * 1e3
    band_rows = H // nb
    gather_ms = W * band_rows * 2 / (a.xgmi_gbs * 1e9) * 1e3
    pre = max(t["h2d"][b] + t["census"][b] for b in range(nb))
    down_end, up_end = {}, {}
    tcur = pre
    for b in range(nb):                      # horizontal scans precede the down sweep on a band's stream
        tcur = max(tcur, pre + t["horiz"][b]) + t["down"][b]
        down_end[b] = tcur
        tcur += xgmi_ms if b + 1 < nb else 0.0
    tcur = pre
    for b in reversed(range(nb)):
        tcur += t["up"][b]
        up_end[b] = tcur
        tcur += xgmi_ms if b > 0 else 0.0
    finish = max(max(down_end[b], up_end[b]) + t["wta"][b] for b in range(nb)) + gather_ms + t["post"][-1]
    res["exact_8gpu_model_ms"] = {"critical_path_ms": round(finish, 3), "xgmi_seam_ms": round(xgmi_ms, 4),
                                  "down_chain_ms": round(down_end[nb - 1] - pre, 3),
                                  "up_chain_ms": round(up_end[0] - pre, 3),
                                  "note": "device time only (host staging excluded); bands' own steps alone"}
    ov = ov_ms + gather_ms + t["post"][-1]
    res["overlap_8gpu_model_ms"] = {"critical_path_ms": round(ov, 3),
                                    "note": "one band + halos per GPU, independent; device time only"}
    res["full_frame_1gpu_ms"] = full_ms
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
