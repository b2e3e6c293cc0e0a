"""Benchmark of the MI355X-native SGM hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--config c3|c2|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` alone (no WORLD_SIZE in the environment) starts the N rank processes itself, before
this process makes any GPU call (one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 set for each), and exits with the first failing rank's code; it exits
non-zero if fewer than N devices are visible. Under torchrun the ranks come from the
environment and WORLD_SIZE must equal --gpus. `--dry-run` runs the same rank logic with gloo
and no HIP (a stand-in sleep per frame) for the CPU tests.

Workload (BASELINE.json configs[2], the config the metric is quoted on): 1920x1080 stereo
pairs, D = 256, 9x7 census + Hamming cost, 8-path SGM, WTA + uniqueness + subpixel +
LR check (`--config c2`: D = 128, no subpixel / LR). A step = one pass of the hot path over
F synthetic frames per rank, inputs resident in HBM before timing. Frames are independent,
so each rank owns its own frames (frame shard, weak scaling, no data-path collective); the
only collectives are the timing barrier and the max-over-ranks reduction.

`roofline` is the dominant kernel (algorithmic bytes / its average HIP-event duration over
the timed region); `pipeline` is the whole frame (SURVEY §8d B_alg / per-frame device
time). `cpu_baseline` times the CPU port (oracle) on a bounded sample on rank 0 at N = 1.

C5 (BASELINE configs[4], 4096x3000 D=512, one frame): `--config c5` times it on its own — at
N = 1 the single-device full frame (sgm_match_device), at N > 1 the overlap tile mode
(sgm_match_tiled_device: N row bands + 128-row halos, one band per GPU, rows moved over xGMI)
driven by one process (rank 0 under torchrun, the other ranks wait at a barrier) — and reports
the disagreement with the 1-GPU full frame. The default C3 run adds the same measurement as
its `c5` block (a child process after the C3 timed region, while the other ranks wait).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), GB/s
METRIC = "stereo pairs/sec + ms/frame, 1920×1080 D=256 8-path SGM, 1/2/4/8 MI355X"

CONFIGS = {
    "c3": dict(name="C3: 1920x1080 D=256 census9x7 8-path SGM + subpixel + LR-check", w=1920, h=1080, D=256,
               subpixel=1, lr_check=1),
    "c2": dict(name="C2: 1920x1080 D=128 census9x7 8-path SGM (no subpixel / LR)", w=1920, h=1080, D=128,
               subpixel=0, lr_check=0),
    "c5": dict(name="C5: 4096x3000 D=512 census9x7 8-path SGM + subpixel + LR-check, one frame (N > 1: row-band "
                    "overlap tiles, one band per GPU, 128-row halos)", w=4096, h=3000, D=512, subpixel=1, lr_check=1),
}
C5_HALO = 128           # overlap mode, 0 disagreement at C5 with 128-row halos
RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
            "TORCHELASTIC_MAX_RESTARTS", "GROUP_WORLD_SIZE")


def shard_frames(n_frames_per_rank, rank, seed0=0):
    """Frame ids owned by `rank` (distinct synthetic frames per rank)."""
    return [seed0 + rank * n_frames_per_rank + i for i in range(n_frames_per_rank)]


def max_over_ranks(x, device=None):
    """MAX of a float over all ranks (the timing reduction; RCCL on GPUs, gloo in tests)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def algorithmic_bytes(w, h, D, width1=None):
    """SURVEY §8d B_alg per stereo pair: W*H*(2 + 16*D + 2) — images in, 8 u8 path volumes
    written + read once (16 B/cell), int16 disparity out. With `width1` the same dataflow
    over the cells the engine actually aggregates (x >= minX1, OpenCV's width1 = W - D + 1
    columns), the conservative basis reported beside the graded one."""
    return 4.0 * w * h + 16.0 * (w if width1 is None else width1) * h * D


def load_pmc_traffic(config):
    """HBM bytes per launch from the committed PMC profile (profiles/latest_pmc_<config>.json,
    written by tools/refresh_profiles.sh with the source revision it profiled), if any."""
    path = os.path.join(ROOT, "profiles", f"latest_pmc_{config}.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path))
    except Exception:
        return None


def hbm_copy_gbps(device, nbytes=2 << 30, reps=5):
    """Achievable HBM copy bandwidth on this GPU (reported beside the 8 TB/s
    spec peak): a device-to-device copy of `nbytes`, read + write bytes counted."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return round(gbps, 1)


def cpu_baseline(cfg, budget_s=20.0):
    """Times the CPU port of the same workload (oracle, multi-threaded C) on host cores."""
    import numpy as np
    import importlib.util
    spec = importlib.util.spec_from_file_location("sgm_oracle", os.path.join(ROOT, "oracle", "sgm_oracle.py"))
    orc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(orc)
    import __graft_entry__ as ge
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    left, right, _ = synth.stereo_pair(cfg["h"], cfg["w"], 0, cfg["D"], seed=12345, with_truth=False)
    p = orc.make_params(orc.MODE_CENSUS8, num_disparities=cfg["D"], subpixel=cfg["subpixel"],
                        lr_check=cfg["lr_check"])
    # cores: the CPUs this process may run on (affinity) and the cgroup quota, against the
    # threads the port actually uses (OMP_NUM_THREADS: the GPU box's per-GPU CPU share is 16)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or affinity
    threads = max(1, min(threads, affinity, int(quota) if quota else affinity))
    orc.set_threads(threads)
    threads = orc.num_threads()
    cpu_model = ""
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    n, t0 = 0, time.perf_counter()
    while True:
        orc.match(p, left, right)
        n += 1
        if time.perf_counter() - t0 > budget_s / 2 or n >= 8:
            break
    dt = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "pairs/s", "cores": threads, "kind": "port", "cpu_model": cpu_model,
           "host_cpus_visible": os.cpu_count(), "host_cpus_affinity": affinity, "cgroup_cpu_quota": quota,
           "threads_used": threads,
           "sample": f"{n} full {cfg['w']}x{cfg['h']} D={cfg['D']} frames of the same census-SGM workload, "
                     f"oracle/sgm_oracle.c (OpenMP over lines, {threads} threads)"}
    # the reference's own CPU path: OpenCV-SGBM restatement, single thread, same geometry
    pr = orc.make_params(orc.MODE_OCV_SGBM5, min_disparity=0, num_disparities=cfg["D"], block_size=5,
                         speckle_window_size=0)
    orc.set_threads(1)
    t0 = time.perf_counter()
    orc.match(pr, left, right)
    dt1 = time.perf_counter() - t0
    orc.set_threads(threads)
    out["reference_path"] = {"value": 1.0 / dt1, "unit": "pairs/s", "cores": 1, "kind": "port",
                             "sample": f"1 frame {cfg['w']}x{cfg['h']} D={cfg['D']} OpenCV-StereoSGBM "
                                       f"MODE_SGBM restatement (block 5), single-threaded like OpenCV"}
    # the 8-path MODE_HH restatement at 1920x1080 D=128, single thread
    ph = orc.make_params(orc.MODE_OCV_HH8, min_disparity=0, num_disparities=128, block_size=5,
                         speckle_window_size=0)
    orc.set_threads(1)
    t0 = time.perf_counter()
    orc.match(ph, left, right)
    dth = time.perf_counter() - t0
    out["reference_path_hh"] = {"value": 1.0 / dth, "unit": "pairs/s", "cores": 1, "kind": "port",
                                "ms_per_frame": round(dth * 1e3, 1),
                                "sample": f"1 frame {cfg['w']}x{cfg['h']} D=128 OpenCV-StereoSGBM MODE_HH "
                                          f"restatement (block 5), single-threaded"}
    out["c1_reference_matcher"] = c1_reference_matcher(orc, synth)
    orc.set_threads(threads)
    return out


def c1_reference_matcher(orc, synth, reps=20):
    """BASELINE configs[0] (C1): the reference's own matcher at the generate_disparity node
    defaults (640x480, minD 9, D 64, block 15, MODE_SGBM + medianBlur + filterSpeckles),
    single-threaded CPU restatement beside the engine's bit-exact GPU restatement of it on the
    same frame (device buffers, HIP events on the engine's stream). Reported beside the
    census metric, never as `value`."""
    import numpy as np
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    left, right, _ = synth.stereo_pair(480, 640, 9, 64, seed=1, with_truth=False)
    p = pkg.default_params(pkg.MODE_OCV_SGBM5)
    eng = pkg.Engine(torch.cuda.current_device(), p)
    dl, dr = torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda()
    out = torch.empty((480, 640), dtype=torch.int16, device="cuda")
    st = torch.cuda.Stream()
    run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), 640, 480, 640, out.data_ptr(), 640, st.cuda_stream)
    run()
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        run()
    e1.record(st)
    st.synchronize()
    gpu_ms = e0.elapsed_time(e1) / reps
    got = out.cpu().numpy()
    eng.close()
    op = orc.make_params(orc.MODE_OCV_SGBM5, **{k: v for k, v in p.as_dict().items() if k != "mode"})
    orc.set_threads(1)
    t0 = time.perf_counter()
    ref = orc.match(op, left, right)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    return {"config": "C1 640x480 minD 9 D 64 block 15 MODE_SGBM + median + speckle (node defaults)",
            "cpu_ms_per_frame": round(cpu_ms, 2), "cpu_cores": 1, "kind": "port",
            "gpu_ms_per_frame": round(gpu_ms, 4), "gpu_pairs_per_s": round(1000.0 / gpu_ms, 1),
            "bit_exact": bool(np.array_equal(got, ref))}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_devices():
    """HIP devices this process may use; torch.cuda.device_count() does not initialise the GPU
    on this image, so it is safe before the rank processes are started."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(n, argv, dry_run=False):
    """`bench.py --gpus N` without WORLD_SIZE: one child process per rank (this process never
    touches the GPU), the torchrun environment set for each. Returns the exit code: 0 if every
    rank succeeded, else the first failing rank's code (the others are terminated)."""
    if not dry_run:
        vis = visible_devices()
        if vis < (1 if "--share-device" in argv else n):
            print(f"bench.py: --gpus {n} but only {vis} HIP device(s) visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = {k: v for k, v in os.environ.items() if k not in RANK_ENV}
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.remove(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    return rc


def dry_step(rank, n_frames):
    """--dry-run stand-in for one step of a rank (no HIP): rank r takes (1 + r) ms per frame,
    so the ranks finish at different times and the MAX reduction is visible."""
    time.sleep(1e-3 * (1 + rank) * n_frames)


def c5_frame_ms(pkg, torch, eng, dl, dr, out, W, H, devices, steps, warmup, stream, tstream):
    """ms per C5 frame over `steps` timed frames: the full frame on one device, or the overlap
    tile mode over `devices` (one band each), inputs resident in HBM of the engine's device."""
    if len(devices) == 1:
        run = lambda: eng.match_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, stream)
    else:
        run = lambda: eng.match_tiled_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, len(devices),
                                             C5_HALO, devices=devices, stream=stream)
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    tstream.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def run_c5(args, n_gpus, pkg, torch, device):
    """C5 on one process driving devices 0..n_gpus-1 (see the module docstring)."""
    cfg = CONFIGS["c5"]
    W, H, D = cfg["w"], cfg["h"], cfg["D"]
    synth = __import__("__graft_entry__")._load_file("sgm_synth", os.path.join(ROOT, "i3dr_stereo_camera-ros_amd",
                                                                                "synth.py"))
    left, right, _ = synth.stereo_pair(H, W, 0, D, seed=5, with_truth=False)
    params = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=0, p1=10, p2=120,
                                uniqueness_ratio=5, subpixel=1, lr_check=1, disp12_max_diff=1, median=0,
                                speckle_window_size=0)
    eng = pkg.Engine(device, params)
    dl, dr = torch.from_numpy(left).to(device), torch.from_numpy(right).to(device)
    out = torch.empty((H, W), dtype=torch.int16, device=device)
    tstream = torch.cuda.Stream(device)
    stream = tstream.cuda_stream
    devices = list(range(n_gpus))
    ms = c5_frame_ms(pkg, torch, eng, dl, dr, out, W, H, devices, args.steps, args.warmup, stream, tstream)
    res = {"workload": cfg["name"], "width": W, "height": H, "num_disparities": D, "n_gpus": n_gpus,
           "ms_per_frame": round(ms, 4), "pairs_per_s": round(1000.0 / ms, 3), "frames_timed": args.steps,
           "mode": "full frame, sgm_match_device" if n_gpus == 1 else
                   f"overlap tiles: {n_gpus} row bands + {C5_HALO}-row halos, sgm_match_tiled_device "
                   f"(one band per GPU, host thread + stream per device, rows over xGMI)"}
    b_alg = algorithmic_bytes(W, H, D)
    res["roofline"] = {"bound": "hbm", "B_alg_per_frame": b_alg, "achieved": round(b_alg / (ms * 1e-3) / 1e9, 1),
                       "peak": HBM_PEAK_GBS * n_gpus, "unit": "GB/s",
                       "frac": round(b_alg / (ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * n_gpus), 4),
                       "basis": "SURVEY 8d B_alg of one C5 frame over the frame time, against N x 8 TB/s"}
    if n_gpus == 1:
        eng.set_profiling(True)
        eng.match_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, stream)
        tstream.synchronize()
        res["stages"] = {n: round(t, 4) for n, t, _ in eng.stage_times()}
        eng.set_profiling(False)
        res["disagreement_vs_full_frame"] = 0.0
    else:
        tiled = out.cpu().numpy()
        eng.match_device(dl.data_ptr(), dr.data_ptr(), W, H, W, out.data_ptr(), W, stream)
        tstream.synchronize()
        full = out.cpu().numpy()
        res["disagreement_vs_full_frame"] = float((tiled != full).mean())
    eng.close()
    return res


def c5_leg(args, world):
    """The default run's `c5` block: bench.py --config c5 in a child process (own HIP context,
    a fault there cannot take the C3 line with it), over the same number of GPUs."""
    env = {k: v for k, v in os.environ.items() if k not in RANK_ENV}
    cmd = [sys.executable, os.path.abspath(__file__), "--config", "c5", "--gpus", str(world), "--steps",
           str(args.c5_frames), "--warmup", "1", "--no-cpu-baseline", "--c5-only"]
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.c5_timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {args.c5_timeout} s"}
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}: {p.stderr.strip()[-400:]}"}
    return json.loads(lines[-1])


def device_identity(device=None, local_rank=0):
    """Which physical device a rank ran on: HIP ordinal, PCI domain:bus:device and UUID (torch's
    device properties), so an N-rank line shows N distinct GPUs. `device=None` (dry run, no HIP)
    reports the rank's local ordinal only."""
    if device is None:
        return {"ordinal": local_rank, "pci": None, "uuid": None, "name": "dry run (no HIP)"}
    import torch
    pr = torch.cuda.get_device_properties(device)
    pci = None
    if hasattr(pr, "pci_bus_id"):
        pci = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    uuid = str(getattr(pr, "uuid", "")) or None
    return {"ordinal": int(device), "pci": pci, "uuid": uuid, "name": pr.name,
            "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))}


def distinct_devices(shard):
    """Number of distinct physical devices in a shard record (PCI address + UUID; the ordinal
    when neither is known)."""
    keys = set()
    for r in shard:
        d = r.get("device") or {}
        keys.add((d.get("pci"), d.get("uuid")) if (d.get("pci") or d.get("uuid")) else ("ordinal", d.get("ordinal")))
    return len(keys)


def gather_shard(seeds, elapsed, distributed, busy=None, device=None, group=None):
    """Per-rank record of the frame shard: the synthetic frame seeds each rank owned, its own
    timed-region length (the line's value uses the MAX of these), the device it ran on and the
    world size it saw. Gathered over `group` (the CPU-side gloo group: no RCCL kernel)."""
    mine = {"seeds": list(seeds), "elapsed_s": round(elapsed, 6), "device": device}
    if busy is not None:
        mine["busy_s"] = round(busy, 6)
    if not distributed:
        mine["world_size"] = 1
        return [mine]
    import torch.distributed as dist
    mine["world_size"] = dist.get_world_size()
    mine["rank"] = dist.get_rank()
    objs = [None] * dist.get_world_size()
    dist.all_gather_object(objs, mine, group=group)
    return objs


def dry_main(args, world, rank):
    """--dry-run: the rank / shard / timing logic of main() with gloo and no HIP."""
    import torch.distributed as dist
    distributed = world > 1
    if distributed:
        dist.init_process_group("gloo")
    ids = shard_frames(args.distinct, rank)
    for _ in range(args.warmup):
        dry_step(rank, 1)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dry_step(rank, 1)
    busy = time.perf_counter() - t0        # this rank's own work, before the closing barrier
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = max_over_ranks(elapsed)
    shard = gather_shard(ids, elapsed, distributed, busy, device_identity(None, rank))
    if rank == 0:
        frames_total = args.frames * args.steps * world
        print(json.dumps({"metric": METRIC, "value": round(frames_total / elapsed_max, 3), "unit": "pairs/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed_max * 1e3 / args.steps, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "dry run (no HIP work)",
                          "elapsed_max_s": elapsed_max, "shard": shard, "distinct_devices": distinct_devices(shard),
                          "config": {"workload": "dry run", "parallelism": f"frame-shard x{world}"}}))
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=64, help="frames per rank per step (BASELINE C4: batch 64)")
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic pairs per rank")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one sgm_match_device call per frame")
    ap.add_argument("--rectify", action="store_true",
                    help="raw frames in: rectification (maps of a synthetic calibration) fused into the census")
    ap.add_argument("--host-io", action="store_true",
                    help="host buffers in and out (sgm_match_batch: pinned rings, H2D/D2H overlapped with the "
                         "kernels); PCIe-inclusive, reported beside the device-resident value, never as it")
    ap.add_argument("--dry-run", action="store_true", help="rank logic only: gloo, no HIP (CPU tests)")
    ap.add_argument("--no-c5", action="store_true", help="skip the default run's C5 block")
    ap.add_argument("--c5-frames", type=int, default=10, help="timed C5 frames of the default run's c5 block")
    ap.add_argument("--c5-timeout", type=int, default=300)
    ap.add_argument("--c5-only", action="store_true", help=argparse.SUPPRESS)
    # test-only: every rank on device 0 over gloo (RCCL cannot put two ranks on one GPU), so the
    # N > 1 path (launcher -> ranks -> HIP engine -> MAX -> one line) runs on a one-GPU box
    ap.add_argument("--share-device", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    # --gpus N without a torchrun environment: start the N ranks here, before any GPU call
    # (C5 is one process driving every device, so it needs no rank processes)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.config != "c5":
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dry_run))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: n_gpus must equal --gpus", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        return dry_main(args, world, rank)
    cfg = CONFIGS[args.config]

    import numpy as np
    import torch
    import torch.distributed as dist
    import __graft_entry__ as ge

    distributed = world > 1
    n_vis = torch.cuda.device_count()
    need = 1 if args.share_device else max(world, args.gpus if args.config == "c5" else 1)
    if args.share_device:
        local_rank = 0
    if n_vis < need or local_rank >= n_vis:
        print(f"bench.py: needs {need} HIP device(s) (rank {rank}, local rank {local_rank}), {n_vis} visible",
              file=sys.stderr)
        sys.exit(2)
    if distributed:
        torch.cuda.set_device(local_rank)
        if args.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        # waits outside the timed region (while rank 0 alone runs the single-frame / C5 / CPU legs,
        # which drive every device) and the shard gather go over a CPU-side gloo group: a waiting
        # rank then holds no spinning RCCL kernel on its device
        wait_group = dist.new_group(backend="gloo")
    else:
        torch.cuda.set_device(0)
        wait_group = None
    device = torch.cuda.current_device()
    pkg = ge.load_package()

    if args.config == "c5":
        c5 = None
        if rank == 0:
            c5 = run_c5(args, max(world, args.gpus), pkg, torch, device)
        if distributed:
            dist.barrier(group=wait_group)
        if rank == 0:
            if args.c5_only:
                print(json.dumps(c5))
            else:
                res = {"metric": METRIC, "value": c5["pairs_per_s"], "unit": "pairs/s", "n_gpus": c5["n_gpus"],
                       "steps": args.steps, "warmup": args.warmup, "ms_per_step": c5["ms_per_frame"],
                       "ms_per_frame": c5["ms_per_frame"], "higher_is_better": True, "scaling": "strong",
                       "vs_baseline": None, "dtype": "u8", "data": "synthetic (numpy PCG64 textured pair, resident in HBM)",
                       "config": {"workload": c5["workload"], "width": c5["width"], "height": c5["height"],
                                  "num_disparities": c5["num_disparities"],
                                  "parallelism": "single device" if c5["n_gpus"] == 1 else f"row-band tiles x{c5['n_gpus']}"},
                       "roofline": c5["roofline"], "c5": c5}
                print(json.dumps(res))
        if distributed:
            dist.destroy_process_group()
        return

    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    W, H, D = cfg["w"], cfg["h"], cfg["D"]
    params = pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D, min_disparity=0, p1=10, p2=120,
                                uniqueness_ratio=5, subpixel=cfg["subpixel"], lr_check=cfg["lr_check"],
                                disp12_max_diff=1, median=0, speckle_window_size=0)
    eng = pkg.Engine(device, params)

    # inputs resident in HBM before timing (distinct frames per rank)
    ids = shard_frames(args.distinct, rank)
    dl, dr = [], []
    for i in ids:
        l, r, _ = synth.stereo_pair(H, W, 0, D, seed=i, with_truth=False)
        dl.append(torch.from_numpy(l).to(device))
        dr.append(torch.from_numpy(r).to(device))
    out = torch.empty((args.frames, H, W), dtype=torch.int16, device=device)
    torch.cuda.synchronize()
    tstream = torch.cuda.Stream(device)        # the stream every kernel and HIP event runs on
    stream = tstream.cuda_stream

    maps = None
    if args.rectify:      # maps once per calibration, remap fused with the census
        f = 0.9 * W
        K = np.array([[f, 0, W / 2 + 3.3], [0, f * 1.01, H / 2 - 2.1], [0, 0, 1]])
        Dd = np.array([-0.21, 0.07, 0.0012, -0.0009, -0.011])
        P = np.array([[0.98 * f, 0, W / 2 - 5.0, 0], [0, 0.98 * f, H / 2 + 1.5, 0], [0, 0, 1, 0]])
        maps = [torch.empty((H, W), dtype=torch.float32, device=device) for _ in range(2)]
        eng.rectify_map(K, Dd, None, P, W, H, maps[0].data_ptr(), maps[1].data_ptr(), W)
        eng.synchronize()
        eng.set_rectification((maps[0].data_ptr(), maps[1].data_ptr()), (maps[0].data_ptr(), maps[1].data_ptr()),
                              W, W, H)
    ptr_l = [dl[f % len(dl)].data_ptr() for f in range(args.frames)]
    ptr_r = [dr[f % len(dr)].data_ptr() for f in range(args.frames)]
    ptr_o = [out[f].data_ptr() for f in range(args.frames)]

    if args.host_io:      # host buffers (pageable numpy frames), streamed by sgm_match_batch
        host_l = [dl[f % len(dl)].cpu().numpy() for f in range(args.frames)]
        host_r = [dr[f % len(dr)].cpu().numpy() for f in range(args.frames)]
        host_o = [np.empty((H, W), np.int16) for _ in range(args.frames)]

    def step():
        if args.host_io:
            eng.match_batch(host_l, host_r, devices=[device], outs=host_o)
        elif args.no_pipeline:
            for f in range(args.frames):
                eng.match_device(ptr_l[f], ptr_r[f], W, H, W, ptr_o[f], W, stream)
        else:   # frame pipeline: paths of frame f+1 share a launch with the WTA of frame f
            eng.match_device_batch(ptr_l, ptr_r, W, H, W, ptr_o, W, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    eng.set_profiling(True)          # hipEvents around every stage, no host sync per frame
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stages = eng.stage_times()
    launches = eng.stage_launches()
    n_prof = eng.profiled_matches()
    eng.set_profiling(False)

    elapsed_max = max_over_ranks(elapsed, None if args.share_device else device)
    shard = gather_shard(ids, elapsed, distributed, device=device_identity(device), group=wait_group)

    # single-frame latency beside the batch throughput (BASELINE's C2 is quoted as a single
    # frame): one sgm_match_device per frame on resident buffers, HIP events on the stream
    single = None
    if rank == 0 and not args.host_io:
        reps = 10
        one = lambda i: eng.match_device(ptr_l[i % len(ptr_l)], ptr_r[i % len(ptr_r)], W, H, W, ptr_o[i % len(ptr_o)],
                                         W, stream)
        one(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(tstream)
        for i in range(reps):
            one(i)
        e1.record(tstream)
        torch.cuda.synchronize()
        eng.set_profiling(True)          # per-stage split in a separate pass
        for i in range(reps):
            one(i)
        torch.cuda.synchronize()
        single = {"ms": round(e0.elapsed_time(e1) / reps, 4), "pairs_per_s": round(1000.0 * reps / e0.elapsed_time(e1), 1),
                  "stages": {n: round(ms, 4) for n, ms, _ in eng.stage_times()},
                  "note": "one frame per sgm_match_device call (census -> 8 directions -> WTA), no batching"}
        eng.set_profiling(False)

    frames_total = args.frames * args.steps * world
    value = frames_total / elapsed_max
    ms_per_step = elapsed_max * 1e3 / args.steps

    if rank == 0:
        g = pkg.effective_geometry(params, W, H)
        b_alg = algorithmic_bytes(W, H, D)                   # graded
        b_alg_w1 = algorithmic_bytes(W, H, D, g["width1"])   # cells actually aggregated
        roofline = pipeline = None
        if stages:
            # per-frame device time: every launch of every stage, over the profiled frames
            dev_frame_ms = sum(ms * launches[n] for n, ms, _ in stages) / max(n_prof, 1)
            dom = max(stages, key=lambda s: s[1] * launches[s[0]])   # the kernel that takes the most time
            # the dominant launch in stereo pairs: its engine-side bytes (width1 cells) over one
            # pair's, to the nearest half pair (a path sweep or a WTA of one frame is half the
            # volume round trip); its graded bytes are that many SURVEY pairs
            pairs_per_launch = round(2.0 * dom[2] / b_alg_w1) / 2.0
            dom_bytes = pairs_per_launch * b_alg
            dom_achieved = dom_bytes / (dom[1] * 1e-3) / 1e9
            dom_achieved_w1 = dom[2] / (dom[1] * 1e-3) / 1e9
            pipe_achieved = b_alg / (dev_frame_ms * 1e-3) / 1e9
            pipe_achieved_w1 = b_alg_w1 / (dev_frame_ms * 1e-3) / 1e9
            # HBM bytes from PMC counters need rocprofv3 (a separate run): `traffic` stays null
            # here; the committed PMC summary of the same launch kind is quoted beside it
            pmc = load_pmc_traffic(args.config)
            traffic_profile = None
            if pmc and pmc.get("config") == args.config and dom[0] in pmc.get("kernels", {}):
                traffic_profile = {"hbm_bytes_per_launch": pmc["kernels"][dom[0]].get("hbm_bytes_per_launch"),
                                   "source": f"profiles/latest_pmc_{args.config}.json (rocprofv3 --pmc, separate run; "
                                             "tools/refresh_profiles.sh)", "git": pmc.get("git")}
            copy_gbps = hbm_copy_gbps(device)
            roofline = {"bound": "hbm", "kernel": dom[0], "achieved": round(dom_achieved, 1),
                        "measured_copy_GBps": copy_gbps,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(dom_achieved / HBM_PEAK_GBS, 4),
                        "traffic": None, "traffic_profile": traffic_profile,
                        "algorithmic_bytes_per_launch": dom_bytes,
                        "pairs_per_launch": pairs_per_launch, "avg_launch_ms": round(dom[1], 5),
                        "basis": "SURVEY 8d B_alg = W*H*(16*D+4) per pair (counts all W columns, including "
                                 "the W-width1 columns OpenCV never aggregates)",
                        "width1_basis": {"bytes_per_launch": dom[2], "achieved": round(dom_achieved_w1, 1),
                                         "frac": round(dom_achieved_w1 / HBM_PEAK_GBS, 4),
                                         "basis": "the same dataflow over the width1*H*D cells aggregated"}}
            pipeline = {"bound": "hbm", "B_alg_per_pair": b_alg, "device_ms_per_pair": round(dev_frame_ms, 5),
                        "achieved": round(pipe_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(pipe_achieved / HBM_PEAK_GBS, 4),
                        "width1_basis": {"B_alg_per_pair": b_alg_w1, "achieved": round(pipe_achieved_w1, 1),
                                         "frac": round(pipe_achieved_w1 / HBM_PEAK_GBS, 4)}}
        res = {
            "metric": METRIC, "value": round(value, 3), "unit": "pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "ms_per_frame": round(elapsed_max * 1e3 / (args.frames * args.steps), 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (numpy PCG64 textured pairs, piecewise-planar truth, " +
                    ("host buffers: PCIe in/out inside the timed region)" if args.host_io else "resident in HBM)"),
            "config": {"workload": cfg["name"], "width": W, "height": H, "num_disparities": D,
                       "frames_per_rank_per_step": args.frames, "global_batch": args.frames * world,
                       "distinct_frames_per_rank": args.distinct, "parallelism": f"frame-shard x{world}",
                       "frame_pipeline": not args.no_pipeline, "rectify_fused": bool(args.rectify),
                       **({"shared_device_test": True} if args.share_device else {}),
                       "host_io": bool(args.host_io)},
            "roofline": roofline,
            "pipeline": pipeline,
            "stages": [{"name": n, "avg_ms": round(ms, 5), "launches": launches[n], "alg_bytes": b,
                        "GBps": round(b / (ms * 1e-3) / 1e9, 1)} for n, ms, b in stages],
            "profiled_frames": n_prof,
            "single_frame": single,
            "shard": shard,
            "distinct_devices": distinct_devices(shard),
        }
    eng.close()
    if rank == 0:
        if args.config == "c3" and not args.no_c5 and not args.host_io and not args.rectify:
            res["c5"] = c5_leg(args, world)          # the other ranks wait at the barrier below
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(res))
    if distributed:
        # rank 0's single-frame / C5 / CPU legs end before the group does; the wait is on the gloo
        # group, so devices 1..N-1 are idle while the C5 child tiles over them
        dist.barrier(group=wait_group)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
