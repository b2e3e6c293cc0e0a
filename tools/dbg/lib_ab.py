"""Interleaved A/B of library builds (LIBS=a.so,b.so) on census batches and single frames
(CASES=HxWxD,...; NF frames per batch). Each build runs in its own child process."""
import os, subprocess, sys, json
libs = os.environ["LIBS"].split(",")
child = r'''
import os, sys
sys.path.insert(0, "/root/repo")
import torch
import __graft_entry__ as ge
pkg = ge.load_package()
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
cases = [tuple(int(v) for v in c.split("x")) for c in os.environ.get("CASES", "1080x1920x256").split(",")]
n = int(os.environ.get("NF", "16"))
for (H, W, D) in cases:
    eng = pkg.Engine(0, pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
    fr = [synth.stereo_pair(H, W, 0, D, seed=i, with_truth=False) for i in range(4)]
    dl = [torch.from_numpy(fr[i % 4][0]).cuda() for i in range(n)]; dr = [torch.from_numpy(fr[i % 4][1]).cuda() for i in range(n)]
    outs = torch.empty((n, H, W), dtype=torch.int16, device="cuda"); st = torch.cuda.Stream()
    args = ([t.data_ptr() for t in dl], [t.data_ptr() for t in dr], W, H, W, [outs[i].data_ptr() for i in range(n)], W, st.cuda_stream)
    eng.match_device_batch(*args); st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); eng.match_device_batch(*args); e1.record(st); st.synchronize()
    bms = e0.elapsed_time(e1) / n
    run = lambda: eng.match_device(dl[0].data_ptr(), dr[0].data_ptr(), W, H, W, outs[0].data_ptr(), W, st.cuda_stream)
    run(); st.synchronize()
    e0.record(st); [run() for _ in range(3)]; e1.record(st); st.synchronize()
    print(f"{os.path.basename(os.environ['SGM_HIP_LIB']):22s} {H}x{W} D={D}: batch {bms:.3f} ms/frame, single {e0.elapsed_time(e1) / 3:.3f} ms", flush=True)
    eng.close()
'''
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for lib in libs:
        r = subprocess.run([sys.executable, "-c", child], env=dict(os.environ, SGM_HIP_LIB=lib), capture_output=True, text=True, timeout=600)
        sys.stdout.write(r.stdout); sys.stdout.flush()
        if r.returncode:
            sys.stdout.write(r.stderr[-2000:]); sys.exit(r.returncode)
