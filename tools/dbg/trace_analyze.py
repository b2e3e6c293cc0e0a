"""Analyse an SGM_TRACE path-launch timeline: span, per-direction durations, per-CU load."""
import sys, collections
import numpy as np
for path in sys.argv[1:]:
    a = np.fromfile(path, np.uint64).reshape(-1, 4)
    a = a[a[:, 3] > 0]
    it, hw, t0, t1 = a[:, 0], a[:, 1], a[:, 2].astype(np.int64), a[:, 3].astype(np.int64)
    T0 = t0.min()
    s0 = (t0 - T0) / 100.0  # us (100 MHz)
    s1 = (t1 - T0) / 100.0
    dirs = ((it & np.uint64(0xFFFFFFFF)) >> np.uint64(24)).astype(int)
    span = s1.max()
    hwi = hw.astype(np.int64)
    cu = (hwi & 0xFFFFFFFF) >> 8 & 0xF           # CU_ID bits 11:8
    se = (hwi & 0xFFFFFFFF) >> 13 & 0x7           # SE_ID bits 15:13
    simd = (hwi & 0xFFFFFFFF) >> 4 & 0x3
    xcc = hwi >> 32 & 0xF
    key = xcc * 1000 + se * 100 + cu
    print(f"{path}: records {len(a)}  span {span:.1f} us")
    for d in range(8):
        m = dirs == d
        if m.any():
            dur = s1[m] - s0[m]
            print(f"  dir {d}: n {m.sum():4d} dur mean {dur.mean():7.1f} max {dur.max():7.1f} us  last end {s1[m].max():7.1f}")
    # per-CU busy (union of wave intervals of SIMD 0 only)
    ends = collections.defaultdict(float)
    for k, e in zip(key, s1):
        ends[k] = max(ends[k], e)
    e = np.array(list(ends.values()))
    print(f"  CUs {len(e)}: last-wave end min {e.min():.1f} median {np.median(e):.1f} max {e.max():.1f} us")
    # timeline of concurrent waves
    ts = np.linspace(0, span, 11)
    conc = [int(((s0 <= t) & (s1 > t)).sum()) for t in ts]
    print("  concurrent waves at 0..100%:", conc)
