import os, sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import __graft_entry__ as ge
pkg = ge.load_package()
from conftest import to_oracle_params
import importlib.util
spec = importlib.util.spec_from_file_location("sgm_oracle", "oracle/sgm_oracle.py"); oracle = importlib.util.module_from_spec(spec); spec.loader.exec_module(oracle)
from conftest import _load
synth = _load("sgm_synth", ge.PKG_DIR + "/synth.py")
eng = pkg.Engine(0)
for kw in [dict(num_disparities=32, min_disparity=5, uniqueness_ratio=15), dict(num_disparities=32, min_disparity=0, uniqueness_ratio=15),
           dict(num_disparities=32, min_disparity=5), dict(num_disparities=64, uniqueness_ratio=15), dict(num_disparities=16, p1=3, p2=20, disp12_max_diff=3),
           dict(num_disparities=32, min_disparity=-9), dict(num_disparities=256, uniqueness_ratio=0), dict(num_disparities=512)]:
    D, minD = kw["num_disparities"], kw.get("min_disparity", 0)
    h, w = 61, max(D + minD, 0) + 133
    left, right, _ = synth.stereo_pair(h, w, max(minD, 0), D, seed=D + 17)
    p = pkg.default_params(pkg.MODE_CENSUS8, **kw)
    eng.set_params(p)
    got = eng.match(left, right)
    ref = oracle.match(to_oracle_params(oracle, p), left, right)
    bad = np.argwhere(got != ref)
    print(kw, "diff", len(bad), [(int(y), int(x), int(got[y, x]), int(ref[y, x])) for y, x in bad[:8]])
    p.median = 0; eng.set_params(p)
    got = eng.match(left, right); ref = oracle.match(to_oracle_params(oracle, p), left, right)
    bad = np.argwhere(got != ref)
    print("   nomedian diff", len(bad), [(int(y), int(x), int(got[y, x]), int(ref[y, x])) for y, x in bad[:8]])
