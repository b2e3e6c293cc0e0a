"""Per-direction path-kernel timing at C3 (run under rocprofv3 --kernel-trace)."""
import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from conftest import _load
pkg = ge.load_package()
synth = _load("sgm_synth", ge.PKG_DIR + "/synth.py")
eng = pkg.Engine(0)
D = int(os.environ.get("D", 256))
left, right, _ = synth.stereo_pair(1080, 1920, 0, D, seed=1)
eng.set_params(pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
for rep in range(3):
    for d in range(8):
        eng.census_path(left, right, d)
eng.match(left, right)
print("ok")
