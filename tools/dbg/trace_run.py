"""Run the C3 path launch with SGM_TRACE set (debug timeline), several variants."""
import os, sys, subprocess
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from conftest import _load
pkg = ge.load_package()
synth = _load("sgm_synth", ge.PKG_DIR + "/synth.py")
eng = pkg.Engine(0)
D = int(os.environ.get("TRACE_D", "256"))
left, right, _ = synth.stereo_pair(1080, 1920, 0, D, seed=1)
eng.set_params(pkg.default_params(pkg.MODE_CENSUS8, num_disparities=D))
out = os.environ["SGM_TRACE"]
for rep in range(3):
    eng.match(left, right)
print("ok")
