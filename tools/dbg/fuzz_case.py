"""Debug one fuzz case (tests/test_gpu_fuzz.py): cost volume and final output vs oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__ as ge
from conftest import to_oracle_params
import test_gpu_fuzz as tf

pkg = ge.load_package()
orc = ge._load_file("sgm_oracle", os.path.join(ROOT, "oracle", "sgm_oracle.py"))
synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
eng = pkg.Engine(0)
for seed in map(int, sys.argv[1:]):
    rng, mode, h, w, kw, kind = tf._case(pkg, seed)
    p = pkg.default_params(mode, **kw)
    eng.set_params(p)
    left, right = tf._images(rng, synth, h, w, kw["min_disparity"], kw["num_disparities"], kind, seed)
    op = to_oracle_params(orc, p)
    cg, cr = eng.ocv_cost(left, right), orc.ocv_cost(op, left, right)
    print(seed, kw, "cost differ:", int((cg != cr).sum()), "of", cg.size, "max", int(cr.max()), int(cr.min()))
    g, r = eng.match(left, right), orc.match(op, left, right)
    idx = np.argwhere(g != r)
    print("  out differ:", len(idx), [(tuple(i), int(g[tuple(i)]), int(r[tuple(i)])) for i in idx[:8]])
    for variant in ("SGM_OCV_NO_BUF", "SGM_OCV_LPL"):
        pass
eng.close()
