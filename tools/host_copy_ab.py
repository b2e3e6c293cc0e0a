"""A/B of the adapter's copy-out: MatcherCore::forwardMatch (plugin_core_test
time) on the C3 census frame without post filters, output registered (sgm_host_register) or
pageable, interleaved rounds. One JSON line per run. (Round 4 also timed a banded copy-out
behind a banded WTA, SGM_OUT_CHUNKS=4: no gain, removed; profiles/r04_host_copy_ab.jsonl.)

    python tools/host_copy_ab.py [--rounds 3] [--reps 30]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    synth = ge._load_file("sgm_synth", os.path.join(ge.PKG_DIR, "synth.py"))
    core = os.path.join(ge.PKG_DIR, "lib", "plugin_core_test")
    h, w, D = 1080, 1920, 256
    left, right, _ = synth.stereo_pair(h, w, 0, D, seed=3, with_truth=False)
    with tempfile.TemporaryDirectory() as td:
        lf, rf = os.path.join(td, "l.raw"), os.path.join(td, "r.raw")
        left.tofile(lf)
        right.tofile(rf)
        for rnd in range(a.rounds):
            for name, reg in (("pageable", 0), ("registered", 1)):
                env = dict(os.environ)
                r = subprocess.run([core, "time", lf, rf, str(w), str(h), "2", str(D), "0", "5", str(a.reps), "0",
                                    str(reg)], capture_output=True, text=True, timeout=300, env=env)
                rec = {"round": rnd, "variant": name}
                if r.returncode == 0:
                    rec.update(json.loads(r.stdout.strip().splitlines()[-1]))
                else:
                    rec["error"] = r.stderr[-300:]
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
