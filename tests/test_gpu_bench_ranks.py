"""bench.py's N > 1 path end to end on one MI355X (VERDICT r4 "do this" #5): the launcher
starts 2 real rank processes, each runs the HIP engine on its own frames (both on device 0,
`--share-device`: a test-only switch that takes gloo for the rank group, since RCCL cannot
place two ranks on one GPU), the timed region is bracketed by barriers, the MAX over ranks is
reduced, and rank 0 prints one JSON line. The driver's 8-GPU run takes the same code with one
device per rank and RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


@pytest.mark.timeout(400)
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_bench_two_ranks_on_one_device(config):
    env = {k: v for k, v in os.environ.items() if k not in RANK_VARS}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", config,
                        "--steps", "3", "--warmup", "1", "--frames", "4", "--distinct", "2", "--share-device",
                        "--no-c5", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=360,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout                       # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["shared_device_test"]
    assert res["config"]["global_batch"] == 8
    shard = res["shard"]
    assert len(shard) == 2
    seeds = [s for r in shard for s in r["seeds"]]
    assert len(seeds) == len(set(seeds)) == 4                # disjoint frames per rank
    el = max(r["elapsed_s"] for r in shard)
    assert res["ms_per_step"] == pytest.approx(el * 1e3 / 3, rel=1e-3)   # the MAX over ranks
    assert res["value"] == pytest.approx(4 * 3 * 2 / el, rel=1e-3)
    assert res["roofline"]["frac"] > 0.05 and res["single_frame"]["ms"] > 0
    # the record names each rank's device (both on device 0 here) and the world size it saw
    assert [r["world_size"] for r in shard] == [2, 2]
    devs = [r["device"] for r in shard]
    assert all(d["ordinal"] == 0 and (d["pci"] or d["uuid"]) for d in devs), devs
    assert devs[0]["pci"] == devs[1]["pci"] and res["distinct_devices"] == 1
