"""bench.py's own rank launcher (`--gpus N` without torchrun, the command the driver runs) on
CPU: `--dry-run` runs the rank / shard / MAX-timing logic with gloo and no HIP, so the test
sees N rank processes with disjoint frames and the MAX timing, and the error exits (too few
devices, WORLD_SIZE != --gpus) without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def _bench(*argv, env_extra=None, timeout=150):
    env = {k: v for k, v in os.environ.items() if k not in RANK_VARS}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def _line(p):
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout              # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


@pytest.mark.timeout(200)
@pytest.mark.parametrize("n", [2, 3])
def test_launcher_starts_n_ranks_with_disjoint_frames(n):
    res = _line(_bench("--gpus", str(n), "--dry-run", "--steps", "4", "--warmup", "1", "--frames", "5",
                       "--distinct", "3"))
    assert res["n_gpus"] == n
    shard = res["shard"]
    assert len(shard) == n
    seeds = [s for r in shard for s in r["seeds"]]
    assert len(seeds) == len(set(seeds)) == 3 * n                 # disjoint, every rank its own frames
    el = [r["elapsed_s"] for r in shard]
    assert res["elapsed_max_s"] == pytest.approx(max(el), abs=2e-6)  # MAX over ranks, not rank 0's time
    busy = [r["busy_s"] for r in shard]
    assert busy[-1] > busy[0]                                      # rank r sleeps (1 + r) ms per step
    assert res["elapsed_max_s"] >= max(busy)                       # the slowest rank bounds the time
    assert res["value"] == pytest.approx(5 * 4 * n / res["elapsed_max_s"], rel=1e-3)
    # self-proving record: every rank reports the world size it saw and its device
    assert [r["world_size"] for r in shard] == [n] * n
    assert [r["rank"] for r in shard] == list(range(n))
    assert sorted(r["device"]["ordinal"] for r in shard) == list(range(n))
    assert res["distinct_devices"] == n


def test_single_rank_dry_run():
    res = _line(_bench("--dry-run", "--steps", "2", "--warmup", "0"))
    assert res["n_gpus"] == 1 and len(res["shard"]) == 1
    assert res["shard"][0]["world_size"] == 1 and res["distinct_devices"] == 1


def test_waits_outside_the_timed_region_use_a_gloo_group():
    """The post-timing waits (rank 0 alone runs the single-frame / C5 / CPU legs, and the C5 child
    tiles over every device) and the shard gather go over a gloo group, so ranks 1..N-1 hold no
    RCCL kernel on their devices while C5 is timed."""
    import ast
    src = open(os.path.join(ROOT, "bench.py")).read()
    tree = ast.parse(src)
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    code = ast.get_source_segment(src, main)
    assert 'wait_group = dist.new_group(backend="gloo")' in code
    tail = code[code.index("eng.close()"):]                 # everything after the timed region
    barriers = [l.strip() for l in tail.splitlines() if "dist.barrier(" in l]
    assert barriers and all("group=wait_group" in b for b in barriers), barriers
    assert "group=wait_group" in code[code.index("shard = gather_shard"):].splitlines()[0]


def test_world_size_must_equal_gpus():
    p = _bench("--gpus", "3", "--dry-run", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "must equal --gpus" in p.stderr


def test_too_few_devices_exits_nonzero():
    # this container has no GPU: the launcher must refuse instead of timing fewer GPUs
    p = _bench("--gpus", "4", "--steps", "1")
    assert p.returncode != 0 and "HIP device" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
