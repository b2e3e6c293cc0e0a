"""Multi-rank logic of bench.py on CPU (gloo, world_size 2): frame sharding is disjoint and
covers every frame once, and the timing reduction is a MAX over ranks. The GPU path uses
the same functions over RCCL (bench.py --gpus N under torchrun)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    frames = bench.shard_frames(3, rank)
    t = bench.max_over_ranks(0.5 + rank)         # rank 1 is the slowest
    objs = [None] * world
    dist.all_gather_object(objs, frames)
    q.put((rank, frames, t, objs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_sharding_and_max_timing_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    res.sort()
    for rank, frames, t, objs in res:
        assert t == pytest.approx(1.5)                      # MAX over ranks, not the local time
        allf = [f for fr in objs for f in fr]
        assert len(allf) == len(set(allf)) == 3 * world     # disjoint, every frame once
    assert res[0][1] != res[1][1]


def test_shard_frames_single_rank():
    import bench
    assert bench.shard_frames(4, 0) == [0, 1, 2, 3]
    assert bench.max_over_ranks(2.5) == 2.5
