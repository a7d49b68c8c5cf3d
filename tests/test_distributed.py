"""CPU (gloo, world_size 2): the N>1 path of bench.py -- disjoint image shards per
rank, max-over-ranks wall time, whole-job MPix/s.  No GPU, no RCCL: the data path
has no collective (images are independent)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = bench.reduce_max(elapsed, dist, "cpu")
    seeds = bench.shard_seeds(rank, 32)
    gathered = [None] * world
    dist.all_gather_object(gathered, seeds)
    q.put((rank, m, gathered, bench.aggregate_mpix(world, 32 * 10, 4096, m)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_aggregation():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, m, gathered, value in res:
        assert m == 2.0  # max over ranks
        a, b = set(gathered[0]), set(gathered[1])
        assert a and b and not (a & b)  # disjoint shards
        assert value == pytest.approx(2 * 32 * 10 * 4096 * 4096 / 2.0 / 1e6)


def _lt_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "rust-image-transform_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import loadtest
    from imagekit import ImageFormat
    fmts = [ImageFormat.webp, ImageFormat.jpeg, ImageFormat.avif]
    mine = loadtest.shard(loadtest.make_requests(257, 8, fmts, 0), rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, [(s, w, h, f.value) for s, w, h, f in mine])
    q.put((rank, gathered))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_loadtest_request_sharding(world):
    """tools/loadtest.py (configs[3]): every request served by exactly one rank, the
    same mix on every rank (seeded), w/h in [200, 800) as loadtest/src/main.rs:84-85."""
    sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "rust-image-transform_amd")]
    import loadtest
    from imagekit import ImageFormat
    fmts = [ImageFormat.webp, ImageFormat.jpeg, ImageFormat.avif]
    allreq = [(s, w, h, f.value) for s, w, h, f in loadtest.make_requests(257, 8, fmts, 0)]
    assert all(200 <= w < 800 and 200 <= h < 800 and 0 <= s < 8 for s, w, h, _ in allreq)
    assert {f for *_, f in allreq} == {0, 1, 2}
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered = res[0][1]
    assert sum(len(g) for g in gathered) == len(allreq)
    served = sorted(i for r in range(world) for i in range(r, len(allreq), world))
    assert served == list(range(len(allreq)))
    for r in range(world):
        assert gathered[r] == allreq[r::world]
