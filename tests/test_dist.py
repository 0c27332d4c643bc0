"""Multi-process (gloo, world size 2, CPU) tests of the sharding and timing logic the
multi-GPU bench uses: every block is owned by exactly one rank, per-rank ranges are
contiguous and balanced, and the max-over-ranks reduction returns the slowest rank."""

import os
import socket

import pytest

from alpenglow_amd.shard import block_range, max_over_ranks


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("total", [0, 1, 7, 4096, 65536])
def test_block_range_partitions(world, total):
    seen = []
    for r in range(world):
        a, b = block_range(r, world, total)
        assert 0 <= a <= b <= total
        seen.extend(range(a, b))
        assert b - a in (total // world, total // world + 1)
    assert seen == list(range(total))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = block_range(rank, world, 65536)
    # every rank "processes" its blocks; the reported time is the max over ranks
    t = max_over_ranks(1.0 + rank, dist)
    cnt = __import__("torch").tensor([b - a])
    dist.all_reduce(cnt)
    q.put((rank, t, int(cnt.item())))
    dist.destroy_process_group()


def test_gloo_world2_max_and_coverage():
    import torch.multiprocessing as mp

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, cnt in res:
        assert t == 2.0          # slowest rank's time everywhere
        assert cnt == 65536      # blocks covered exactly once in total
