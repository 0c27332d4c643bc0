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


# ---- the bench's rank logic (bench.py uses exactly these) ----------------------------

from alpenglow_amd.shard import SEED_BASE, RankPlan, erasure_patterns  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_plan_weak_and_strong(world):
    B, steps = 1 << 20, 20
    weak = [RankPlan(r, world, 4096) for r in range(world)]
    assert [p.first for p in weak] == [4096 * r for r in range(world)]
    assert all(p.nblocks == 4096 and p.scaling == "weak" for p in weak)
    assert {p.processed_bytes(B, steps) for p in weak} == {world * 4096 * B * steps}
    strong = [RankPlan(r, world, 4096, stream_blocks=65536) for r in range(world)]
    assert sum(p.nblocks for p in strong) == 65536 and all(p.scaling == "strong" for p in strong)
    assert {p.processed_bytes(B, steps) for p in strong} == {65536 * B * steps}
    # seeds: block g of the stream is SEED_BASE + g on whichever rank owns it
    seeds = [p.seed_base + i for p in strong for i in range(p.nblocks)]
    assert seeds == [SEED_BASE + g for g in range(65536)]


def test_random_patterns_independent_of_world():
    k, m, e, lc = 32, 32, 16, 8
    whole = RankPlan(0, 1, 64)
    o1, r1 = erasure_patterns(whole, k, m, e, lc, True)
    parts = [erasure_patterns(RankPlan(r, 4, 16), k, m, e, lc, True) for r in range(4)]
    assert sum((p[0] for p in parts), []) == o1 and sum((p[1] for p in parts), []) == r1
    for b in range(64):
        assert o1[b * k:(b + 1) * k].count(0) == e and r1[b * m:(b + 1) * m].count(0) == lc
    o, r = erasure_patterns(whole, k, m, e, lc, False)
    assert o == [0] * e + [1] * (k - e) and r == [0] * lc + [1] * (m - lc)


def _bench_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = RankPlan(rank, world, 0, stream_blocks=1001)
    # every rank reports the bytes of the whole job; time is the slowest rank's
    wall = max_over_ranks(0.5 * (rank + 1), dist)
    own = torch.tensor([plan.first, plan.nblocks], dtype=torch.int64)
    got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(got, own)
    q.put((rank, wall, plan.processed_bytes(1 << 20, 5), [tuple(int(v) for v in g) for g in got]))
    dist.destroy_process_group()


def test_gloo_world2_bench_rank_logic():
    import torch.multiprocessing as mp

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, wall, processed, ranges in res:
        assert wall == 1.0
        assert processed == 1001 * (1 << 20) * 5
        assert ranges == [(0, 501), (501, 500)]  # contiguous, disjoint, covering the stream


# ---- bench.py's own launcher (`--gpus N` without torchrun) ------------------------------

import json  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("extra,firsts", [((), [0, 4096]), (("--stream-blocks", "65536"), [0, 32768])])
def test_bench_launcher_world2(extra, firsts):
    """`python bench.py --gpus 2` (the driver's form without torchrun) starts two fresh rank
    processes (gloo here, --dry-device: no GPU call) and rank 0 reports the 2-rank world,
    both ranks' wall times and their disjoint block ranges in its one JSON line."""
    r = _bench("--gpus", "2", "--dry-device", "--steps", "3", "--warmup", "0", *extra)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks"]["world_size"] == 2 and line["ranks"]["backend"] == "gloo"
    assert len(line["ranks"]["wall_s"]) == 2 and line["ranks"]["first_block"] == firsts
    assert line["scaling"] == ("strong" if extra else "weak")
    assert line["verify"]["per_rank"] == [True, True] and line["verify"]["all_ranks_ok"] is True
    if extra:  # the main measurement already is the stream: no second one
        assert "strong_stream" not in line
    else:      # BASELINE configs[4] from the driver's own command: the 65536-block stream
        sub = line["strong_stream"]
        assert sub["scaling"] == "strong" and sub["stream_blocks"] == 65536
        assert sub["first_block"] == [0, 32768] and sub["blocks_per_rank"] == [32768, 32768]
        assert len(sub["wall_s"]) == 2
        assert sub["verify"] == {"per_rank": [True, True], "all_ranks_ok": True}


@pytest.mark.parametrize("bad", [0, 1])
def test_bench_strong_stream_verify_fails_job(bad):
    """A rank whose stream range fails verification makes the job exit 4, with the weak
    measurement's verdicts intact and the stream's per-rank flags naming the rank."""
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--dry-stream-verify-fail-rank", str(bad))
    assert r.returncode == 4, (r.returncode, r.stderr)
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["strong_stream"]["verify"]["per_rank"] == [i != bad for i in range(2)]
    assert line["strong_stream"]["verify"]["all_ranks_ok"] is False
    assert line["verify"]["per_rank"] == [i != bad for i in range(2)]  # the job verdict folds it in


def test_bench_strong_stream_flags():
    """--strong-stream 0 turns the sub-line off; the headline shape has it on by default at
    every N, including the driver's N = 1 line (whose `value` stays configs[1] + configs[2]);
    other shapes (sweep points) have it off unless asked."""
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--strong-stream", "0")
    assert r.returncode == 0, r.stderr
    assert "strong_stream" not in json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    r = _bench("--gpus", "1", "--dry-device", "--steps", "1")
    assert r.returncode == 0, r.stderr
    sub = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])["strong_stream"]
    assert sub["stream_blocks"] == 65536 and sub["first_block"] == [0] and sub["blocks_per_rank"] == [65536]
    r = _bench("--gpus", "1", "--dry-device", "--steps", "1", "--k", "16", "--m", "4")
    assert r.returncode == 0, r.stderr
    assert "strong_stream" not in json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    r = _bench("--gpus", "1", "--dry-device", "--steps", "1", "--strong-stream", "1000")
    assert r.returncode == 0, r.stderr
    sub = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])["strong_stream"]
    assert sub["first_block"] == [0] and sub["blocks_per_rank"] == [1000]


@pytest.mark.parametrize("bad", [0, 1])
def test_bench_verify_aggregated_over_ranks(bad):
    """A rank whose verification fails (rank 1 here stands for GPUs 1-7, whose own checks
    rank 0 never sees) makes the whole job exit non-zero, and rank 0's line names it: the
    flags are all-gathered by the same _finish the device branch runs."""
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--dry-verify-fail-rank", str(bad))
    assert r.returncode == 4, (r.returncode, r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    v = json.loads(lines[0])["verify"]
    assert v["all_ranks_ok"] is False
    assert v["per_rank"] == [i != bad for i in range(2)]
    assert f"verification failed on rank(s) [{bad}]" in r.stderr


def test_bench_no_verify_reports_unverified():
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--no-verify")
    assert r.returncode == 0, r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["verify"] is None


def test_verify_over_ranks_single():
    from alpenglow_amd.shard import verify_over_ranks

    assert verify_over_ranks(True) == [True]
    assert verify_over_ranks(False) == [False]
    assert verify_over_ranks(None) == [None]


def test_bench_launcher_fails_loudly():
    """A rank that fails makes the launcher exit non-zero; an external launcher whose world
    differs from --gpus is refused."""
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--dry-fail-rank", "1")
    assert r.returncode != 0
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "launcher started 1 rank" in r.stderr


def _fake_sysfs(tmp_path, nodes):
    """A sysfs tree with one GPU per entry of ``nodes`` (bdf -> NUMA node) and node cpulists
    that split this process's CPUs in two."""
    cpus = sorted(os.sched_getaffinity(0))
    half = max(1, len(cpus) // 2)
    groups = {0: cpus[:half], 1: cpus[half:] or cpus[:half]}
    for node, cs in groups.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(",".join(str(c) for c in cs) + "\n")
    for bdf, node in nodes.items():
        d = tmp_path / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    return groups


def test_numa_helpers(tmp_path):
    from alpenglow_amd import shard

    groups = _fake_sysfs(tmp_path, {"0000:11:00.0": 1, "0000:21:00.0": -1})
    assert shard.parse_cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    assert shard.pci_numa_node("0000:11:00.0", str(tmp_path)) == 1
    assert shard.pci_numa_node("0000:21:00.0", str(tmp_path)) == -1  # single-node host
    assert shard.pci_numa_node("0000:99:00.0", str(tmp_path)) == -1  # no such device
    assert shard.node_cpus(1, str(tmp_path)) == set(groups[1])
    import numpy as np

    a = np.ones(1 << 22, np.uint8)
    assert shard.pages_numa_node(a.ctypes.data, a.nbytes) >= 0  # this host's node of the pages


def test_bench_pcie_numa_per_rank(tmp_path):
    """SURVEY §8e / VERDICT r5: with --pcie every rank binds to its GPU's NUMA node before it
    allocates its host staging, and rank 0's line carries one `pcie_inclusive` entry per rank
    with the node chosen, the CPUs bound and the node the staging pages landed on."""
    groups = _fake_sysfs(tmp_path, {"0000:11:00.0": 0, "0000:21:00.0": 1})
    r = _bench("--gpus", "2", "--dry-device", "--steps", "1", "--pcie", "--strong-stream", "0",
               "--dry-bdfs", "0000:11:00.0,0000:21:00.0", env_extra={"AG_SYSFS_ROOT": str(tmp_path)})
    assert r.returncode == 0, r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    pc = line["pcie_inclusive"]
    assert pc["n_ranks"] == 2 and [p["rank"] for p in pc["per_rank"]] == [0, 1]
    for rank, p in enumerate(pc["per_rank"]):
        numa = p["numa"]
        assert numa["bdf"] == ["0000:11:00.0", "0000:21:00.0"][rank]
        assert numa["numa_node"] == rank
        assert numa["cpus"] == len(groups[rank])
        assert isinstance(numa["staging_node"], int)
