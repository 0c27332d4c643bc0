#!/usr/bin/env python3
"""bench.py -- GiB/s device-resident RS shred encode+reconstruct, batched 1 MiB blocks.

Workload (BASELINE.json configs[1] + configs[2]): per GPU, 4096 random 1 MiB blocks,
32 data : 32 coding shards (shard = 32 KiB), inputs resident in HBM.  One step =
  encode:      32 data shards -> 32 coding shards for every block
  reconstruct: 16 of the 32 data shards erased per block, restored from the coding set
through the C ABI (libalpenglow_rs.so).  value = block payload bytes that went through
encode AND reconstruct, summed over ranks, per second of the max-over-ranks wall time.

Multi-GPU: one process per GPU.  Under an external launcher (torchrun: WORLD_SIZE set) the
launcher's world must equal --gpus; without one, `--gpus N` (N > 1) makes this process a
launcher that starts N fresh rank processes before any GPU call and exits non-zero if any
rank fails.  Each rank shards its own independent blocks (weak scaling, or --stream-blocks
for BASELINE configs[4]'s one stream split over the GPUs); there is no data-path collective,
the only collectives are the timing barrier, the max-over-ranks reduction and the gather of
per-rank wall times reported in the line.  For the headline shape (and no --stream-blocks)
the same run then also times configs[4]'s 65 536 x 1 MiB stream split contiguously over the
ranks -- at every N, N = 1 included (128 GiB of codewords in one GPU's HBM) -- and reports
it as the `strong_stream` sub-line (value, per-rank walls and verdicts); `value` stays the
weak-scaling figure, so the N = 1 line equals configs[1] + configs[2].

Also printed in the JSON line: per-kernel HIP-event timings on the launch stream with the
HBM roofline, a CPU baseline (the C oracle, a restatement of the reference algorithm, on a
bounded sample of the same blocks, rank 0 at N=1) and, with --pcie, the host-buffer
(PCIe-inclusive) rate of every rank, each rank's pinned staging on its GPU's NUMA node.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nblocks", type=int, default=4096, help="blocks per GPU (weak scaling)")
    ap.add_argument("--stream-blocks", type=int, default=0,
                    help="strong scaling: split one stream of this many blocks over the GPUs "
                         "(BASELINE configs[4]: 65536)")
    ap.add_argument("--strong-stream", type=int, default=-1,
                    help="after the main measurement, also time one stream of this many blocks split "
                         "contiguously over the ranks and report it as `strong_stream` (BASELINE "
                         "configs[4]); default: 65536 for the headline shape (32:32, 4096 x 1 MiB per "
                         "GPU, 16 data shreds erased) without --stream-blocks, else off")
    ap.add_argument("--block-bytes", type=int, default=1 << 20)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--erase", type=int, default=-1,
                    help="data shards erased per block (default: k/2, at most m)")
    ap.add_argument("--lose-coding", type=int, default=0,
                    help="coding shreds also lost per block (forces the general decoder)")
    ap.add_argument("--random-patterns", action="store_true",
                    help="seeded random erasure pattern per block instead of the first e data shreds")
    ap.add_argument("--only", choices=["both", "encode", "decode"], default="both",
                    help="profiling aid: time only one of the two kernels")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pcie", action="store_true",
                    help="also time host-buffer calls, on every rank, with each rank's host staging "
                         "on its GPU's NUMA node")
    ap.add_argument("--pcie-blocks", type=int, default=4096, help="blocks in the host-buffer run")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-settle", action="store_true",
                    help="skip the untimed clock-settle steps that follow the W warmup steps")
    ap.add_argument("--dry-device", action="store_true",
                    help="launcher / rank plumbing only (gloo, no GPU call, no kernel): the timed "
                         "steps are empty and the line reports no throughput (tests/test_dist.py)")
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-verify-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-stream-verify-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-bdfs", default="", help=argparse.SUPPRESS)  # per-rank PCI addresses (--dry-device)
    args = ap.parse_args()
    args.strong_stream_default = args.strong_stream < 0
    if args.strong_stream < 0:
        args.strong_stream = STREAM_BLOCKS if _headline_shape(args) and not args.stream_blocks else 0
    return args


def _headline_shape(args) -> bool:
    """The driver's workload (BASELINE configs[1] + [2]): the shape configs[4]'s stream uses."""
    return (args.k == 32 and args.m == 32 and args.block_bytes == 1 << 20 and args.erase in (-1, 16)
            and not args.lose_coding and not args.random_patterns and args.only == "both"
            and args.nblocks == 4096)


STREAM_BLOCKS = 65536  # BASELINE configs[4]: a 64k-block stream batch-sharded one range per GPU


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn_ranks(args) -> int:
    """`--gpus N` without an external launcher: start N fresh rank processes (this process
    makes no GPU call), one per GPU, and wait for them.  Returns the exit status: 0 only if
    every rank exited 0; the first failure stops the other ranks (their exact PIDs)."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def _init_rank(args, world: int, rank: int, local: int):
    """Bind this rank's device, then join the process group (shared by the device and the
    --dry-device branches).  The device is bound before init_process_group and passed as
    its device_id, so RCCL's communicator is created on this rank's GPU, never on GPU 0.
    Returns (dist or None, device or None)."""
    import torch.distributed as dist

    dev = None
    if not args.dry_device:
        import torch

        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world == 1:
        return None, dev
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.dry_device:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    if dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has "
                         f"{dist.get_world_size()} rank(s)")
    return dist, dev


def _finish(args, d, dev, rank: int, line, ok) -> int:
    """Shared tail of both branches: every rank's verify verdict is gathered onto every
    rank (a rank whose blocks came out wrong must not let the job exit 0), rank 0 prints
    its line with the per-rank verdicts, and every rank returns the exit status: 4 when
    any rank failed its verification, else 0."""
    from alpenglow_amd.shard import verify_over_ranks

    flags = verify_over_ranks(ok, d, dev)
    failed = [r for r, f in enumerate(flags) if f is False]
    if rank == 0:
        if line.get("verify") is not None or any(f is not None for f in flags):
            line["verify"] = dict(line.get("verify") or {}, per_rank=flags, all_ranks_ok=not failed)
        print(json.dumps(line), flush=True)
    if failed and rank == 0:
        print(f"bench.py: verification failed on rank(s) {failed}", file=sys.stderr, flush=True)
    return 4 if failed else 0


def _dry_main(args, world: int, rank: int, local: int) -> int:
    """The multi-rank harness without a device: gloo group, rank plan, barrier-bracketed
    empty steps, max-over-ranks wall time, gathered per-rank walls, the verify aggregation
    and exit status of the device branch (_finish), one JSON line."""
    from alpenglow_amd.shard import RankPlan, gather_over_ranks, max_over_ranks

    d, _ = _init_rank(args, world, rank, local)
    if rank == args.dry_fail_rank:
        raise SystemExit(3)
    plan = RankPlan(rank, world, args.nblocks, args.stream_blocks)
    if d:
        d.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if d:
        d.barrier()
    wall = time.perf_counter() - t0
    wall_max = max_over_ranks(wall, d)
    walls = gather_over_ranks(wall, d)
    firsts = gather_over_ranks(plan.first, d)
    # a rank's "verification" here is only the flag the test asks for (--dry-verify-fail-rank)
    ok = None if args.no_verify else rank != args.dry_verify_fail_rank
    pcie = None
    if args.pcie:
        # the NUMA placement only (no device, no transfer): bind to the GPU's node, allocate and
        # touch the staging there, report the node its pages landed on
        import numpy as np

        from alpenglow_amd.shard import bind_to_gpu_node, gather_objects, pages_numa_node

        bdfs = [b for b in args.dry_bdfs.split(",") if b]
        numa = bind_to_gpu_node(bdfs[rank] if rank < len(bdfs) else None)
        stage = np.ones(1 << 22, np.uint8)
        numa["staging_node"] = pages_numa_node(stage.ctypes.data, stage.nbytes)
        pcie = gather_objects(dict(rank=rank, numa=numa, blocks=0, matches_device_result=None), d)
    sub = None
    if args.strong_stream:
        splan = RankPlan(rank, world, 0, args.strong_stream)
        if d:
            d.barrier()
        t0 = time.perf_counter()
        if d:
            d.barrier()
        swall = time.perf_counter() - t0
        sok = None if args.no_verify else rank != args.dry_stream_verify_fail_rank
        sub = _stream_line(args, splan, d, None, swall, sok, value=None, ms_per_step=None)
        ok = _and_ok(ok, sok)
    line = None
    if rank == 0:
        line = {
            "metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": wall_max * 1e3 / max(args.steps, 1), "higher_is_better": True,
            "scaling": plan.scaling, "vs_baseline": None, "dry_device": True,
            "ranks": {"backend": "gloo" if world > 1 else None, "world_size": world, "wall_s": walls,
                      "first_block": [int(f) for f in firsts], "blocks_per_rank": plan.nblocks},
            "config": {"workload": _workload(args, world, plan.nblocks)},
            "verify": None,
        }
        if sub is not None:
            line["strong_stream"] = sub
        if pcie is not None:
            line["pcie_inclusive"] = _pcie_line(pcie)
    status = _finish(args, d, None, rank, line, ok)
    if d:
        d.destroy_process_group()
    return status


METRIC = "GiB/s device-resident RS shred encode+reconstruct, batched 1 MiB blocks"


def _and_ok(a, b):
    """Combine two verdicts (True / False / None = not verified)."""
    if a is False or b is False:
        return False
    if a is None and b is None:
        return None
    return True


def _stream_line(args, plan, d, dev, wall, ok, value, ms_per_step):
    """The `strong_stream` sub-line (BASELINE configs[4]): every rank's timed wall, first
    block and verdict gathered over the ranks (collectives: all ranks must call this).
    Returns the dict on rank 0, None elsewhere."""
    from alpenglow_amd.shard import gather_over_ranks, verify_over_ranks

    walls = gather_over_ranks(wall, d, dev)
    firsts = gather_over_ranks(plan.first, d, dev)
    counts = gather_over_ranks(plan.nblocks, d, dev)
    flags = verify_over_ranks(ok, d, dev)
    if plan.rank != 0:
        return None
    failed = [r for r, f in enumerate(flags) if f is False]
    return {
        "value": value, "unit": "GiB/s", "scaling": "strong", "stream_blocks": plan.total,
        "block_bytes": args.block_bytes, "steps": args.steps, "ms_per_step": ms_per_step,
        "wall_s": walls, "first_block": [int(f) for f in firsts], "blocks_per_rank": [int(c) for c in counts],
        "verify": None if all(f is None for f in flags) else {"per_rank": flags, "all_ranks_ok": not failed},
        "workload": f"{plan.total} x {_size(args.block_bytes)} block stream split contiguously over "
                    f"{plan.world} GPU(s), {args.k}:{args.m} encode + reconstruct",
    }


def _size(B):
    return f"{B >> 20} MiB" if B % (1 << 20) == 0 else f"{B / 1024:g} KiB" if B % 1024 == 0 else f"{B} B"


def _workload(args, world, n, e=None, lc=0):
    B = args.block_bytes
    s = (f"{args.stream_blocks} x {_size(B)} block stream over {world} GPU(s)" if args.stream_blocks
         else f"{n} x {_size(B)} blocks per GPU")
    if e is None:
        return s
    return (s + f", {args.k}:{args.m} encode + reconstruct with {e}/{args.k} data shreds erased"
            + (f" and {lc}/{args.m} coding shreds lost" if lc else "")
            + (" (random pattern per block)" if args.random_patterns else ""))


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args))  # launcher: no GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_device:
        sys.exit(_dry_main(args, world, rank, local))
    import torch

    from alpenglow_amd import rs

    dist, dev = _init_rank(args, world, rank, local)

    from alpenglow_amd.shard import RankPlan, erasure_patterns, gather_over_ranks, max_over_ranks

    k, m, B = args.k, args.m, args.block_bytes
    plan = RankPlan(rank, world, args.nblocks, args.stream_blocks)
    n = plan.nblocks
    if B % k or (B // k) % 2:
        raise SystemExit("block bytes must split into k even-sized shards")
    S = B // k
    e = args.erase if args.erase >= 0 else min(k // 2, m)
    lc = args.lose_coding
    if e + lc > m:
        raise SystemExit("erased data + lost coding shreds must not exceed m")
    cw_stride = (k + m) * S

    ctx = rs.Context(local)
    stream = torch.cuda.Stream(dev)  # explicit stream: torch work, kernels and events share it
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # codeword buffer: block b = k data shards then m coding shards (HBM-resident)
    cw = torch.empty((n, cw_stride), dtype=torch.uint8, device=dev)
    seed_base = plan.seed_base
    rs.fill_splitmix(ctx, cw, n, k * S, cw_stride, seed_base)
    data_ptr, par_ptr = cw.data_ptr(), cw.data_ptr() + k * S
    opres, rpres = erasure_patterns(plan, k, m, e, lc, args.random_patterns)
    opres_b, rpres_b = bytes(opres), bytes(rpres)  # converted once, outside the timed region

    def encode():
        rs.encode_batch(ctx, k, m, S, n, data_ptr, cw_stride, par_ptr, cw_stride)

    def reconstruct():
        rs.decode_batch(ctx, k, m, S, n, data_ptr, cw_stride, par_ptr, cw_stride, opres_b, rpres_b,
                        mode=rs.DECODE_ANY_K)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    do_enc = args.only in ("both", "encode")
    do_dec = args.only in ("both", "decode")
    def step():
        if do_enc:
            encode()
        if do_dec:
            reconstruct()

    encode()  # parity must exist before the first reconstruct
    for _ in range(args.warmup):
        step()
    settle = _settle(step, stream, torch) if not args.no_settle else 0

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        if do_enc:
            encode()
        ev[s][1].record(stream)
        if do_dec:
            reconstruct()
        ev[s][2].record(stream)
    barrier()
    wall = time.perf_counter() - t0
    enc_ms = sum(ev[s][0].elapsed_time(ev[s][1]) for s in range(args.steps)) / args.steps
    dec_ms = sum(ev[s][1].elapsed_time(ev[s][2]) for s in range(args.steps)) / args.steps

    wall_max = max_over_ranks(wall, dist, dev)
    walls = gather_over_ranks(wall, dist, dev)
    ms_per_step = wall_max * 1e3 / args.steps

    # full-size property check: zero the erased shards, reconstruct, compare with a fresh
    # regeneration of the data; and a 2-block bit-exact spot check of the parity vs oracle
    verify, ok = None, None
    view = None
    if not args.no_verify:
        # zero every shred the decoder is told is absent (erased data AND lost coding), so a
        # decoder that read an absent shred could not pass
        view = cw.view(n, k + m, S)
        lost = torch.tensor(opres, dtype=torch.uint8).view(-1, k)[: n if args.random_patterns else 1] == 0
        lost_r = torch.tensor(rpres, dtype=torch.uint8).view(-1, m)[: n if args.random_patterns else 1] == 0
        view[:, :k][lost.to(dev).expand(n, k)] = 0
        view[:, k:][lost_r.to(dev).expand(n, m)] = 0
        reconstruct()
        ref = torch.empty((n, k * S), dtype=torch.uint8, device=dev)
        rs.fill_splitmix(ctx, ref, n, k * S, k * S, seed_base)
        ok_rec = bool(torch.equal(cw[:, : k * S], ref))
        del ref
        encode()  # restore the zeroed coding shreds for the CPU baseline's parity comparison
        verify = {"reconstruct_restores_all_blocks": ok_rec}
        ok = ok_rec

    line = None
    if rank == 0:
        # each byte went through encode and reconstruct, once per timed step
        processed = plan.processed_bytes(B, args.steps)
        enc_bytes = n * B * (1 + m / k)
        dec_bytes = n * B * (1 + e / k)
        kern = {
            "encode": {"ms": enc_ms, "algorithmic_bytes": enc_bytes,
                       "achieved_GBps": enc_bytes / (enc_ms * 1e-3) / 1e9 if enc_ms else None},
            "reconstruct": {"ms": dec_ms, "algorithmic_bytes": dec_bytes,
                            "achieved_GBps": dec_bytes / (dec_ms * 1e-3) / 1e9 if dec_ms else None},
        }
        dom = "encode" if enc_ms >= dec_ms else "reconstruct"
        traffic = _pmc_traffic(dom, k, m, S, n)
        ach = kern[dom]["achieved_GBps"]
        line = {
            "metric": METRIC,
            "value": processed / (wall_max) / GIB,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": settle,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": plan.scaling,
            "vs_baseline": None,
            "dtype": "u8 (GF(2^16) symbols, bitsliced u32 planes)",
            "data": "synthetic (splitmix64 random blocks, device-generated)",
            "ranks": {"backend": "nccl (RCCL)" if dist else None,
                      "world_size": dist.get_world_size() if dist else 1,
                      "wall_s": walls, "blocks_per_rank": n},
            "config": {"workload": _workload(args, world, n, e, lc),
                       "blocks_per_gpu": n, "block_bytes": B, "shard_bytes": S,
                       "data_shreds": k, "coding_shreds": m, "erased_data_shreds": e,
                       "lost_coding_shreds": lc, "random_patterns": bool(args.random_patterns),
                       "parallelism": f"blocks sharded over {world} GPU(s), no collective",
                       "only": args.only},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": (ach / HBM_PEAK_GBPS) if ach else None,
                         "traffic": traffic},
            "kernels": kern,
            "step_roofline_frac": ((enc_bytes + dec_bytes) / ((enc_ms + dec_ms) * 1e-3) / 1e9
                                   / HBM_PEAK_GBPS) if (enc_ms + dec_ms) else None,
            "verify": verify,
        }
    # CPU baseline (rank 0, N = 1 only) on a bounded sample of the same blocks
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = _cpu_baseline(args, cw, k, m, S, e)
            ok = ok is not False and line["cpu_baseline"]["gpu_parity_matches_cpu"]
        else:
            line["cpu_baseline"] = None
    if args.pcie:
        # every rank moves its own blocks through its own host staging, concurrently
        from alpenglow_amd.shard import bind_to_gpu_node, gather_objects, gpu_bdf

        numa = bind_to_gpu_node(gpu_bdf(local))
        pc = _pcie(args, ctx, cw, k, m, S, e, torch, dev, barrier, numa)
        pc["rank"] = rank
        ok = _and_ok(ok, pc["matches_device_result"])
        per = gather_objects(pc, dist)
        if rank == 0:
            line["pcie_inclusive"] = _pcie_line(per)
    if args.strong_stream:
        # BASELINE configs[4]: the weak workload's buffers go first (the stream's codewords
        # are strong_stream / world x (k + m) x S bytes per rank: 128 GiB at N = 1)
        del cw, view
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        try:
            sub, sok = _strong_stream(args, ctx, dist, dev, torch, stream, rank, world, k, m, S, e, lc)
        except torch.cuda.OutOfMemoryError:
            # the default 128 GiB stream on one GPU whose HBM another tenant holds part of: the
            # main measurement stands; an explicitly requested stream (or any N > 1) fails loudly
            if world > 1 or not args.strong_stream_default:
                raise
            torch.cuda.empty_cache()
            sub, sok = {"skipped": "out of device memory", "stream_blocks": args.strong_stream}, None
        ok = _and_ok(ok, sok)
        if rank == 0:
            line["strong_stream"] = sub
    status = _finish(args, dist, dev, rank, line, ok)
    ctx.close()
    if dist:
        dist.destroy_process_group()
    sys.exit(status)


def _strong_stream(args, ctx, dist, dev, torch, stream, rank, world, k, m, S, e, lc):
    """BASELINE configs[4]: one stream of args.strong_stream blocks split into contiguous
    per-rank ranges (RankPlan strong), each rank encoding + reconstructing its range with no
    data-path collective; the same step, warmup / settle, barrier-bracketed K steps and
    max-over-ranks wall as the main measurement.  Verified afterwards on every rank (erased
    and lost shards zeroed, reconstructed, compared with a fresh regeneration group by
    group).  Returns (sub-line on rank 0 else None, this rank's verdict)."""
    from alpenglow_amd import rs
    from alpenglow_amd.shard import RankPlan, erasure_patterns, max_over_ranks

    plan = RankPlan(rank, world, 0, args.strong_stream)
    n, B, cw_stride = plan.nblocks, k * S, (k + m) * S
    cw = torch.empty((n, cw_stride), dtype=torch.uint8, device=dev)
    rs.fill_splitmix(ctx, cw, n, B, cw_stride, plan.seed_base)
    data_ptr, par_ptr = cw.data_ptr(), cw.data_ptr() + B
    opres, rpres = erasure_patterns(plan, k, m, e, lc, args.random_patterns)
    opres_b, rpres_b = bytes(opres), bytes(rpres)
    do_enc, do_dec = args.only in ("both", "encode"), args.only in ("both", "decode")

    def encode():
        rs.encode_batch(ctx, k, m, S, n, data_ptr, cw_stride, par_ptr, cw_stride)

    def reconstruct():
        rs.decode_batch(ctx, k, m, S, n, data_ptr, cw_stride, par_ptr, cw_stride, opres_b, rpres_b,
                        mode=rs.DECODE_ANY_K)

    def step():
        if do_enc:
            encode()
        if do_dec:
            reconstruct()

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    encode()
    for _ in range(args.warmup):
        step()
    if not args.no_settle:
        _settle(step, stream, torch, max_steps=50)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    wall = time.perf_counter() - t0
    wall_max = max_over_ranks(wall, dist, dev)
    ok = None
    if not args.no_verify:
        view = cw.view(n, k + m, S)
        lost = torch.tensor(opres, dtype=torch.uint8).view(-1, k)[: n if args.random_patterns else 1] == 0
        lost_r = torch.tensor(rpres, dtype=torch.uint8).view(-1, m)[: n if args.random_patterns else 1] == 0
        view[:, :k][lost.to(dev).expand(n, k)] = 0
        view[:, k:][lost_r.to(dev).expand(n, m)] = 0
        reconstruct()
        group = max(1, min(n, (4 << 30) // B))
        ref = torch.empty((group, B), dtype=torch.uint8, device=dev)
        ok = True
        for g0 in range(0, n, group):
            g = min(group, n - g0)
            rs.fill_splitmix(ctx, ref, g, B, B, plan.seed_base + g0)
            ok = ok and bool(torch.equal(cw[g0:g0 + g, :B], ref[:g]))
        del ref, view
    del cw
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    value = plan.processed_bytes(args.block_bytes, args.steps) / wall_max / GIB
    sub = _stream_line(args, plan, dist, dev, wall, ok, value, wall_max * 1e3 / args.steps)
    return sub, ok


def _settle(step, stream, torch, max_steps=200, min_steps=3, tol=0.01, window=4):
    """Untimed steps after the W warmup steps until the GPU has reached its steady state:
    a fresh box runs the first ~10-20 launches of each kernel 5-15% slower (clock ramp, cold
    TLBs; profiles/r01_kernel_trace_steady.txt).  Stops once the last `window` step times
    agree within `tol` (each step timed alone with HIP events on the launch stream), at
    most `max_steps` steps (about 0.6 s at the headline shape).  Returns the steps run."""
    times = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(max_steps):
        ev0.record(stream)
        step()
        ev1.record(stream)
        ev1.synchronize()
        times.append(ev0.elapsed_time(ev1))
        if i + 1 >= max(min_steps, window):
            last = times[-window:]
            if (max(last) - min(last)) <= tol * min(last):
                return i + 1
    return max_steps


def _pmc_traffic(kernel, k, m, S, n):
    """HBM bytes per launch measured with rocprofv3 PMC counters (profiles/pmc_traffic.json,
    written by tools/pmc_summary.py from separate --pmc passes); None when absent or for a
    different shape."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        rec = d["kernels"][kernel]
        if rec.get("shape") != [n, k, m, S]:
            return None
        return rec["hbm_bytes_per_launch"]
    except Exception:
        return None


def _host_cpus():
    """CPUs this process may use: the affinity set, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_baseline(args, cw, k, m, S, e):
    """The reference's CPU path timed on this host: oracle/rs_cpu_avx2.c restates the
    crate's Avx2 engine (nibble-table vpshufb multiplies over the crate's chunk layout,
    the per-call FWHT erasure locator of its decoder).  1 thread and all host CPUs, one
    block per thread, on a bounded sample of the same device blocks (bit-exact against the
    GPU's parity and restored shards), plus BASELINE configs[0] (one 64 KiB block) and the
    reference's own benches/shredder.rs slice shape, single-threaded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import ro_c

    engine = "avx2" if ro_c.avx2_available() and S % 64 == 0 else "scalar"
    nall = args.cpu_threads or _host_cpus()
    op = np.array([0] * e + [1] * (k - e), np.uint8)
    rp = np.array([0] * args.lose_coding + [1] * (m - args.lose_coding), np.uint8)
    B = k * S

    def run(nblk, threads):
        host = cw[:nblk].cpu().numpy().reshape(nblk, k + m, S)
        data = np.ascontiguousarray(host[:, :k])
        t = time.perf_counter()
        rec = ro_c.encode_blocks(data, m, threads=threads, engine=engine)
        te = time.perf_counter() - t
        cwh = np.concatenate([data, rec], axis=1)
        t = time.perf_counter()
        out = ro_c.decode_blocks(cwh, k, op, rp, threads=threads, engine=engine)
        td = time.perf_counter() - t
        ok = bool(np.array_equal(rec, host[:, k:])) and bool(np.array_equal(out, data))
        return {"blocks": nblk, "threads": threads, "encode_GiBps": nblk * B / te / GIB,
                "reconstruct_GiBps": nblk * B / td / GIB, "value": nblk * B / (te + td) / GIB,
                "seconds": te + td, "gpu_parity_matches_cpu": ok}

    # 1 thread: probe, then a sample of about a third of the budget
    probe = run(2, 1)
    n1 = int(max(2, min(cw.shape[0], args.cpu_seconds / 3 / max(probe["seconds"] / 2, 1e-6))))
    t1 = run(n1, 1)
    # all CPUs: one block per thread, about half the budget
    per_block = t1["seconds"] / n1
    nn = int(max(nall, min(cw.shape[0], args.cpu_seconds / 2 * nall / max(per_block, 1e-6))))
    nn = max(nall, nn // nall * nall)
    ta = run(min(nn, cw.shape[0]), nall)
    extra = _cpu_reference_shapes(ro_c, np, engine)
    return {
        "value": ta["value"],
        "unit": "GiB/s",
        "cores": nall,
        "kind": "port",
        "sample": f"{ta['blocks']} (all CPUs) and {t1['blocks']} (1 thread) of the same {B >> 20} MiB blocks, "
                  f"{k}:{m} encode + reconstruct with {e} data shreds erased; oracle/rs_cpu_avx2.c, the "
                  f"crate's {'Avx2' if engine == 'avx2' else 'scalar'} engine restated, one block per thread",
        "encode_GiBps": ta["encode_GiBps"],
        "reconstruct_GiBps": ta["reconstruct_GiBps"],
        "threads_1": t1,
        "threads_all": ta,
        "host_cpus": nall,
        "gpu_parity_matches_cpu": t1["gpu_parity_matches_cpu"] and ta["gpu_parity_matches_cpu"],
        "cpu": _cpu_model(),
        **extra,
    }


def _cpu_reference_shapes(ro_c, np, engine, seconds=1.0):
    """Single-threaded rates of BASELINE configs[0] (one 64 KiB block, 32:32, S = 2 KiB:
    encode + reconstruct of 16 erased data shreds) and of benches/shredder.rs's slice
    (/root/reference/benches/shredder.rs:19-61: a maximum 32 767-byte payload -> 32 data
    shreds of 1 KiB; deshred from the 32 coding shreds only), RS work only."""
    out = {}
    rng = np.random.default_rng(5)
    for name, S, erased in (("config0_64KiB_block", 2048, 16), ("shredder_bench_slice", 1024, 32)):
        data = rng.integers(0, 256, size=(1, 32, S), dtype=np.uint8)
        op = np.array([0] * erased + [1] * (32 - erased), np.uint8)
        rp = np.ones(32, np.uint8)
        n, te, td = 0, 0.0, 0.0
        while te + td < seconds:
            t = time.perf_counter()
            rec = ro_c.encode_blocks(data, 32, threads=1, engine=engine)
            te += time.perf_counter() - t
            cwh = np.concatenate([data, rec], axis=1)
            t = time.perf_counter()
            ro_c.decode_blocks(cwh, 32, op, rp, threads=1, engine=engine)
            td += time.perf_counter() - t
            n += 1
        out[name] = {"calls": n, "encode_us": te / n * 1e6, "reconstruct_us": td / n * 1e6,
                     "encode_plus_reconstruct_GiBps": n * 32 * S / (te + td) / GIB, "threads": 1,
                     "erased_data_shreds": erased}
    return out


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _pcie_line(per: list) -> dict:
    """The `pcie_inclusive` sub-line: one rank's dict at N = 1; at N > 1 every rank's dict
    (`per_rank`, with the NUMA node each chose) and the job's aggregate rates (bytes of all
    ranks over the slowest rank's time; the ranks ran concurrently between barriers)."""
    if len(per) == 1:
        return per[0]
    out = {"per_rank": per, "n_ranks": len(per)}
    if all(p.get("bytes") for p in per):
        tot = sum(p["bytes"] for p in per)
        out["encode_GiBps"] = tot / max(p["encode_s"] for p in per) / GIB
        out["reconstruct_GiBps"] = tot / max(p["reconstruct_s"] for p in per) / GIB
        out["encode_plus_reconstruct_GiBps"] = tot / max(p["encode_s"] + p["reconstruct_s"] for p in per) / GIB
    out["matches_device_result"] = all(p.get("matches_device_result") for p in per)
    return out


def _pcie(args, ctx, cw, k, m, S, e, torch, dev, barrier, numa):
    """Host-buffer (PCIe-inclusive) rate: blocks start and end in pinned host memory; the
    library pipelines H2D / kernels / D2H over two staging slots.  Also reports the raw
    pinned-copy rates of the same bytes for context.  The caller bound this rank to its GPU's
    NUMA node first (`numa`), so the pinned buffers allocated and touched here sit on that
    node (reported as `numa.staging_node`); the timed runs start after a barrier, so at N > 1
    the ranks' transfers overlap as they would in service."""
    from alpenglow_amd import rs
    from alpenglow_amd.shard import pages_numa_node

    nb = min(cw.shape[0], args.pcie_blocks)
    stride = (k + m) * S
    host = torch.empty((nb, stride), dtype=torch.uint8, pin_memory=True)
    host.copy_(cw[:nb])
    torch.cuda.synchronize()
    ref = host.clone()
    opres = [0] * e + [1] * (k - e)
    rpres = [0] * args.lose_coding + [1] * (m - args.lose_coding)

    def run():
        t = time.perf_counter()
        rs.encode_batch(ctx, k, m, S, nb, host.data_ptr(), stride, host.data_ptr() + k * S, stride,
                        memory=rs.MEM_HOST)
        te = time.perf_counter() - t
        host.view(nb, k + m, S)[:, :e].zero_()
        t = time.perf_counter()
        rs.decode_batch(ctx, k, m, S, nb, host.data_ptr(), stride, host.data_ptr() + k * S, stride, opres,
                        rpres, mode=rs.DECODE_ANY_K, memory=rs.MEM_HOST)
        td = time.perf_counter() - t
        return te, td

    numa = dict(numa, staging_node=pages_numa_node(host.data_ptr(), host.numel()))
    run()  # warm-up: staging buffers, streams
    barrier()
    te, td = run()
    barrier()
    ok = bool(torch.equal(host, ref))
    # raw pinned copies of one batch's data bytes (contiguous), each direction alone
    dbuf = torch.empty((nb, k * S), dtype=torch.uint8, device=dev)
    src = torch.empty((nb, k * S), dtype=torch.uint8, pin_memory=True)
    dbuf.copy_(src, non_blocking=True)  # warm
    barrier()
    t = time.perf_counter()
    dbuf.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    th = time.perf_counter() - t
    t = time.perf_counter()
    src.copy_(dbuf, non_blocking=True)
    torch.cuda.synchronize()
    tdn = time.perf_counter() - t
    B = k * S
    return {"blocks": nb, "bytes": nb * B, "encode_s": te, "reconstruct_s": td, "numa": numa,
            "encode_GiBps": nb * B / te / GIB, "reconstruct_GiBps": nb * B / td / GIB,
            "encode_plus_reconstruct_GiBps": nb * B / (te + td) / GIB, "matches_device_result": ok,
            "pinned_h2d_GBps": nb * B / th / 1e9, "pinned_d2h_GBps": nb * B / tdn / 1e9,
            "note": "host buffers pinned; encode moves k*S up and m*S down per block, reconstruct "
                    "moves the recovery shards up and the erased shards down"}


if __name__ == "__main__":
    main()
