"""Multi-GPU sharding of independent blocks.

Blocks (and slices) are independent Reed-Solomon codeword sets, so a stream of blocks
splits into contiguous per-rank ranges with no data-path collective.  The only
collectives are timing ones: a barrier and a max-over-ranks reduction.
"""

from __future__ import annotations


def block_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous [start, end) share of ``total`` blocks for ``rank`` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of ``value`` over all ranks (the bench's wall-time reduction)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
