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


def gather_over_ranks(value: float, dist=None, device=None) -> list:
    """``value`` of every rank, in rank order (the bench's per-rank wall times)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [value]
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def verify_over_ranks(ok, dist=None, device=None) -> list:
    """Every rank's verification verdict, in rank order: True (verified), False (a check
    failed) or None (not verified).  All ranks receive the whole list, so each can exit
    non-zero when any rank failed (bench.py: a wrong result on GPU 5 must not exit 0)."""
    code = -1.0 if ok is None else (1.0 if ok else 0.0)
    flags = gather_over_ranks(code, dist, device)
    return [None if f < 0 else bool(f) for f in flags]


# ---- the bench's per-rank plan (bench.py; tested under gloo in tests/test_dist.py) ----

SEED_BASE = 0x5EED_A19E_0000_0000  # block b is seeded SEED_BASE + b


class RankPlan:
    """Which blocks of the global stream one rank owns and what it reports.

    weak scaling   (``stream_blocks == 0``): every rank owns ``nblocks`` blocks, rank r the
                   global blocks [r * nblocks, (r + 1) * nblocks);
    strong scaling (``stream_blocks > 0``):  one stream of ``stream_blocks`` blocks split
                   into contiguous ranges (``block_range``).
    Block g of the stream is generated from seed ``SEED_BASE + g`` on whichever rank owns
    it, so the ranks' blocks are disjoint parts of one stream."""

    def __init__(self, rank: int, world: int, nblocks: int, stream_blocks: int = 0):
        if world <= 0 or not 0 <= rank < world:
            raise ValueError("bad rank/world")
        self.rank, self.world = rank, world
        if stream_blocks:
            self.first, last = block_range(rank, world, stream_blocks)
            self.nblocks = last - self.first
            self.total = stream_blocks
            self.scaling = "strong"
        else:
            self.first, self.nblocks = rank * nblocks, nblocks
            self.total = world * nblocks
            self.scaling = "weak"

    @property
    def seed_base(self) -> int:
        return SEED_BASE + self.first

    def processed_bytes(self, block_bytes: int, steps: int) -> int:
        """Block payload bytes that went through the timed steps on all ranks together."""
        return self.total * block_bytes * steps


def erasure_patterns(plan: RankPlan, k: int, m: int, erased: int, lost_coding: int, random_patterns: bool):
    """Per-block presence flags (opres: k per block, rpres: m per block) for the blocks of
    ``plan``; one shared pattern (the first ``erased`` data and ``lost_coding`` coding
    shreds lost) unless ``random_patterns``.  Random patterns are a function of the global
    block index only, so they do not depend on the world size."""
    if not random_patterns:
        return [0] * erased + [1] * (k - erased), [0] * lost_coding + [1] * (m - lost_coding)
    import random

    opres, rpres = [], []
    for g in range(plan.first, plan.first + plan.nblocks):
        rng = random.Random(0xA1_0000_0000 + g)
        lost, lost_r = set(rng.sample(range(k), erased)), set(rng.sample(range(m), lost_coding))
        opres += [0 if i in lost else 1 for i in range(k)]
        rpres += [0 if j in lost_r else 1 for j in range(m)]
    return opres, rpres


def gather_objects(obj, dist=None) -> list:
    """``obj`` (any picklable value) of every rank, in rank order (per-rank sub-lines)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


# ---- NUMA placement of a rank's host staging (blocks arrive from the
# disseminator in host memory, disseminator/rotor.rs:108-112, network/udp.rs:9-12) ----------

def _sysfs_root() -> str:
    import os

    return os.environ.get("AG_SYSFS_ROOT", "/sys")


def parse_cpulist(text: str) -> set:
    """The kernel's cpulist format ("0-3,8,10-11") as a set of CPU ids."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def gpu_bdf(device_index: int):
    """PCI address (domain:bus:device.function) of torch device ``device_index``, or None."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return None


def pci_numa_node(bdf, sysfs=None) -> int:
    """NUMA node of PCI device ``bdf`` from /sys/bus/pci/devices/<bdf>/numa_node (-1: unknown
    or a single-node host)."""
    import os

    if not bdf:
        return -1
    try:
        return int(open(os.path.join(sysfs or _sysfs_root(), "bus/pci/devices", bdf, "numa_node")).read())
    except (OSError, ValueError):
        return -1


def node_cpus(node: int, sysfs=None) -> set:
    import os

    if node < 0:
        return set()
    try:
        return parse_cpulist(open(os.path.join(sysfs or _sysfs_root(), f"devices/system/node/node{node}/cpulist")).read())
    except OSError:
        return set()


def bind_to_gpu_node(bdf, sysfs=None) -> dict:
    """Bind this rank's host threads to the CPUs of its GPU's NUMA node (intersected with the
    CPUs the process may use), so that host staging it allocates and touches afterwards is
    placed on that node (first-touch, the default local policy) and its copies do not cross
    the socket link.  Returns what was chosen (reported per rank in the bench line)."""
    import os

    node = pci_numa_node(bdf, sysfs)
    allowed = os.sched_getaffinity(0)
    cpus = node_cpus(node, sysfs) & allowed
    bound = bool(cpus) and cpus != allowed
    if bound:
        os.sched_setaffinity(0, cpus)
    return {"bdf": bdf, "numa_node": node, "cpus": len(cpus) if cpus else len(allowed), "bound": bound}


def pages_numa_node(ptr: int, nbytes: int, samples: int = 16) -> int:
    """NUMA node holding the pages of host range [ptr, ptr + nbytes) (the node of most sampled
    pages, via move_pages(2) with no target nodes: a query), or -1 when it cannot be told."""
    import collections
    import ctypes
    import os
    import platform

    if nbytes <= 0 or platform.machine() != "x86_64":
        return -1
    page = os.sysconf("SC_PAGE_SIZE")
    first = ptr // page * page
    npages = (ptr + nbytes - first + page - 1) // page
    k = max(1, min(samples, npages))
    addrs = (ctypes.c_void_p * k)(*[first + (i * npages // k) * page for i in range(k)])
    status = (ctypes.c_int * k)()
    libc = ctypes.CDLL(None, use_errno=True)
    libc.syscall.restype = ctypes.c_long
    SYS_move_pages = 279  # x86_64
    if libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(k), addrs, None, status, 0) != 0:
        return -1
    nodes = [s for s in status if s >= 0]
    return collections.Counter(nodes).most_common(1)[0][0] if nodes else -1
