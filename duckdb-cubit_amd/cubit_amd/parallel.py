"""Row-range partitioning across GPUs and the one exchange step of the path.

SURVEY.md §8e: bitmap segments partition by row range (every bitvector, visibility mask and
probe column is split identically), so evaluation and decode need no communication; local
row ids + partition base = global row ids, already globally ordered by rank. The only
exchange is the optional concatenation of per-partition row ids at one rank (RCCL over xGMI
with the "nccl" backend, gloo on the CPU).
The reference has no analogue (DuckDB is single-process; its threads share one morsel cursor
over the row groups of one table, row_group_collection.cpp:174-224 — the same split of one
table into row ranges that `partition_orders` / `partition_range` make across ranks).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

ROW_GROUP = 122880  # STANDARD_ROW_GROUPS_SIZE (storage_info.hpp:20)


def partition_range(total: int, rank: int, world: int, align: int = 1) -> Tuple[int, int]:
    """[begin, end) of `rank`'s share of `total` units, boundaries on multiples of `align`
    (row groups keep every partition word-aligned: 122,880 = 1,920 bitvector words)."""
    units = (total + align - 1) // align
    b = units * rank // world * align
    e = units * (rank + 1) // world * align
    return min(b, total), min(e, total)


def partition_orders(total_orders: int, rank: int, world: int) -> Tuple[int, int]:
    """TPC-H lineitem partitions follow order boundaries (all lines of an order stay
    together, rows stay in dbgen's row-id order)."""
    return partition_range(total_orders, rank, world)


class RowIdExchange:
    """Concatenation of every rank's row ids at rank `dst` with no host synchronisation on
    the data path (SURVEY §8e's exchange step).

    Each rank's ids are sent as one fixed-size slot of `slot` elements (its buffer's first
    `slot` ids; the ones past its count are padding), so the point-to-point sizes are known
    on the host before any count is: the counts travel beside the payload (an all_gather of
    one 8-byte value per rank into a preallocated tensor), every call is asynchronous on the
    stream, and the counts are read once, when the caller asks for the result. `slot` must be
    at least every rank's count; `result()` checks that from the gathered counts and raises
    otherwise (the caller then re-posts with a larger slot). The root's own ids stay where its
    scan wrote them; the result is the list of runs in rank order, as the decode's tile runs
    with their directory.

    RCCL send/recv sizes must match on both sides, so a slot is the smallest unit the root
    can receive without first learning the count; with a slot from the previous query's
    counts (or the planner's estimate) the padding is a few per cent of the payload."""

    def __init__(self, slot: int, device=None, dst: int = 0, group=None, dtype=None):
        import torch
        import torch.distributed as dist

        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst = dst
        self.group = group
        self.slot = int(slot)
        dtype = dtype or torch.int64
        self.counts = torch.zeros(self.world, dtype=torch.int64, device=device)
        self._count_views = list(torch.split(self.counts, 1))
        self._nccl = dist.get_backend(group) == "nccl"
        self.recv = None
        if self.rank == dst:
            # exactly `slot` per rank: a recv larger than the matching send never completes on
            # RCCL (and is a size mismatch on gloo)
            self.recv = torch.empty((self.world, self.slot), dtype=dtype, device=device)
        self._local = None
        self._works = []

    def post(self, local, count) -> None:
        """Start the exchange of `local[:count]` (`count`: a 1-element int64 tensor on the
        same device, e.g. the scan's device count). Returns without waiting."""
        import torch.distributed as dist

        if local.numel() < self.slot:
            raise ValueError(f"row-id buffer of {local.numel()} < slot {self.slot}")
        self.wait()
        self._local = local
        mine = count.reshape(-1)[:1]
        if self._nccl:
            dist.all_gather_into_tensor(self.counts, mine, group=self.group)  # one collective, no copies
        else:
            dist.all_gather(self._count_views, mine, group=self.group)
        if self.world == 1 or self.slot == 0:
            return  # every rank has the same slot, so all of them skip the payload together
        if self.rank == self.dst:
            ops = [dist.P2POp(dist.irecv, self.recv[r], r, group=self.group)
                   for r in range(self.world) if r != self.dst]
        else:
            ops = [dist.P2POp(dist.isend, local[: self.slot], self.dst, group=self.group)]
        self._works = dist.batch_isend_irecv(ops)

    def wait(self) -> None:
        for w in self._works:
            w.wait()
        self._works = []

    def sizes(self) -> List[int]:
        """The gathered counts (one device → host read)."""
        self.wait()
        return [int(x) for x in self.counts.cpu().tolist()]

    def runs(self) -> Optional[list]:
        """Rank-ordered list of (tensor, count) runs at the root (None elsewhere)."""
        sizes = self.sizes()
        over = [(r, c) for r, c in enumerate(sizes) if c > self.slot]
        if over:
            raise RuntimeError(f"row counts {over} exceed the exchange slot of {self.slot}")
        if self.rank != self.dst:
            return None
        return [(self._local if r == self.dst else self.recv[r], c) for r, c in enumerate(sizes)]

    def result(self):
        """The concatenation at the root (None elsewhere)."""
        import torch

        runs = self.runs()
        if runs is None:
            return None
        return torch.cat([t[:c] for t, c in runs])


def gather_rowids(local, dst: int = 0, group=None) -> Optional[object]:
    """Concatenate every rank's 1-D int64 tensor at rank `dst` in rank order (None elsewhere),
    exact sizes: one all_reduce(MAX) of the counts sizes the slot, then one RowIdExchange."""
    import torch
    import torch.distributed as dist

    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    m = n.clone()
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    slot = int(m.item())
    if local.numel() < slot:
        padded = torch.empty(slot, dtype=local.dtype, device=local.device)
        padded[: local.numel()] = local
        local = padded
    ex = RowIdExchange(slot, device=local.device, dst=dst, group=group, dtype=local.dtype)
    ex.post(local, n)
    return ex.result()
