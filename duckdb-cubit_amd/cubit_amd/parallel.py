"""Row-range partitioning across GPUs and the one exchange step of the path.

SURVEY.md §8e: bitmap segments partition by row range (every bitvector, visibility mask and
probe column is split identically), so evaluation and decode need no communication; local
row ids + partition base = global row ids, already globally ordered by rank. The only
exchange is the optional concatenation of per-partition row ids at one rank — counts by
all_gather, then a gather of the variable-length row-id arrays by point-to-point
send/recv (RCCL over xGMI with the "nccl" backend, gloo on the CPU).
The reference has no analogue (DuckDB is single-process; its threads append to a shared
sink, row_group_collection.cpp:174-224).
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


def gather_rowids(local, dst: int = 0, group=None) -> Optional[object]:
    """Concatenate every rank's 1-D int64 tensor at rank `dst` in rank order (None elsewhere).

    Counts go by all_gather (one 8-byte value per rank); payloads by batched isend/irecv,
    so each partition crosses the fabric once (root ingress bound: 7 xGMI links)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    sizes: List[int] = [int(c.item()) for c in counts]
    if rank == dst:
        out = torch.empty(sum(sizes), dtype=local.dtype, device=local.device)
        ops, off = [], 0
        for r in range(world):
            if r == dst:
                out[off: off + sizes[r]].copy_(local)
            elif sizes[r]:
                ops.append(dist.P2POp(dist.irecv, out[off: off + sizes[r]], r, group=group))
            off += sizes[r]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return out
    if sizes[rank]:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, local, dst, group=group)]):
            w.wait()
    return None
