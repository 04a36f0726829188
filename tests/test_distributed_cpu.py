"""The multi-GPU path's partitioning and its one exchange step, on CPU with gloo
(world_size 2): per-rank partitions of a TPC-H lineitem table, per-partition Q6 row ids
(oracle, global ids), concatenated at rank 0 == the whole-table result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cubit_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sf, result_path):
    import sys

    from conftest import ROOT

    for p in (str(ROOT / "duckdb-cubit_amd"), str(ROOT)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from cubit_amd import datagen
    from cubit_amd import filters as F
    from cubit_amd import parallel as P
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ob, oe = P.partition_orders(datagen.tpch_orders(sf), rank, world)
        li = datagen.tpch_lineitem(sf, ob, oe)
        cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)]
        local = O.table_scan(cols, F.serialize(F.q6_filter_set()), li.n_rows, li.row_base)
        out = P.gather_rowids(torch.from_numpy(local), dst=0)
        # the bench's form: fixed-size slots posted without reading any count on the host,
        # the counts gathered beside them and read once at the end; a buffer larger than its
        # count (as the scan's capacity-sized row-id buffer) and a few repeated posts
        q = torch.tensor([len(local)], dtype=torch.int64)
        qmax = q.clone()
        dist.all_reduce(qmax, op=dist.ReduceOp.MAX)
        buf = torch.full((int(qmax.item()) + 100,), -1, dtype=torch.int64)
        buf[: len(local)] = torch.from_numpy(local)
        ex = P.RowIdExchange(int(qmax.item()) + 7)
        for _ in range(3):
            ex.post(buf, torch.tensor([len(local), 0], dtype=torch.int64))
        slots = ex.result()
        # a slot below some rank's count is refused on every rank
        small = P.RowIdExchange(1)
        small.post(buf, q)
        refused = False
        try:
            small.runs()
        except RuntimeError:
            refused = True
        if rank == 0:
            np.save(result_path, out.numpy())
            np.save(str(result_path) + ".slots.npy", slots.numpy())
            np.save(str(result_path) + ".refused.npy", np.array([refused]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_partitioned_q6_gathers_to_whole_table_result(tmp_path, world, li01):
    from cubit_amd import filters as F
    from oracle import oracle as O

    res = tmp_path / "rows.npy"
    mp.spawn(_worker, args=(world, _free_port(), 0.1, str(res)), nprocs=world, join=True)
    got = np.load(res)
    ref = O.table_scan([O.Column(li01.l_shipdate), O.Column(li01.l_discount), O.Column(li01.l_quantity)],
                       F.serialize(F.q6_filter_set()), li01.n_rows)
    assert np.array_equal(got, ref)
    assert np.array_equal(np.load(str(res) + ".slots.npy"), ref)
    assert bool(np.load(str(res) + ".refused.npy")[0])


def test_partition_range_alignment_and_cover():
    n = 10_000_019
    parts = [parallel.partition_range(n, r, 8, parallel.ROW_GROUP) for r in range(8)]
    assert parts[0][0] == 0 and parts[-1][1] == n
    for (b0, e0), (b1, e1) in zip(parts, parts[1:]):
        assert e0 == b1
        assert b1 % parallel.ROW_GROUP == 0 and b1 % 64 == 0
    sizes = [e - b for b, e in parts]
    assert max(sizes) - min(sizes) <= 2 * parallel.ROW_GROUP


def _empty_worker(rank, world, port, result_path):
    import sys

    from conftest import ROOT

    for p in (str(ROOT / "duckdb-cubit_amd"), str(ROOT)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from cubit_amd import parallel as P

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every rank's filter keeps nothing: slot 0, no point-to-point op may be posted
        none = P.gather_rowids(torch.empty(0, dtype=torch.int64), dst=0)
        ex = P.RowIdExchange(0)
        ex.post(torch.empty(0, dtype=torch.int64), torch.zeros(1, dtype=torch.int64))
        none_slots = ex.result()
        # only the last rank keeps rows (ragged: the others send padding)
        mine = torch.arange(5, dtype=torch.int64) + 100 * rank if rank == world - 1 else torch.empty(0, dtype=torch.int64)
        some = P.gather_rowids(mine, dst=0)
        if rank == 0:
            np.save(result_path, np.array([none.numel(), none_slots.numel()]))
            np.save(str(result_path) + ".some.npy", some.numpy())
        else:
            assert none is None and none_slots is None and some is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_of_empty_results(tmp_path, world):
    """when every rank's result is empty the slot is 0; the root must not post a
    1-element receive against 0-element sends (a hang on RCCL, a size mismatch on gloo)."""
    res = tmp_path / "empty.npy"
    mp.spawn(_empty_worker, args=(world, _free_port(), str(res)), nprocs=world, join=True)
    assert np.load(res).tolist() == [0, 0]
    assert np.load(str(res) + ".some.npy").tolist() == [100 * (world - 1) + i for i in range(5)]
