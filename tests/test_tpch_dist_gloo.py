"""CPU, world_size 2 and 8 (gloo; 8 = C4/C5's GPU count): the multi-GPU TPC-H plans (tpch.q3_dist / q9_dist: broadcast
of filtered dimension sides, hash-repartition shuffles with payload, all-reduce / top-k
merges) on rank-sharded generated tables, with the oracle as the per-rank local join and a
numpy restatement of the partition (test-local stand-ins for the HIP kernels). Results
must equal the pandas restatement over the whole (concatenated) tables."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rendezvous

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))


def oracle_join(build, probe):
    import oracle

    b, p = oracle.inner_join(build.numpy(), probe.numpy())
    return torch.from_numpy(b.astype(np.int64)), torch.from_numpy(p.astype(np.int64))


def _worker(rank, world, port, sf, q, max_bytes=None):
    sys.path[:0] = [ROOT, HERE, os.path.join(ROOT, "oracle")]
    rendezvous.join(rank, world, port)
    from test_distributed_gloo import cpu_partition

    from datafusion_parallelism_amd import distributed, tpch

    if max_bytes:  # force the multi-round exchange path
        distributed.A2A_MAX_BYTES = max_bytes

    t = tpch.generate(sf, "cpu", seed=7, q9=True, rank=rank, world=world)
    r3 = tpch.q3_dist(t, "BUILDING", "1995-03-15", group=None, join_fn=oracle_join, partition_fn=cpu_partition)
    r9 = tpch.q9_dist(t, join_fn=oracle_join, partition_fn=cpu_partition)
    res = (r3.l_orderkey, r3.revenue, r3.o_orderdate, r3.o_shippriority, r3.groups, r9)
    allres = [None] * world
    dist.all_gather_object(allres, res)
    if rank == 0:
        q.put(allres)
    dist.destroy_process_group()



def test_generator_shards_concatenate_to_the_whole_tables():
    from datafusion_parallelism_amd import tpch

    whole = tpch.generate(0.01, "cpu", seed=7, q9=True)
    shards = [tpch.generate(0.01, "cpu", seed=7, q9=True, rank=r, world=3) for r in range(3)]
    for f in ("c_custkey", "c_mktsegment", "o_orderkey", "o_custkey", "o_orderdate", "l_orderkey",
              "l_extendedprice", "l_discount", "l_shipdate", "l_partkey", "l_suppkey", "l_quantity", "p_partkey",
              "p_green", "s_suppkey", "s_nationkey", "ps_partkey", "ps_suppkey", "ps_supplycost"):
        assert torch.equal(torch.cat([getattr(s, f) for s in shards]), getattr(whole, f)), f


def test_generator_shape_cpu():
    """Key structure of the spec: sparse order keys, customers with orders, 1-7 lines,
    4 suppliers per part, lineitem (part, supplier) pairs present in partsupp."""
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(0.01, "cpu", q9=True)
    ok = t.o_orderkey.numpy()
    assert len(ok) == 15000 and ok[0] == 1 and ok[8] == 33 and len(np.unique(ok)) == len(ok)
    assert (t.o_custkey.numpy() % 3 != 0).all()
    n = len(t.l_orderkey)
    assert abs(n / 15000 - 4.0) < 0.2
    ps = set(zip(t.ps_partkey.tolist(), t.ps_suppkey.tolist()))
    assert len(ps) == 4 * len(t.p_partkey)
    assert all((a, b) in ps for a, b in zip(t.l_partkey[:2000].tolist(), t.l_suppkey[:2000].tolist()))


@pytest.mark.parametrize("world,max_bytes", [(2, None), (2, 20000), (8, None)])
def test_q3_q9_distributed_match_pandas(oracle_mod, world, max_bytes):
    from tpch_ref import frames, q3_pandas, q9_pandas

    from datafusion_parallelism_amd import tpch

    sf = 0.01
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = rendezvous.parent_store()  # held until the ranks exit
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, world, port, sf, q, max_bytes)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(r == res[0] for r in res), "ranks disagree"
    okeys, rev, odate, osp, groups, r9 = res[0]
    shards = [tpch.generate(sf, "cpu", seed=7, q9=True, rank=r, world=world) for r in range(world)]
    customer, orders, lineitem, part, supplier, partsupp = frames(shards)
    want, ngroups = q3_pandas(customer, orders, lineitem, tpch.SEGMENTS.index("BUILDING"), tpch.day("1995-03-15"))
    assert groups == ngroups
    assert okeys == want.l_orderkey.tolist() and rev == want.revenue.tolist()
    assert odate == want.o_orderdate.tolist() and osp == want.o_shippriority.tolist()
    want9 = q9_pandas(orders, lineitem, part, supplier, partsupp)
    assert len(r9) > 0 and r9 == want9
