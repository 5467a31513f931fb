"""GPU: TPC-H-shaped Q3 against a pandas restatement of the
query on the same generated tables (test infrastructure; the official answer set needs
dbgen's data, which cannot be generated here)."""
import numpy as np
import pytest

from tpch_ref import q3_pandas, q9_pandas
from conftest import init_one_rank_nccl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sf,date", [(0.01, "1995-03-15"), (0.05, "1995-03-15"), (0.05, "1993-06-01")])
def test_q3_matches_pandas(dfp, sf, date):
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(sf, "cuda:0", seed=3)
    got = tpch.q3(t, "BUILDING", date)
    customer, orders, lineitem = t.to_pandas()
    want, ngroups = q3_pandas(customer, orders, lineitem, tpch.SEGMENTS.index("BUILDING"), tpch.day(date))
    assert got.groups == ngroups
    assert got.l_orderkey == want.l_orderkey.tolist()
    assert got.revenue == want.revenue.tolist()
    assert got.o_orderdate == want.o_orderdate.tolist()
    assert got.o_shippriority == want.o_shippriority.tolist()


def test_generator_shape(dfp):
    """Key structure of the spec: sparse order keys, customers with orders, 1-7 lines."""
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(0.01, "cuda:0")
    ok = t.o_orderkey.cpu().numpy()
    assert len(ok) == 15000 and ok[0] == 1 and ok[8] == 33 and len(np.unique(ok)) == len(ok)
    assert (t.o_custkey.cpu().numpy() % 3 != 0).all()
    n = len(t.l_orderkey)
    assert 15000 <= n <= 7 * 15000 and abs(n / 15000 - 4.0) < 0.2
    assert int(t.l_discount.max()) <= 10 and int(t.o_orderdate.max()) <= tpch.ORDERDATE_MAX


@pytest.mark.parametrize("sf", [0.01, 0.05])
def test_q9_matches_pandas(dfp, sf):
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(sf, "cuda:0", seed=5, q9=True)
    got = tpch.q9(t)
    _, orders, lineitem, part, supplier, partsupp = t.to_pandas()
    want = q9_pandas(orders, lineitem, part, supplier, partsupp)
    assert len(got) > 0 and got == want


def test_distributed_plans_one_rank(dfp):
    """q3_dist / q9_dist through RCCL with one rank (broadcasts and shuffles are
    self-copies; the GPU partition kernel and hash joins run for real): equal to the
    one-GPU plans and to pandas."""
    import os

    import torch
    import torch.distributed as dist

    from datafusion_parallelism_amd import tpch

    init_one_rank_nccl()
    try:
        t = tpch.generate(0.05, "cuda:0", seed=11, q9=True)
        got3 = tpch.q3_dist(t, "BUILDING", "1995-03-15")
        one3 = tpch.q3(t, "BUILDING", "1995-03-15")
        assert got3 == one3
        got9 = tpch.q9_dist(t)
        assert got9 == tpch.q9(t)
        _, orders, lineitem, part, supplier, partsupp = t.to_pandas()
        assert got9 == q9_pandas(orders, lineitem, part, supplier, partsupp)
        # the same plans with every local join on an 8-shard radix table
        j = tpch.multi_join([0] * 8, "radix")
        assert tpch.q3_dist(t, "BUILDING", "1995-03-15", join_fn=j) == one3
        assert tpch.q9_dist(t, join_fn=j) == got9
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("plan", ["radix", "broadcast"])
def test_q3_q9_eight_shards_match_pandas(dfp, plan):
    """C4/C5's sharded joins in process: every join of Q3 and Q9 runs on a table sharded
    over 8 GPUs (hj_build_begin_multi with devices [0] * 8 on this one-GPU box: the radix
    plan gives each shard 1/8 of the build side by key hash and merges the shards' pairs;
    the broadcast plan splits the probe rows), at SF 1, against pandas."""
    from tpch_ref import q3_pandas

    from datafusion_parallelism_amd import tpch

    t = tpch.generate(1, "cuda:0", seed=13, q9=True)
    j = tpch.multi_join([0] * 8, plan)
    got3 = tpch.q3(t, "BUILDING", "1995-03-15", join_fn=j)
    customer, orders, lineitem, part, supplier, partsupp = t.to_pandas()
    want, ngroups = q3_pandas(customer, orders, lineitem, tpch.SEGMENTS.index("BUILDING"), tpch.day("1995-03-15"))
    assert got3.groups == ngroups
    assert got3.l_orderkey == want.l_orderkey.tolist() and got3.revenue == want.revenue.tolist()
    assert got3.o_orderdate == want.o_orderdate.tolist() and got3.o_shippriority == want.o_shippriority.tolist()
    got9 = tpch.q9(t, join_fn=j)
    assert len(got9) > 0 and got9 == q9_pandas(orders, lineitem, part, supplier, partsupp)


@pytest.fixture
def budget():
    from datafusion_parallelism_amd.table import set_device_budget

    old = set_device_budget(0)
    yield set_device_budget
    set_device_budget(old)


def test_device_budget_refuses_one_gpu_build(dfp, budget):
    """hj_set_device_budget: a one-device build above the budget raises HJ_ERR_OOM
    ("device budget"), the same build on an 8-shard radix table fits (each shard about
    1/8 of it) and gives the one-GPU pairs."""
    import torch

    from datafusion_parallelism_amd import HashTable
    from datafusion_parallelism_amd._lib import HjError
    from datafusion_parallelism_amd.table import is_budget_error

    g = torch.Generator(device="cuda").manual_seed(5)
    bk = torch.randint(-(2**62), 2**62, (2_000_000,), device="cuda", generator=g)
    pk = torch.cat([bk[::3], torch.randint(-(2**62), 2**62, (500_000,), device="cuda", generator=g)])
    with HashTable(1, "int64", 0) as t:
        t.build(bk)
        peak = t.device_bytes()
        b1, p1 = t.probe(pk, device_output=True)
    assert peak > 0
    budget(peak // 2)
    with pytest.raises(HjError) as ei:
        with HashTable(1, "int64", 0) as t:
            t.build(bk)
    assert is_budget_error(ei.value)
    with HashTable(1, "int64", devices=[0] * 8, plan="radix") as t:
        t.append(0, bk)
        t.finish(0)
        assert 0 < t.device_bytes() <= peak // 2
        b8, p8 = t.probe(pk, device_output=True)
    assert torch.equal(b1, b8) and torch.equal(p1, p8)


@pytest.mark.parametrize("sf", [1, 10])
def test_q9_device_budget_takes_sharded_build(dfp, budget, sf):
    """C5's premise at a smaller scale: with a device budget below Q9's partsupp and orders
    builds, those joins refuse the one-GPU table and take the 8-shard radix build (the
    small builds stay on one GPU); the answer equals the unbudgeted one-GPU plan (and
    pandas at SF 1)."""
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(sf, "cuda:0", seed=17, q9=True)
    free = tpch.planned_join([0] * 8)
    one9 = tpch.q9(t, join_fn=free)
    assert [p for _, p, _ in free.log] == ["one-gpu"] * 4
    rows = [n for n, _, _ in free.log]
    peaks = [b for _, _, b in free.log]
    # the joins in q9's order: green parts, partsupp, supplier, orders
    big = min(peaks[1], peaks[3])
    assert big > max(peaks[0], peaks[2])
    budget(big - 1)
    j = tpch.planned_join([0] * 8)
    got9 = tpch.q9(t, join_fn=j)
    assert got9 == one9 and len(got9) > 0
    assert [p for _, p, _ in j.log] == ["one-gpu", "radix", "one-gpu", "radix"], j.log
    assert [n for n, _, _ in j.log] == rows
    assert all(b <= big - 1 for _, _, b in j.log)
    if sf == 1:
        _, orders, lineitem, part, supplier, partsupp = t.to_pandas()
        assert got9 == q9_pandas(orders, lineitem, part, supplier, partsupp)


def test_q9_sf300_eight_shards_equal_one_gpu(dfp):
    """C5 as configured (BASELINE configs[4]: Q9 at SF300, build sides sharded over 8 GPUs),
    in process on this one GPU: every join on an 8-shard radix table equals the one-GPU
    plan (full-size property; pandas cannot hold SF300)."""
    import torch

    from datafusion_parallelism_amd import tpch

    t = tpch.generate(300, "cuda:0", seed=1, q9=True)
    one9 = tpch.q9(t)
    assert len(one9) == 25 * 7
    torch.cuda.empty_cache()  # the one-GPU plan's freed blocks back to the device for the shards
    assert tpch.q9(t, join_fn=tpch.multi_join([0] * 8, "radix")) == one9
    del t
    torch.cuda.empty_cache()


def test_q3_q9_eight_shards_sf100_equal_one_gpu(dfp):
    """Full size (C4 = Q3 SF100, C5's query Q9 at SF100): the 8-shard radix plans equal the
    one-GPU plans (size-independent property; pandas cannot hold SF100 here)."""
    import torch

    from datafusion_parallelism_amd import tpch

    j = tpch.multi_join([0] * 8, "radix")
    t = tpch.generate(100, "cuda:0", seed=1, q9=True)
    one3 = tpch.q3(t, "BUILDING", "1995-03-15")
    assert one3.groups > 0
    assert tpch.q3(t, "BUILDING", "1995-03-15", join_fn=j) == one3
    one9 = tpch.q9(t)
    assert len(one9) == 25 * 7
    assert tpch.q9(t, join_fn=j) == one9
    del t
    torch.cuda.empty_cache()
