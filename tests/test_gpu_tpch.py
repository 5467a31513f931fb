"""GPU: TPC-H-shaped Q3 against a pandas restatement of the
query on the same generated tables (test infrastructure; the official answer set needs
dbgen's data, which cannot be generated here)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def q3_pandas(customer, orders, lineitem, seg, d, limit=10):
    c = customer[customer.c_mktsegment == seg]
    o = orders[orders.o_orderdate < d]
    li = lineitem[lineitem.l_shipdate > d]
    co = c.merge(o, left_on="c_custkey", right_on="o_custkey")
    col = co.merge(li, left_on="o_orderkey", right_on="l_orderkey")
    col = col.assign(revenue=col.l_extendedprice.astype(np.int64) * (100 - col.l_discount.astype(np.int64)))
    g = col.groupby(["l_orderkey", "o_orderdate", "o_shippriority"], as_index=False)["revenue"].sum()
    g = g.sort_values(["revenue", "o_orderdate"], ascending=[False, True], kind="mergesort")
    return g.head(limit), len(g)


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


def q9_pandas(orders, lineitem, part, supplier, partsupp):
    import pandas as pd
    from datafusion_parallelism_amd import tpch

    p = part[part.p_green]
    x = lineitem.merge(p, left_on="l_partkey", right_on="p_partkey")
    x = x.merge(partsupp, left_on=["l_partkey", "l_suppkey"], right_on=["ps_partkey", "ps_suppkey"])
    x = x.merge(supplier, left_on="l_suppkey", right_on="s_suppkey")
    x = x.merge(orders, left_on="l_orderkey", right_on="o_orderkey")
    dates = pd.to_datetime("1992-01-01") + pd.to_timedelta(x.o_orderdate, unit="D")
    x = x.assign(o_year=dates.dt.year,
                 amount=x.l_extendedprice.astype(np.int64) * (100 - x.l_discount.astype(np.int64))
                 - x.ps_supplycost.astype(np.int64) * x.l_quantity.astype(np.int64) * 100,
                 nation=[tpch.NATIONS[k] for k in x.s_nationkey])
    g = x.groupby(["nation", "o_year"], as_index=False)["amount"].sum()
    g = g.sort_values(["nation", "o_year"], ascending=[True, False], kind="mergesort")
    return [(r.nation, int(r.o_year), int(r.amount)) for r in g.itertuples()]


@pytest.mark.parametrize("sf", [0.01, 0.05])
def test_q9_matches_pandas(dfp, sf):
    from datafusion_parallelism_amd import tpch

    t = tpch.generate(sf, "cuda:0", seed=5, q9=True)
    got = tpch.q9(t)
    _, orders, lineitem, part, supplier, partsupp = t.to_pandas()
    want = q9_pandas(orders, lineitem, part, supplier, partsupp)
    assert len(got) > 0 and got == want
