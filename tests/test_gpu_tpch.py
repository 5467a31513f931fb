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
