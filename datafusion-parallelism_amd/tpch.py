"""TPC-H-shaped tables and Q3 on the GPU join (BASELINE.json
configs[3]: TPC-H Q3, lineitem ⋈ orders ⋈ customer).

There is no network for dbgen / tpchgen-cli, so `generate` builds the three tables Q3
reads on the device from a counter-based generator (splitmix64, `hj_gen_uniform_keys`),
following the TPC-H specification's key structure and value domains: SF·150,000
customers, 5 market segments; SF·1,500,000 orders with sparse order keys (8 of every 32),
customer keys drawn from the 2/3 of customers that have orders, order dates in
[1992-01-01, 1998-08-02]; 1-7 lineitems per order, ship date = order date + [1, 121]
days, quantity 1-50, discount 0.00-0.10, extended price = quantity x the part's retail
price (spec formula). The values differ from dbgen's (other random streams), so results
are checked against a pandas restatement of the query on the same tables
(tests/test_gpu_tpch.py), not against the official answer set.

Money is fixed point (cents); revenue = extendedprice x (100 - discount%) is exact in
units of 1e-4.

Q3 (the reference's tpc/ harness runs it through DataFusion SQL):
    select l_orderkey, sum(l_extendedprice * (1 - l_discount)) as revenue,
           o_orderdate, o_shippriority
    from customer, orders, lineitem
    where c_mktsegment = 'BUILDING' and c_custkey = o_custkey and l_orderkey = o_orderkey
      and o_orderdate < date '1995-03-15' and l_shipdate > date '1995-03-15'
    group by l_orderkey, o_orderdate, o_shippriority
    order by revenue desc, o_orderdate
    limit 10
Plan: customer filter -> build; orders filter -> probe (right-semi on o_custkey) ->
build on o_orderkey; lineitem filter -> probe; per-order revenue sums; top 10. Both
joins run on the hash-join kernels; filters, the group-by sum and the top-k are torch
device ops.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import check
from .table import HashTable

SEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
EPOCH = _dt.date(1992, 1, 1)


def day(d: str | _dt.date) -> int:
    """Days since 1992-01-01."""
    if isinstance(d, str):
        d = _dt.date.fromisoformat(d)
    return (d - EPOCH).days


ORDERDATE_MAX = day("1998-08-02")  # STARTDATE .. ENDDATE - 151 days


def _uniform(n: int, seed: int, lo: int, hi: int, device) -> torch.Tensor:
    """n int64 values in [lo, hi] (splitmix64 counter stream on the device)."""
    out = torch.empty(max(n, 1), dtype=torch.int64, device=device)
    if n:
        check(_lib.load().hj_gen_uniform_keys(out.data_ptr(), n, seed, hi - lo + 1,
                                              torch.cuda.current_stream(device).cuda_stream))
    return out[:n] + lo


@dataclass
class Tables:
    sf: float
    # customer
    c_custkey: torch.Tensor
    c_mktsegment: torch.Tensor  # int8 code into SEGMENTS
    # orders
    o_orderkey: torch.Tensor
    o_custkey: torch.Tensor
    o_orderdate: torch.Tensor  # int32 days since 1992-01-01
    o_shippriority: torch.Tensor  # int32 (0, as in dbgen)
    # lineitem
    l_orderkey: torch.Tensor
    l_extendedprice: torch.Tensor  # int64 cents
    l_discount: torch.Tensor  # int32 percent 0..10
    l_shipdate: torch.Tensor  # int32 days

    @property
    def device(self):
        return self.l_orderkey.device

    def to_pandas(self):
        import pandas as pd

        def h(t):
            return t.cpu().numpy()

        customer = pd.DataFrame({"c_custkey": h(self.c_custkey), "c_mktsegment": h(self.c_mktsegment)})
        orders = pd.DataFrame({"o_orderkey": h(self.o_orderkey), "o_custkey": h(self.o_custkey),
                               "o_orderdate": h(self.o_orderdate), "o_shippriority": h(self.o_shippriority)})
        lineitem = pd.DataFrame({"l_orderkey": h(self.l_orderkey), "l_extendedprice": h(self.l_extendedprice),
                                 "l_discount": h(self.l_discount), "l_shipdate": h(self.l_shipdate)})
        return customer, orders, lineitem


def generate(sf: float, device="cuda:0", seed: int = 1) -> Tables:
    dev = torch.device(device)
    nc = int(150_000 * sf)
    no = int(1_500_000 * sf)
    # customer
    c_custkey = torch.arange(1, nc + 1, dtype=torch.int64, device=dev)
    c_mktsegment = _uniform(nc, seed * 1000 + 1, 0, 4, dev).to(torch.int8)
    # orders: sparse keys (8 used of every 32), customers not divisible by 3
    i = torch.arange(no, dtype=torch.int64, device=dev)
    o_orderkey = (i // 8) * 32 + (i % 8) + 1
    ck = _uniform(no, seed * 1000 + 2, 1, nc, dev)
    o_custkey = torch.where(ck % 3 == 0, torch.where(ck > 1, ck - 1, ck + 1), ck)
    o_orderdate = _uniform(no, seed * 1000 + 3, 0, ORDERDATE_MAX, dev).to(torch.int32)
    o_shippriority = torch.zeros(no, dtype=torch.int32, device=dev)
    # lineitem: 1..7 per order
    nl_per = _uniform(no, seed * 1000 + 4, 1, 7, dev)
    l_order_row = torch.repeat_interleave(torch.arange(no, device=dev), nl_per)
    nl = l_order_row.numel()
    l_orderkey = o_orderkey[l_order_row]
    npart = int(200_000 * sf) if sf >= 0.005 else 1000
    partkey = _uniform(nl, seed * 1000 + 5, 1, npart, dev)
    retail_cents = 90000 + (partkey // 10) % 20001 + 100 * (partkey % 1000)
    quantity = _uniform(nl, seed * 1000 + 6, 1, 50, dev)
    l_extendedprice = quantity * retail_cents
    l_discount = _uniform(nl, seed * 1000 + 7, 0, 10, dev).to(torch.int32)
    l_shipdate = (o_orderdate[l_order_row].to(torch.int64) + _uniform(nl, seed * 1000 + 8, 1, 121, dev)).to(
        torch.int32)
    return Tables(sf, c_custkey, c_mktsegment, o_orderkey, o_custkey, o_orderdate, o_shippriority, l_orderkey,
                  l_extendedprice, l_discount, l_shipdate)


@dataclass
class Q3Result:
    l_orderkey: list
    revenue: list  # units of 1e-4 (cents x percent)
    o_orderdate: list
    o_shippriority: list
    groups: int  # qualifying (order) groups before the limit


def q3(t: Tables, segment: str = "BUILDING", date: str = "1995-03-15", limit: int = 10) -> Q3Result:
    dev = t.device
    seg = SEGMENTS.index(segment)
    d = day(date)
    # customer ⋈ orders: build on the segment's customers, probe the date-filtered orders
    cust = t.c_custkey[t.c_mktsegment == seg]
    o_rows = torch.nonzero(t.o_orderdate < d).squeeze(1)
    with HashTable(1, "int64", dev.index or 0) as tc:
        tc.build(cust)
        _, po = tc.probe(t.o_custkey[o_rows].contiguous(), device_output=True)
    sel = o_rows[po.to(torch.int64)]  # qualifying orders (custkeys are unique: <= 1 match each)
    # orders ⋈ lineitem: build on the qualifying orders' keys, probe the date-filtered lines
    l_rows = torch.nonzero(t.l_shipdate > d).squeeze(1)
    with HashTable(1, "int64", dev.index or 0) as to:
        to.build(t.o_orderkey[sel].contiguous())
        bo, pl = to.probe(t.l_orderkey[l_rows].contiguous(), device_output=True)
    lines = l_rows[pl.to(torch.int64)]
    rev = t.l_extendedprice[lines] * (100 - t.l_discount[lines].to(torch.int64))
    sums = torch.zeros(sel.numel(), dtype=torch.int64, device=dev).index_add_(0, bo, rev)
    has = torch.zeros(sel.numel(), dtype=torch.bool, device=dev)
    has[bo] = True
    g = torch.nonzero(has).squeeze(1)
    odate = t.o_orderdate[sel[g]]
    # order by revenue desc, o_orderdate asc (stable sorts, last key first)
    o1 = torch.argsort(odate, stable=True)
    o2 = torch.argsort(-sums[g][o1], stable=True)
    top = g[o1][o2][:limit]
    rows = sel[top]
    return Q3Result(t.o_orderkey[rows].tolist(), sums[top].tolist(), t.o_orderdate[rows].tolist(),
                    t.o_shippriority[rows].tolist(), int(g.numel()))
