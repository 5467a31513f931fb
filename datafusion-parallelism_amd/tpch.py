"""TPC-H-shaped tables and Q3 on the GPU join (BASELINE.json
configs[3]: TPC-H Q3, lineitem ⋈ orders ⋈ customer).

There is no network for dbgen / tpchgen-cli, so `generate` builds the three tables Q3
reads on the device from a counter-based generator (splitmix64 of (stream, row counter);
lineitem columns are keyed by (order, line number), as in dbgen),
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

Multi-GPU (C4/C5: Q3 at SF100 and Q9 at SF300 on 8 GPUs): `generate(..., rank, world)`
produces rank r's block of every table (the same rows the one-GPU tables hold at those
positions), and `q3_dist` / `q9_dist` run the plans with one process per GPU: filtered
dimension sides are broadcast (`all_gather_rows`), the large sides are hash-repartitioned
on the join key with their payload (`shuffle`, RCCL all-to-all), every join is a local
GPU hash join, and the group-by results merge with one all-reduce (Q9) or an all-gather
of per-rank top-k candidates (Q3).

Q9 (BASELINE.json configs[4], the six-way join):
    select nation, o_year, sum(l_extendedprice * (1 - l_discount)
                               - ps_supplycost * l_quantity) as sum_profit
    from part, supplier, lineitem, partsupp, orders, nation
    where s_suppkey = l_suppkey and ps_suppkey = l_suppkey and ps_partkey = l_partkey
      and p_partkey = l_partkey and o_orderkey = l_orderkey and s_nationkey = n_nationkey
      and p_name like '%green%'
    group by nation, o_year order by nation, o_year desc
`generate(..., q9=True)` adds part (p_name's colour words reduced to the flag "contains
green": 5 distinct words of the spec's 92, so probability 5/92), supplier (nation
uniform), partsupp (4 suppliers per part by the spec's formula, supply cost 1.00-1000.00)
and lineitem's partkey / suppkey / quantity consistent with partsupp. Five joins run on
the hash-join kernels; (partkey, suppkey) is one int64 key partkey << 32 | suppkey.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass

import torch

from .table import HashTable

SEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
EPOCH = _dt.date(1992, 1, 1)


def day(d: str | _dt.date) -> int:
    """Days since 1992-01-01."""
    if isinstance(d, str):
        d = _dt.date.fromisoformat(d)
    return (d - EPOCH).days


ORDERDATE_MAX = day("1998-08-02")  # STARTDATE .. ENDDATE - 151 days


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= 1 << 63 else c


def _mix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 tensors (two's-complement wrap = uint64 arithmetic;
    logical shifts by masking)."""
    z = x + _s64(0x9E3779B97F4A7C15)
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _s64(0x94D049BB133111EB)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def _uni(counter: torch.Tensor, stream: int, lo: int, hi: int) -> torch.Tensor:
    """Values in [lo, hi] for the given row counters (< 2^40) of one random stream: a
    pure function of (stream, counter), so any block of rows can be generated alone."""
    z = _mix(counter + (stream << 40))
    return ((z >> 11) & ((1 << 53) - 1)) % (hi - lo + 1) + lo


def _span(n: int, rank: int, world: int) -> tuple[int, int]:
    """Rank's block [lo, hi) of n rows."""
    return n * rank // world, n * (rank + 1) // world


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
    # Q9 columns (generate(..., q9=True))
    l_partkey: torch.Tensor | None = None
    l_suppkey: torch.Tensor | None = None
    l_quantity: torch.Tensor | None = None
    p_partkey: torch.Tensor | None = None
    p_green: torch.Tensor | None = None  # bool: p_name like '%green%'
    s_suppkey: torch.Tensor | None = None
    s_nationkey: torch.Tensor | None = None
    ps_partkey: torch.Tensor | None = None
    ps_suppkey: torch.Tensor | None = None
    ps_supplycost: torch.Tensor | None = None  # int64 cents

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
        if self.l_partkey is None:
            return customer, orders, lineitem
        lineitem = lineitem.assign(l_partkey=h(self.l_partkey), l_suppkey=h(self.l_suppkey),
                                   l_quantity=h(self.l_quantity))
        part = pd.DataFrame({"p_partkey": h(self.p_partkey), "p_green": h(self.p_green)})
        supplier = pd.DataFrame({"s_suppkey": h(self.s_suppkey), "s_nationkey": h(self.s_nationkey)})
        partsupp = pd.DataFrame({"ps_partkey": h(self.ps_partkey), "ps_suppkey": h(self.ps_suppkey),
                                 "ps_supplycost": h(self.ps_supplycost)})
        return customer, orders, lineitem, part, supplier, partsupp


def _supplier_of(partkey: torch.Tensor, i: torch.Tensor, ns: int) -> torch.Tensor:
    """The spec's i-th (0..3) supplier of a part: (ps_partkey + i * (S/4 + (ps_partkey-1)/S)) % S + 1."""
    return (partkey + i * (ns // 4 + (partkey - 1) // ns)) % ns + 1


def generate(sf: float, device="cuda:0", seed: int = 1, q9: bool = False, rank: int = 0, world: int = 1) -> Tables:
    """TPC-H-shaped tables at scale factor sf; with world > 1, rank's block of each table
    (customer, orders + their lineitems, part + its partsupp, supplier by row blocks)."""
    dev = torch.device(device)
    assert 0 <= seed < 1 << 16 and 0 <= rank < world

    def st(k):  # stream id of column k
        return seed * 64 + k

    nc = int(150_000 * sf)
    no = int(1_500_000 * sf)
    # customer
    c0, c1 = _span(nc, rank, world)
    ci = torch.arange(c0, c1, dtype=torch.int64, device=dev)
    c_custkey = ci + 1
    c_mktsegment = _uni(ci, st(1), 0, 4).to(torch.int8)
    # orders: sparse keys (8 used of every 32), customers not divisible by 3
    o0, o1 = _span(no, rank, world)
    i = torch.arange(o0, o1, dtype=torch.int64, device=dev)
    o_orderkey = (i // 8) * 32 + (i % 8) + 1
    ck = _uni(i, st(2), 1, nc)
    o_custkey = torch.where(ck % 3 == 0, torch.where(ck > 1, ck - 1, ck + 1), ck)
    o_orderdate = _uni(i, st(3), 0, ORDERDATE_MAX).to(torch.int32)
    o_shippriority = torch.zeros(i.numel(), dtype=torch.int32, device=dev)
    # lineitem: 1..7 per order, columns keyed by (order, line number)
    nl_per = _uni(i, st(4), 1, 7)
    l_order_row = torch.repeat_interleave(torch.arange(i.numel(), device=dev), nl_per)
    nl = l_order_row.numel()
    first = torch.cumsum(nl_per, 0) - nl_per
    lc = i[l_order_row] * 8 + (torch.arange(nl, device=dev) - first[l_order_row])
    l_orderkey = o_orderkey[l_order_row]
    npart = int(200_000 * sf) if sf >= 0.005 else 1000
    partkey = _uni(lc, st(5), 1, npart)
    retail_cents = 90000 + (partkey // 10) % 20001 + 100 * (partkey % 1000)
    quantity = _uni(lc, st(6), 1, 50)
    l_extendedprice = quantity * retail_cents
    l_discount = _uni(lc, st(7), 0, 10).to(torch.int32)
    l_shipdate = (o_orderdate[l_order_row].to(torch.int64) + _uni(lc, st(8), 1, 121)).to(torch.int32)
    t = Tables(sf, c_custkey, c_mktsegment, o_orderkey, o_custkey, o_orderdate, o_shippriority, l_orderkey,
               l_extendedprice, l_discount, l_shipdate)
    if q9:
        ns = max(int(10_000 * sf), 4)
        t.l_partkey, t.l_quantity = partkey, quantity
        t.l_suppkey = _supplier_of(partkey, _uni(lc, st(9), 0, 3), ns)
        p0, p1 = _span(npart, rank, world)
        pi = torch.arange(p0, p1, dtype=torch.int64, device=dev)
        t.p_partkey = pi + 1
        t.p_green = _uni(pi, st(10), 0, 91) < 5
        s0, s1 = _span(ns, rank, world)
        si = torch.arange(s0, s1, dtype=torch.int64, device=dev)
        t.s_suppkey = si + 1
        t.s_nationkey = _uni(si, st(11), 0, 24)
        psi = torch.arange(4 * p0, 4 * p1, dtype=torch.int64, device=dev)  # partsupp rows of the part block
        t.ps_partkey = psi // 4 + 1
        t.ps_suppkey = _supplier_of(t.ps_partkey, psi % 4, ns)
        t.ps_supplycost = _uni(psi, st(12), 100, 100_000)
    return t


@dataclass
class Q3Result:
    l_orderkey: list
    revenue: list  # units of 1e-4 (cents x percent)
    o_orderdate: list
    o_shippriority: list
    groups: int  # qualifying (order) groups before the limit


def q3(t: Tables, segment: str = "BUILDING", date: str = "1995-03-15", limit: int = 10,
       join_fn=None) -> Q3Result:
    """join_fn(build, probe) -> (build rows, probe rows): the one-GPU hash join by default;
    multi_join(devices) runs every join on a table sharded over several GPUs."""
    join = join_fn or _join
    dev = t.device
    seg = SEGMENTS.index(segment)
    d = day(date)
    # customer ⋈ orders: build on the segment's customers, probe the date-filtered orders
    cust = t.c_custkey[t.c_mktsegment == seg]
    o_rows = torch.nonzero(t.o_orderdate < d).squeeze(1)
    _, po = join(cust, t.o_custkey[o_rows])
    sel = o_rows[po]  # qualifying orders (custkeys are unique: <= 1 match each)
    # orders ⋈ lineitem: build on the qualifying orders' keys, probe the date-filtered lines
    l_rows = torch.nonzero(t.l_shipdate > d).squeeze(1)
    bo, pl = join(t.o_orderkey[sel], t.l_orderkey[l_rows])
    lines = l_rows[pl]
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


NATIONS = ["ALGERIA", "ARGENTINA", "BRAZIL", "CANADA", "EGYPT", "ETHIOPIA", "FRANCE", "GERMANY", "INDIA",
           "INDONESIA", "IRAN", "IRAQ", "JAPAN", "JORDAN", "KENYA", "MOROCCO", "PERU", "CHINA", "ROMANIA",
           "SAUDI ARABIA", "VIETNAM", "RUSSIA", "UNITED KINGDOM", "UNITED STATES", "MOZAMBIQUE"]


def year_of(days: torch.Tensor) -> torch.Tensor:
    """Calendar year of days since 1992-01-01 (1992 .. 1998; leap years 1992, 1996)."""
    starts = torch.tensor([day(f"{y}-01-01") for y in range(1992, 2000)], device=days.device)
    return torch.bucketize(days.to(torch.int64), starts, right=True) - 1 + 1992


def _join(build: torch.Tensor, probe: torch.Tensor):
    """Inner-join pairs (build row int64, probe row int64) on the GPU hash join."""
    dev = probe.device
    with HashTable(1, "int64", dev.index or 0) as t:
        t.build(build.contiguous())
        b, p = t.probe(probe.contiguous(), device_output=True)
    return b, p.to(torch.int64)


def multi_join(devices: list[int], plan: str = "radix"):
    """A join_fn whose every join runs on one table sharded over `devices`
    (hj_build_begin_multi): the radix plan gives each GPU 1/G of the build side by key
    hash and merges the shards' pairs into canonical order — the in-process form of C4/C5's
    sharded builds (a build side larger than one GPU's HBM). Devices may repeat (tests on
    one GPU)."""
    def join(build: torch.Tensor, probe: torch.Tensor):
        with HashTable(1, "int64", devices=list(devices), plan=plan) as t:
            t.append(0, build.contiguous())
            t.finish(0)
            b, p = t.probe(probe.contiguous(), device_output=True)
        return b, p.to(torch.int64)

    return join


def planned_join(devices: list[int], plan: str = "radix"):
    """A join_fn that builds each join on one GPU while its build fits the device budget
    (hj_set_device_budget / DFP_HJ_DEVICE_BUDGET_BYTES), and shards a build that does not
    over `devices` with the radix plan (every shard a one-device table of about 1/G of the
    build): C5's premise, a build side larger than one GPU, at any scale. join.log records
    one (build rows, "one-gpu" | plan, peak device bytes of the table) per join."""
    from ._lib import HjError
    from .table import is_budget_error

    log: list[tuple[int, str, int]] = []

    def join(build: torch.Tensor, probe: torch.Tensor):
        dev = probe.device
        try:
            with HashTable(1, "int64", dev.index or 0) as t:
                t.build(build.contiguous())
                peak = t.device_bytes()
                b, p = t.probe(probe.contiguous(), device_output=True)
            log.append((int(build.numel()), "one-gpu", peak))
            return b, p.to(torch.int64)
        except HjError as e:
            if not is_budget_error(e):
                raise
        with HashTable(1, "int64", devices=list(devices), plan=plan) as t:
            t.append(0, build.contiguous())
            t.finish(0)
            peak = t.device_bytes()
            b, p = t.probe(probe.contiguous(), device_output=True)
        log.append((int(build.numel()), plan, peak))
        return b, p.to(torch.int64)

    join.log = log
    return join


def q9(t: Tables, color_flag: str = "green", join_fn=None) -> list[tuple[str, int, int]]:
    """-> [(nation, o_year, sum_profit in 1e-4 units)] ordered by nation, o_year desc.
    join_fn: as q3's."""
    if t.l_partkey is None:
        raise ValueError("generate(..., q9=True) tables are needed")
    _join = join_fn or globals()["_join"]
    dev = t.device
    # lineitem ⋈ part (p_name like '%green%')
    _, li = _join(t.p_partkey[t.p_green], t.l_partkey)
    lk = t.l_partkey[li]
    ls = t.l_suppkey[li]
    # ⋈ partsupp on (partkey, suppkey)
    b_ps, p_l = _join((t.ps_partkey << 32) | t.ps_suppkey, (lk << 32) | ls)
    li, ls = li[p_l], ls[p_l]
    cost = t.ps_supplycost[b_ps]
    # ⋈ supplier on suppkey -> nation
    b_s, p_l = _join(t.s_suppkey, ls)
    li, cost, nation = li[p_l], cost[p_l], t.s_nationkey[b_s]
    # ⋈ orders on orderkey -> year
    b_o, p_l = _join(t.o_orderkey, t.l_orderkey[li])
    li, cost, nation = li[p_l], cost[p_l], nation[p_l]
    year = year_of(t.o_orderdate[b_o])
    amount = (t.l_extendedprice[li] * (100 - t.l_discount[li].to(torch.int64))
              - cost * t.l_quantity[li] * 100)
    # ⋈ nation is the 25-row dimension: group by (nationkey, year)
    gid = nation * 8 + (year - 1992)
    sums = torch.zeros(25 * 8, dtype=torch.int64, device=dev).index_add_(0, gid, amount)
    present = torch.zeros(25 * 8, dtype=torch.bool, device=dev)
    present[gid] = True
    out = []
    for g in torch.nonzero(present).squeeze(1).tolist():
        out.append((NATIONS[g // 8], 1992 + g % 8, int(sums[g])))
    out.sort(key=lambda r: (r[0], -r[1]))
    return out


# ---- multi-GPU plans (one process per GPU; C4 = Q3 SF100, C5 = Q9 SF300 on 8 GPUs) -----

def _order_q3(okey: torch.Tensor, rev: torch.Tensor, odate: torch.Tensor) -> torch.Tensor:
    """Permutation for: revenue desc, o_orderdate asc, l_orderkey asc (stable sorts, last
    key first) — the one-GPU q3's order, whose groups are already in orderkey order."""
    o = torch.argsort(okey, stable=True)
    o = o[torch.argsort(odate[o], stable=True)]
    return o[torch.argsort(-rev[o], stable=True)]


def q3_dist(t: Tables, segment: str = "BUILDING", date: str = "1995-03-15", limit: int = 10, group=None,
            join_fn=None, partition_fn=None, exchange=None) -> Q3Result:
    """Q3 over rank-sharded tables (generate(..., rank, world)); the result on every rank.

    customer (filtered) is broadcast; the qualifying orders and the ship-date-filtered
    lines are hash-repartitioned on orderkey with their payload, so each order's group
    lives on exactly one rank; the per-rank top-`limit` candidates are gathered and
    merged. `exchange` moves the data (distributed.default_exchange: on an RCCL group the
    hj_dist_shuffle / hj_dist_gather jobs of the C ABI, else torch.distributed);
    `join_fn(build, probe) -> (build rows, probe rows)` defaults to the GPU hash join (the
    stand-in hooks exist only for the CPU gloo tests)."""
    from .distributed import check_ids, default_exchange

    ex = exchange or default_exchange(group, partition_fn)
    join = join_fn or _join
    seg = SEGMENTS.index(segment)
    d = day(date)
    (cust,) = ex.gather([t.c_custkey[t.c_mktsegment == seg]])
    o_rows = torch.nonzero(t.o_orderdate < d).squeeze(1)
    _, po = join(cust, t.o_custkey[o_rows])
    sel = o_rows[po]
    ok, (od, osp) = ex.shuffle(t.o_orderkey[sel], [t.o_orderdate[sel], t.o_shippriority[sel]])
    l_rows = torch.nonzero(t.l_shipdate > d).squeeze(1)
    rev = t.l_extendedprice[l_rows] * (100 - t.l_discount[l_rows].to(torch.int64))
    lk, (lrev,) = ex.shuffle(t.l_orderkey[l_rows], [rev])
    bo, pl = join(ok, lk)
    check_ids(bo, ok.numel(), "q3_dist order rows")
    sums = torch.zeros(ok.numel(), dtype=torch.int64, device=ok.device).index_add_(0, bo, lrev[pl])
    has = torch.zeros(ok.numel(), dtype=torch.bool, device=ok.device)
    has[bo] = True
    g = torch.nonzero(has).squeeze(1)
    okey, r, dt, sp = ok[g], sums[g], od[g], osp[g]
    top = _order_q3(okey, r, dt)[:limit]
    ngroups = ex.sum(torch.tensor([g.numel()], dtype=torch.int64, device=ok.device))
    okey, r, dt, sp = ex.gather([okey[top], r[top], dt[top], sp[top]])
    top = _order_q3(okey, r, dt)[:limit]
    return Q3Result(okey[top].tolist(), r[top].tolist(), dt[top].tolist(), sp[top].tolist(), int(ngroups.item()))


def q9_dist(t: Tables, group=None, join_fn=None, partition_fn=None, exchange=None) -> list[tuple[str, int, int]]:
    """Q9 over rank-sharded tables; the result on every rank.

    green part keys and supplier are broadcast; lineitem (green parts only) and partsupp
    are repartitioned on (partkey, suppkey), then the joined lines and orders on
    orderkey; the (nation, year) sums merge with one sum over the ranks. `exchange`: as
    q3_dist's."""
    from .distributed import check_ids, default_exchange

    if t.l_partkey is None:
        raise ValueError("generate(..., q9=True) tables are needed")
    ex = exchange or default_exchange(group, partition_fn)
    join = join_fn or _join
    dev = t.device
    (green,) = ex.gather([t.p_partkey[t.p_green]])
    _, li = join(green, t.l_partkey)
    gross = t.l_extendedprice[li] * (100 - t.l_discount[li].to(torch.int64))
    psk = (t.l_partkey[li] << 32) | t.l_suppkey[li]
    lk, (ls, lok, gross, qty) = ex.shuffle(psk, [t.l_suppkey[li], t.l_orderkey[li], gross, t.l_quantity[li]])
    pk, (cost,) = ex.shuffle((t.ps_partkey << 32) | t.ps_suppkey, [t.ps_supplycost])
    b_ps, p_l = join(pk, lk)
    amount = gross[p_l] - cost[b_ps] * qty[p_l] * 100
    ls, lok = ls[p_l], lok[p_l]
    s_key, s_nat = ex.gather([t.s_suppkey, t.s_nationkey])
    b_s, p_l = join(s_key, ls)
    nation, amount, lok = s_nat[b_s], amount[p_l], lok[p_l]
    ok, (year,) = ex.shuffle(t.o_orderkey, [year_of(t.o_orderdate)])
    lk2, (nat2, amt2) = ex.shuffle(lok, [nation, amount])
    b_o, p_l = join(ok, lk2)
    gid = nat2[p_l] * 8 + (year[b_o] - 1992)
    check_ids(gid, 25 * 8, "q9_dist (nation, year) group ids")  # exchanged payload indexes the sums
    sums = torch.zeros(25 * 8, dtype=torch.int64, device=dev).index_add_(0, gid, amt2[p_l])
    cnt = torch.zeros(25 * 8, dtype=torch.int64, device=dev).index_add_(0, gid, torch.ones_like(gid))
    sums = ex.sum(sums)
    cnt = ex.sum(cnt)
    out = [(NATIONS[g // 8], 1992 + g % 8, int(sums[g])) for g in torch.nonzero(cnt).squeeze(1).tolist()]
    out.sort(key=lambda r: (r[0], -r[1]))
    return out
