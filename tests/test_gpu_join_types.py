"""GPU: the join types and output materialisation.

* The reference's own SQL KATs for every join type (src/lib.rs:248-726; results compared
  after sorting, the reference's collect_and_sort_results / collect_and_order_results,
  src/lib.rs:756-793).
* Random parity of every join type against a model built from the oracle's inner pairs
  with the reference's per-join-type index rules (src/shared/datafusion_private.rs:85-239,
  src/operator/probe_lookup_implementation/*.rs) - exact order for one partition and
  one probe batch, sorted multisets otherwise.
* The gather / mark / select kernels against pyarrow.compute.take and numpy.
"""
import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

pytestmark = pytest.mark.gpu


def rb(**cols):
    return pa.RecordBatch.from_pydict(cols)


def ids(vals):
    return pa.array(vals, pa.int32())


def sort_rows(tbl: pa.Table, keys):
    return tbl.sort_by([(k, "ascending") for k in keys], null_placement="at_end") if tbl.num_rows else tbl


def run(left, right, jt, flt=None):
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    out = ParallelHashJoin([[left]], [[right]], on=[("id", "id")], join_type=jt, filter=flt,
                           right_schema=right.schema).collect()
    if not out:
        return None
    return pa.Table.from_batches(out)


def rows(tbl):
    return [tuple(tbl.column(i)[r].as_py() for i in range(tbl.num_columns)) for r in range(tbl.num_rows)]


def sorted_rows(tbl, cols):
    return sorted(rows(tbl), key=lambda t: tuple((x is None, x) for x in (t[c] for c in cols)))


# ---- the reference's KATs --------------------------------------------------------

def test_kat_left_join(dfp):
    """src/lib.rs:263-306."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([1, 1, None]), value=["right"] * 3)
    t = run(left, right, "left")
    assert sorted_rows(t, [0]) == sorted([
        (1, "left", 1, "right"), (1, "left", 1, "right"), (2, "left", None, None), (None, "left", None, None)],
        key=lambda r: (r[0] is None, r[0]))


def test_kat_left_semi(dfp):
    """src/lib.rs:324-371."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([1, 1, None]), value=["right"] * 3)
    assert rows(run(left, right, "leftsemi")) == [(1, "left")]


def test_kat_left_anti(dfp):
    """src/lib.rs:389-436: the null-key build row is not matched, so it is returned."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([1, 1, None]), value=["right"] * 3)
    assert sorted_rows(run(left, right, "leftanti"), [0]) == [(2, "left"), (None, "left")]


def test_kat_right_join(dfp):
    """src/lib.rs:454-497 (FULL OUTER JOIN ... WHERE right.id IS NOT NULL, planned as a
    Right join): the WHERE drops the null-key probe row."""
    left = rb(id=ids([1, 1, None]), value=["left"] * 3)
    right = rb(id=ids([1, 2, None]), value=["right"] * 3)
    t = run(left, right, "right")
    t = t.filter(pc.is_valid(t.column(2)))
    assert sorted_rows(t, [2]) == [(1, "left", 1, "right"), (1, "left", 1, "right"), (None, None, 2, "right")]


def test_kat_right_anti(dfp):
    """src/lib.rs:512-575."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([1, 2, 3, None]), value=["right"] * 4)
    assert sorted_rows(run(left, right, "rightanti"), [0]) == [(3, "right"), (None, "right")]


def test_kat_right_semi(dfp):
    """RightSemi on the same inputs: the probe rows with a match."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([1, 2, 3, None, 2]), value=["right"] * 5)
    assert rows(run(left, right, "rightsemi")) == [(1, "right"), (2, "right"), (2, "right")]


def test_kat_full_join(dfp):
    """src/lib.rs:591-645."""
    left = rb(id=ids([1, 2, None]), value=["left"] * 3)
    right = rb(id=ids([2, 3, None]), value=["right"] * 3)
    got = sorted_rows(run(left, right, "full"), [0, 2])
    want = [(1, "left", None, None), (2, "left", 2, "right"), (None, None, 3, "right"),
            (None, None, None, "right"), (None, "left", None, None)]
    assert sorted(got, key=repr) == sorted(want, key=repr)


def test_kat_full_join_with_filter(dfp):
    """src/lib.rs:651-726: ON left.id = right.id AND left.value != right.value."""
    from datafusion_parallelism_amd.operator import JoinFilter

    left = rb(id=ids([1, 2, 3, None]), value=["left", "left", "same", "left"])
    right = rb(id=ids([2, 3, 4, None]), value=["right", "same", "right", "right"])
    flt = JoinFilter(lambda l, r: pc.not_equal(l.column("value"), r.column("value")), ["value"], ["value"])
    got = run(left, right, "full", flt)
    want = [(1, "left", None, None), (2, "left", 2, "right"), (3, "same", None, None), (None, None, 3, "same"),
            (None, None, 4, "right"), (None, None, None, "right"), (None, "left", None, None)]
    assert sorted(rows(got), key=repr) == sorted(want, key=repr)


# ---- random parity per join type --------------------------------------------------

def model(jt, nb, np_, pairs_b, pairs_p):
    """Reference index rules over the canonical inner pairs (one build batch, one probe
    batch, one partition): returns the expected (build_row | None, probe_row | None) list
    in the reference's emission order."""
    pb, pp = list(map(int, pairs_b)), list(map(int, pairs_p))
    mb, mp = set(pb), set(pp)
    inner = list(zip(pb, pp))
    um_probe = [(None, i) for i in range(np_) if i not in mp]
    um_build = [(i, None) for i in range(nb) if i not in mb]
    return {
        "inner": inner,
        "left": inner + um_build,
        "right": inner + um_probe,
        "full": inner + um_probe + um_build,
        "leftsemi": [(i, None) for i in sorted(mb)],
        "leftanti": um_build,
        "rightsemi": [(None, i) for i in sorted(mp)],
        "rightanti": um_probe,
    }[jt]


JOIN_TYPES = ["inner", "left", "right", "full", "leftsemi", "leftanti", "rightsemi", "rightanti"]


@pytest.mark.parametrize("jt", JOIN_TYPES)
def test_join_types_random_exact_order(dfp, oracle_mod, jt):
    rng = np.random.default_rng(7)
    nb, np_ = 3000, 5000
    bk = rng.integers(0, 2500, nb)
    pk = rng.integers(0, 4000, np_)
    bnull = rng.random(nb) < 0.05
    pnull = rng.random(np_) < 0.05
    left = pa.RecordBatch.from_pydict({"id": pa.array(bk, mask=bnull), "bid": np.arange(nb)})
    right = pa.RecordBatch.from_pydict({"id": pa.array(pk, mask=pnull), "pid": np.arange(np_)})
    t = run(left, right, jt)
    ob, op = oracle_mod.inner_join(bk, pk, ~bnull, ~pnull)
    want = model(jt, nb, np_, ob, op)
    got_b = t.column("bid").to_pylist() if "bid" in t.column_names else [None] * t.num_rows
    got_p = t.column("pid").to_pylist() if "pid" in t.column_names else [None] * t.num_rows
    assert list(zip(got_b, got_p)) == want
    # payload columns travel with their rows
    if "bid" in t.column_names:
        idv = t.column(0).to_pylist()
        for b, k in zip(got_b, idv):
            assert k == (None if b is None or bnull[b] else int(bk[b]))


@pytest.mark.parametrize("jt", JOIN_TYPES)
def test_join_types_partitioned_multiset(dfp, oracle_mod, jt):
    """4 build + 4 probe partitions of several batches: the same rows as the model (as
    multisets: partition interleaving is free, as in the reference's tests)."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    rng = np.random.default_rng(11)
    nb, np_ = 6000, 9000
    bk = rng.integers(0, 5000, nb)
    pk = rng.integers(0, 7000, np_)
    bnull = rng.random(nb) < 0.03
    left = pa.Table.from_pydict({"id": pa.array(bk, mask=bnull), "bid": np.arange(nb)})
    right = pa.Table.from_pydict({"id": pa.array(pk), "pid": np.arange(np_)})
    lb = left.to_batches(max_chunksize=700)
    rbs = right.to_batches(max_chunksize=900)
    join = ParallelHashJoin([lb[i::4] for i in range(4)], [rbs[i::4] for i in range(4)], on=[("id", "id")],
                            join_type=jt, right_schema=right.schema)
    out = join.collect()
    t = pa.Table.from_batches(out)
    got_b = t.column("bid").to_pylist() if "bid" in t.column_names else [None] * t.num_rows
    got_p = t.column("pid").to_pylist() if "pid" in t.column_names else [None] * t.num_rows
    ob, op = oracle_mod.inner_join(bk, pk, ~bnull, None)
    want = model(jt, nb, np_, ob, op)
    assert sorted(zip(got_b, got_p), key=repr) == sorted(want, key=repr)


# ---- kernels ----------------------------------------------------------------------

COLUMNS = {
    "int8": pa.array([1, -2, None, 4, 5, None, 7] * 50, pa.int8()),
    "int16": pa.array([1000, None, -3] * 90, pa.int16()),
    "int32": pa.array(list(range(300)), pa.int32()),
    "int64": pa.array([2**40 + i if i % 7 else None for i in range(333)], pa.int64()),
    "float64": pa.array([0.5 * i if i % 5 else None for i in range(321)], pa.float64()),
    "float32": pa.array([1.25 * i for i in range(100)], pa.float32()),
    "bool": pa.array([True, False, None] * 77, pa.bool_()),
    "date32": pa.array(list(range(200)), pa.date32()),
    "decimal128": pa.array([i * 3 for i in range(150)], pa.decimal128(20, 2)),
    "utf8": pa.array(["hello", None, "", "a much longer string " * 5, "x"] * 60, pa.string()),
    "large_utf8": pa.array(["ä", "bb", None] * 100, pa.large_string()),
    "binary": pa.array([b"\x00\x01", None, b"abc" * 40] * 70, pa.binary()),
}


@pytest.mark.parametrize("name", sorted(COLUMNS))
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("sliced", [False, True])
def test_gather_matches_arrow_take(dfp, name, idx_dtype, sliced):
    from datafusion_parallelism_amd.columns import DeviceColumn

    arr = COLUMNS[name]
    if sliced:
        arr = arr.slice(13, len(arr) - 20)
    rng = np.random.default_rng(len(arr))
    idx = rng.integers(0, len(arr), 1000)
    nullmask = rng.random(1000) < 0.1
    idx_t = torch.from_numpy(np.where(nullmask, -1, idx)).to(idx_dtype).cuda()
    got = DeviceColumn.from_arrow(arr, "cuda:0").take(idx_t).to_arrow()
    want = pc.take(arr, pa.array(idx, mask=nullmask, type=pa.int64()))
    assert got.equals(want), name


def test_gather_empty_and_all_null(dfp):
    from datafusion_parallelism_amd.columns import DeviceColumn

    for arr in (pa.array([], pa.int64()), pa.array([], pa.string()), pa.array([None, None], pa.string())):
        col = DeviceColumn.from_arrow(arr, "cuda:0")
        e = col.take(torch.empty(0, dtype=torch.int64, device="cuda:0")).to_arrow()
        assert len(e) == 0 and e.type == arr.type
        n = col.take(torch.full((5,), -1, dtype=torch.int64, device="cuda:0")).to_arrow()
        assert n.null_count == 5 and n.type == arr.type


@pytest.mark.parametrize("n", [0, 1, 15, 4096, 4097, 100003])
def test_mark_and_select(dfp, n):
    from datafusion_parallelism_amd.columns import mark_rows, select_rows

    rng = np.random.default_rng(n)
    idx = rng.integers(-1, max(n, 1), 3 * n + 1)
    flags = mark_rows(torch.from_numpy(idx).cuda(), n)
    want = np.zeros(max(n, 1), np.uint8)
    want[idx[(idx >= 0) & (idx < n)]] = 1
    assert np.array_equal(flags.cpu().numpy()[:n], want[:n])
    for w in (0, 1):
        got = select_rows(flags, w, n).cpu().numpy()
        assert np.array_equal(got, np.nonzero(want[:n] == w)[0])
