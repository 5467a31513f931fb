"""GPU parity of joins on several key columns, or on non-integer keys (SURVEY.md §8a a2 /
a12 in full): hj_composite_keys (the reference's calculate_hash over every key column,
src/shared/shared.rs:11-16) builds and probes the table, hj_filter_equal_pairs restates
equal_rows_arr (src/shared/datafusion_private.rs:52-73), ANDing equality over the
columns. Expected pairs: the oracle's single-key join on a key that is a bijection of the
tuple (two int32 columns packed into one int64; strings numbered by a dictionary), which
has the same pairs in the same canonical order."""
import numpy as np
import pyarrow as pa
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pack(a, b):
    return (a.astype(np.int64) << 32) | (b.astype(np.int64) & 0xFFFFFFFF)


def _gpu_multi(dfp, build_arrays, probe_arrays):
    """Build from the key columns (one batch), probe with the probe key columns, filter."""
    from datafusion_parallelism_amd.columns import DeviceColumn, composite_keys, filter_equal_pairs

    dev = torch.device("cuda", 0)
    bcols = [DeviceColumn.from_arrow(a, dev) for a in build_arrays]
    pcols = [DeviceColumn.from_arrow(a, dev) for a in probe_arrays]
    bk, bv = composite_keys(bcols)
    pk, pv = composite_keys(pcols)
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk, bv)
        b, p = t.probe(pk, pv, device_output=True)
        b, p = filter_equal_pairs(bcols, pcols, b, p)
    return b.cpu().numpy().astype(np.uint64), p.cpu().numpy().view(np.uint32)


def _valid(arrs):
    v = np.ones(len(arrs[0]), dtype=bool)
    for a in arrs:
        v &= ~np.asarray(a.is_null().to_numpy(zero_copy_only=False))
    return v


@pytest.mark.parametrize("nb,np_,krange,null_frac", [
    (1, 1, 2, 0.0),
    (5000, 7000, 40, 0.0),          # many duplicate tuples
    (200_000, 300_000, 700, 0.05),  # nulls in either column
])
def test_two_int32_columns(dfp, oracle_mod, nb, np_, krange, null_frac):
    rng = np.random.default_rng(nb + np_)
    ba, bb = rng.integers(-krange, krange, nb).astype(np.int32), rng.integers(-krange, krange, nb).astype(np.int32)
    pa_, pb = rng.integers(-krange, krange, np_).astype(np.int32), rng.integers(-krange, krange, np_).astype(np.int32)
    masks = [rng.random(n) < null_frac if null_frac else None for n in (nb, nb, np_, np_)]
    arrs = [pa.array(x, type=pa.int32(), mask=m) for x, m in zip((ba, bb, pa_, pb), masks)]
    b, p = _gpu_multi(dfp, arrs[:2], arrs[2:])
    ob, op = oracle_mod.inner_join(_pack(ba, bb), _pack(pa_, pb), _valid(arrs[:2]), _valid(arrs[2:]))
    assert np.array_equal(p, op) and np.array_equal(b, ob)


def test_utf8_key_column(dfp, oracle_mod):
    """A single Utf8 key (not an integer: composite path), incl. empty strings and nulls."""
    rng = np.random.default_rng(11)
    words = np.array(["", "a", "ab", "abc", "longer-string-key-0001", "longer-string-key-0002", "zz"] +
                     [f"k{i}" for i in range(300)], dtype=object)
    bi, pi = rng.integers(0, len(words), 20_000), rng.integers(0, len(words) + 50, 30_000)
    bmask, pmask = rng.random(20_000) < 0.03, rng.random(30_000) < 0.03
    bstr = pa.array([words[i] for i in bi], type=pa.string(), mask=bmask)
    pstr = pa.array([words[i] if i < len(words) else f"miss{i}" for i in pi], type=pa.string(), mask=pmask)
    b, p = _gpu_multi(dfp, [bstr], [pstr])
    ob, op = oracle_mod.inner_join(bi.astype(np.int64), pi.astype(np.int64), ~bmask, ~pmask)
    assert np.array_equal(p, op) and np.array_equal(b, ob)


def test_int64_and_large_utf8_columns(dfp, oracle_mod):
    """(Int64, LargeUtf8) keys: equality ANDed over a fixed- and a variable-width column."""
    rng = np.random.default_rng(5)
    nb, np_ = 50_000, 80_000
    bx, by = rng.integers(0, 50, nb), rng.integers(0, 60, nb)
    px, py = rng.integers(0, 55, np_), rng.integers(0, 66, np_)
    arrs = [pa.array(bx, type=pa.int64()), pa.array([f"s{v}" for v in by], type=pa.large_string()),
            pa.array(px, type=pa.int64()), pa.array([f"s{v}" for v in py], type=pa.large_string())]
    b, p = _gpu_multi(dfp, arrs[:2], arrs[2:])
    ob, op = oracle_mod.inner_join(bx * 1000 + by, px * 1000 + py)
    assert np.array_equal(p, op) and np.array_equal(b, ob)


def test_filter_equal_pairs_drops_unequal_candidates(dfp):
    """hj_filter_equal_pairs alone: crafted candidates (as a composite-key collision would
    give) keep exactly the equal tuples, in order."""
    from datafusion_parallelism_amd.columns import DeviceColumn, filter_equal_pairs

    dev = torch.device("cuda", 0)
    bc = [DeviceColumn.from_arrow(pa.array([1, 2, 3, 4], pa.int32()), dev),
          DeviceColumn.from_arrow(pa.array(["x", "y", "zz", "y"]), dev)]
    pc = [DeviceColumn.from_arrow(pa.array([2, 4, 3], pa.int32()), dev),
          DeviceColumn.from_arrow(pa.array(["y", "y", "z"]), dev)]
    b = torch.tensor([3, 1, 0, 3, 2, 1], dtype=torch.int64, device=dev)
    p = torch.tensor([0, 0, 0, 1, 2, 2], dtype=torch.int32, device=dev)
    fb, fp = filter_equal_pairs(bc, pc, b, p)
    assert fb.tolist() == [1, 3] and fp.tolist() == [0, 1]


def test_operator_two_key_columns(dfp, oracle_mod):
    """ParallelHashJoin with on = [(a, x), (b, y)], 2 partitions, through the reference's
    operator surface (src/operator/parallel_hash_join.rs)."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    rng = np.random.default_rng(3)
    nb, np_ = 6000, 9000
    a, bcol = rng.integers(0, 30, nb).astype(np.int32), rng.integers(0, 20, nb).astype(np.int32)
    x, y = rng.integers(0, 35, np_).astype(np.int32), rng.integers(0, 22, np_).astype(np.int32)
    left = pa.RecordBatch.from_arrays([pa.array(a), pa.array(bcol), pa.array(np.arange(nb))], names=["a", "b", "bid"])
    right = pa.RecordBatch.from_arrays([pa.array(x), pa.array(y), pa.array(np.arange(np_))], names=["x", "y", "pid"])
    j = ParallelHashJoin([[left.slice(0, 2500)], [left.slice(2500)]], [[right.slice(0, 4000)], [right.slice(4000)]],
                         on=[("a", "x"), ("b", "y")])
    out = pa.Table.from_batches(j.collect())
    got = sorted(zip(out.column("bid").to_pylist(), out.column("pid").to_pylist()))
    ob, op = oracle_mod.inner_join(_pack(a, bcol), _pack(x, y))
    assert got == sorted(zip(ob.astype(np.int64).tolist(), op.astype(np.int64).tolist()))
