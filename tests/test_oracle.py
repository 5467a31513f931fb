"""CPU: pin the oracle (oracle/hj_oracle.c + oracle/oracle.py) to every known-answer test
the reference holds for this path (tests/golden/reference_kats.json, transcribed from
the reference's own assertions), and cross-check its two restatements (reference
semantics vs the multithreaded Version 10 table) against each other."""
import ctypes
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))


def chain_of(oracle, keys, key):
    """Build rows chained under `key`, newest first (probe one key)."""
    b, p = oracle.inner_join(np.asarray(keys, np.int64), np.array([key], np.int64))
    return [int(x) for x in b]


def test_exponential_generator_kat(oracle_mod):
    k = KATS["make_exponential_int_array_0_10"]
    assert oracle_mod.make_exponential_int_array(0, 10).tolist() == k["expected"]


def test_exponential_generator_c3_shape(oracle_mod):
    """C3's 10^7 exponential keys with libm powf (f32::powf): 6,603,254 distinct, max
    multiplicity 6. (SURVEY.md §8(d)'s 6,602,610 came from numpy's float32 power.)"""
    e = oracle_mod.make_exponential_int_array(0, 10**7)
    vals, cnt = np.unique(e, return_counts=True)
    assert len(vals) == 6603254 and cnt.max() == 6 and (e == 0).sum() == 6


def test_exponential_generator_is_libm_powf(oracle_mod):
    """src/api_utils.rs:15-23 computes 16f32.pow(x) with f32::powf, i.e. libm powf. The
    restatement calls powf; numpy's float32 power is another approximation, which
    this pins as different (so the C3 input is not numpy's)."""
    import ctypes.util

    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.powf.restype = ctypes.c_float
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    diff = 10**7
    n = np.arange(0, diff, 997, dtype=np.float32)
    x = n / np.float32(diff)
    y = np.array([libm.powf(16.0, float(v)) for v in x], dtype=np.float32)
    v = (((y - np.float32(1.0)) / np.float32(15.0)).astype(np.float32) * np.float32(diff)).astype(np.float32)
    want = np.trunc(v).astype(np.int32)
    got = oracle_mod.make_exponential_int_array(0, diff)[::997]
    assert np.array_equal(got, want)
    assert not np.array_equal(np.power(np.float32(16.0), x).astype(np.float32), y)


def test_exponential_generator_product_equals_oracle(oracle_mod):
    """The product-side generator (hj_gen_exponential_keys, a host function of the HIP
    library; bench.py's C3 input) reproduces the oracle's keys."""
    from datafusion_parallelism_amd.api_utils import make_exponential_int_array

    for lo, hi in [(0, 10), (-50, 4000), (0, 10**6)]:
        assert np.array_equal(make_exponential_int_array(lo, hi), oracle_mod.make_exponential_int_array(lo, hi))


def test_v10_build_lookup_kat(oracle_mod):
    k = KATS["v10_build_lookup_map"]
    rows = [x for b in k["batches"] for x in b]
    for key, asc in k["expected_ascending"].items():
        assert list(reversed(chain_of(oracle_mod, rows, int(key)))) == asc
    for key in k["absent"]:
        assert chain_of(oracle_mod, rows, key) == []


def test_insert_returns_previous_kat(oracle_mod):
    k = KATS["fixed_table_insert_returns_previous"]
    keys = [h for h, _, _ in k["inserts"]]
    values = [v for _, v, _ in k["inserts"]]
    prev = oracle_mod.chain_links(np.array(keys, np.int64))
    got = [None if prev[i] < 0 else values[prev[i]] for i in range(len(keys))]
    assert got == [e for _, _, e in k["inserts"]]


def test_zero_hash_kat(oracle_mod):
    k = KATS["fixed_table_zero_hash"]
    keys = [h for h, _ in k["inserts"]]
    values = [v for _, v in k["inserts"]]
    for key, val in k["expect_get"]:
        assert [values[r] for r in chain_of(oracle_mod, keys, key)] == [val]


@pytest.mark.parametrize("name", ["chain_with_zero", "chain_matching_last"])
def test_chain_kats(oracle_mod, name):
    k = KATS[name]
    order = list(reversed(k["indices"]))  # the test inserts the indices in reverse
    rows = chain_of(oracle_mod, [k["key"]] * len(order), k["key"])
    assert [order[r] for r in rows] == k["indices"]


def test_chain_follows_indexes_kat(oracle_mod):
    k = KATS["chain_follows_indexes"]
    keys, idx = [], []
    for key, indices in k["pairs"].items():
        for i in reversed(indices):
            keys.append(int(key))
            idx.append(i)
    for key, indices in k["pairs"].items():
        assert [idx[r] for r in chain_of(oracle_mod, keys, int(key))] == indices


def test_chain_spanning_blocks_kat(oracle_mod):
    k = KATS["chain_spanning_blocks"]
    stored = [blk * k["block_size"] + i for blk, i in k["inserts"]]  # index + block offset
    rows = chain_of(oracle_mod, [1] * len(stored), 1)
    assert [stored[r] for r in rows] == k["expected"]


def test_partitioned_chain_kats(oracle_mod):
    k = KATS["partitioned_chains"]
    first = k["blocks"][0]
    for key, exp in k["expected_after_block_1"].items():
        assert chain_of(oracle_mod, first, int(key)) == exp
    both = first + k["blocks"][1]
    for key, exp in k["expected_after_block_2"].items():
        assert chain_of(oracle_mod, both, int(key)) == exp


def test_sql_inner_join_no_filter_kat(oracle_mod):
    """Four successive equi-joins of the 1024-row base table with 1024-row small
    tables: every base row survives exactly once, ids preserved."""
    k = KATS["sql_inner_join_no_filter"]
    ids = np.concatenate([np.arange(i * k["batch_size"], (i + 1) * k["batch_size"]) for i in range(k["batches"])])
    base_rows = np.arange(len(ids))
    cur = ids.copy()
    for _ in range(4):
        b, p = oracle_mod.inner_join(ids, cur)  # build = small table, probe = running result
        assert np.array_equal(ids[b], cur[p])
        base_rows = base_rows[p]
        cur = cur[p]
    assert len(cur) == k["expected_rows"] and sorted(cur.tolist()) == list(range(1024))


def test_sql_nulls_and_no_match_kats(oracle_mod):
    k = KATS["sql_inner_join_with_nulls"]
    lv = [x is not None for x in k["left"]]
    rv = [x is not None for x in k["right"]]
    lk = [0 if x is None else x for x in k["left"]]
    rk = [0 if x is None else x for x in k["right"]]
    b, p = oracle_mod.inner_join(lk, rk, lv, rv)
    assert [[lk[i], rk[j]] for i, j in zip(b, p)] == k["expected_left_right_ids"]
    k = KATS["sql_inner_join_without_matches"]
    lv = [x is not None for x in k["left"]]
    rv = [x is not None for x in k["right"]]
    b, _ = oracle_mod.inner_join([0 if x is None else x for x in k["left"]],
                                 [0 if x is None else x for x in k["right"]], lv, rv)
    assert len(b) == k["expected_rows"]


def test_weak_hash_equality_filter(oracle_mod):
    """With a 4-bit hash nearly every candidate is a collision; equal_rows_arr must
    remove them, so the pairs equal those under the strong hash."""
    rng = np.random.default_rng(1)
    bk = rng.integers(0, 300, 2000)
    pk = rng.integers(0, 400, 3000)
    a = oracle_mod.inner_join(bk, pk, hash_mode=0)
    b = oracle_mod.inner_join(bk, pk, hash_mode=1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_pairs_are_brute_force_join(oracle_mod):
    rng = np.random.default_rng(2)
    bk = rng.integers(-50, 50, 700)
    pk = rng.integers(-60, 60, 900)
    bv = rng.random(700) > 0.1
    pv = rng.random(900) > 0.1
    b, p = oracle_mod.inner_join(bk, pk, bv, pv)
    want = [(i, j) for j in range(900) if pv[j] for i in range(699, -1, -1) if bv[i] and bk[i] == pk[j]]
    assert list(zip(b.tolist(), p.tolist())) == want


@pytest.mark.parametrize("nthreads", [1, 4])
def test_v10_restatement_matches_semantics(oracle_mod, nthreads):
    """The multithreaded Version 10 table (CPU baseline) gives the same pair set; at one
    thread also the same order."""
    rng = np.random.default_rng(3)
    bk = rng.integers(0, 20000, 50000)
    pk = rng.integers(0, 40000, 80000)
    ob, op = oracle_mod.inner_join(bk, pk)
    t = oracle_mod.V10Table(bk, nthreads=nthreads)
    vb, vp = t.probe(pk, nthreads=nthreads)
    t.close()
    if nthreads == 1:
        assert np.array_equal(vb, ob) and np.array_equal(vp, op)
    cb, cp = oracle_mod.canonical_pairs(vb, vp)
    assert np.array_equal(cb, ob) and np.array_equal(cp.astype(np.uint32), op)


def test_golden_vectors_reproduce(oracle_mod):
    """The committed oracle vectors are what the oracle computes today."""
    v = np.load(os.path.join(HERE, "golden", "oracle_vectors.npz"))
    names = sorted({k.split("__")[0] for k in v.files})
    for n in names:
        ob, op = oracle_mod.inner_join(v[n + "__bk"], v[n + "__pk"], v[n + "__bv"], v[n + "__pv"])
        assert np.array_equal(ob, v[n + "__ob"]) and np.array_equal(op, v[n + "__op"]), n


def test_canonical_pairs_and_digest(oracle_mod):
    b = np.array([3, 9, 1, 7], np.uint64)
    p = np.array([2, 0, 2, 0], np.uint32)
    cb, cp = oracle_mod.canonical_pairs(b, p)
    assert cb.tolist() == [9, 7, 3, 1] and cp.tolist() == [0, 0, 2, 2]
    assert oracle_mod.pairs_digest(cb, cp) == oracle_mod.pairs_digest(*oracle_mod.canonical_pairs(b[::-1], p[::-1]))


def test_generators(oracle_mod):
    k = oracle_mod.perm_keys(10**6, 7368787, 10**6)
    assert len(np.unique(k)) == 10**6
    u = oracle_mod.uniform_keys(1000, 0xC0FFEE, 2 * 10**7)
    c = np.empty(1000, np.int64)
    oracle_mod.lib().ora_gen_uniform(c.ctypes.data, 1000, 0xC0FFEE, 2 * 10**7)
    assert np.array_equal(u, c)


def _exp_digests():
    import hashlib

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "exponential_digests.json")) as f:
        return json.load(f)["sizes"], hashlib


def _check_exp_digests(gen):
    sizes, hashlib = _exp_digests()
    for r in sizes:
        a = np.ascontiguousarray(gen(r["lo"], r["hi"]).astype("<i4"))
        assert hashlib.sha256(a.tobytes()).hexdigest() == r["libm"]["sha256"], (r["lo"], r["hi"])
        assert np.unique(a).size == r["libm"]["distinct"]


def test_exponential_generator_digests(oracle_mod):
    """the C3 generator pinned at six sizes (up to C3's 10^7) against
    committed digests (tests/golden/make_exponential_digests.py), for the oracle and the
    product generator, so a libm change cannot silently move C3's key multiset. At 10^7
    the libm (f32::powf) keys have 6,603,254 distinct values; numpy's float32 power gives
    SURVEY.md §8(d)'s 6,602,610 (recorded beside it)."""
    from datafusion_parallelism_amd.api_utils import make_exponential_int_array

    _check_exp_digests(oracle_mod.make_exponential_int_array)
    _check_exp_digests(make_exponential_int_array)
    sizes, _ = _exp_digests()
    big = [r for r in sizes if r["hi"] - r["lo"] == 10**7][0]
    assert big["libm"]["distinct"] == 6603254 and big["numpy"]["distinct"] == 6602610


@pytest.mark.gpu
def test_exponential_generator_digests_on_gpu_box():
    """The same digests on the GPU box's libm (GPUTEST): bench.py's C3 keys there are the
    committed multiset."""
    from datafusion_parallelism_amd.api_utils import make_exponential_int_array

    _check_exp_digests(make_exponential_int_array)
