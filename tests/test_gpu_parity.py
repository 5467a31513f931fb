"""GPU parity: the gfx950 build + probe through the C ABI against the oracle
(reference semantics restated in oracle/hj_oracle.c) — bit-exact pairs in canonical
order (probe ascending, build descending) — and against the reference's own KATs.

Run on an MI355X: ``pytest -m gpu``.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min


# (probe mode, table layout): hj_set_probe_mode 3 fused / 4 sliced; hj_set_build_mode 0
# auto (direct-addressed for dense key ranges, built from the tile-local partition) /
# 1 hashed / 2 auto with the histogram partition
# The sliced probe's tiles: 0 auto (2^14 rows dense, 2^15 hashed; hj_set_probe_tile_log),
# "-t15" / "-t14" force the other size for the layout
MODES = {"fused": (3, 0, 0), "fused-hashed": (3, 1, 0), "sliced": (4, 0, 0), "sliced-hashed": (4, 1, 0),
         "sliced-histbuild": (4, 2, 0), "sliced-t15": (4, 0, 15), "sliced-hashed-t14": (4, 1, 14)}


@pytest.fixture(params=list(MODES))
def probe_mode(request, dfp):
    """Run a test under every probe strategy, table layout and probe tile size (identical
    results required)."""
    L = dfp.load()
    pm, bm, tl = MODES[request.param]
    old_p = L.hj_set_probe_mode(pm)
    old_b = L.hj_set_build_mode(bm)
    old_t = L.hj_set_probe_tile_log(tl)
    yield request.param
    L.hj_set_probe_mode(old_p)
    L.hj_set_build_mode(old_b)
    L.hj_set_probe_tile_log(old_t)


def gpu_join(dfp, bkeys, pkeys, bvalid=None, pvalid=None, key_type="int64", device_input=True, parts=None):
    """Build (optionally split into `parts` partitions) and probe on the GPU."""
    bk = np.asarray(bkeys)
    pk = np.asarray(pkeys)
    nparts = 1 if parts is None else len(parts) - 1
    with dfp.HashTable(nparts, key_type, 0) as t:
        for p in range(nparts):
            lo, hi = (0, len(bk)) if parts is None else (parts[p], parts[p + 1])
            keys = torch.from_numpy(bk[lo:hi].copy()).cuda() if device_input else bk[lo:hi]
            t.append(p, keys, None if bvalid is None else np.asarray(bvalid)[lo:hi])
        t.finish_all()
        keys = torch.from_numpy(pk.copy()).cuda() if device_input else pk
        b, pp = t.probe(keys, pvalid)
        return b, pp, t.stats()


def assert_same(b, p, ob, op):
    assert len(b) == len(ob), f"count {len(b)} != oracle {len(ob)}"
    assert np.array_equal(np.asarray(p, np.uint32), op), "probe indices differ"
    assert np.array_equal(np.asarray(b, np.uint64), ob), "build indices differ"


# ---- reference KATs -----------------------------------------------------------

def test_v10_build_lookup_kat(dfp):
    """src/operator/version10/build_implementation.rs:98-178: batches [1,2,3],[2,4,5],
    [1,6,7]; id -> rows (reversed chain order in the reference test)."""
    with dfp.HashTable(1, "int32", 0) as t:
        for batch in ([1, 2, 3], [2, 4, 5], [1, 6, 7]):
            t.append(0, np.array(batch, dtype=np.int32))
        t.finish(0)
        expected = {1: [0, 6], 2: [1, 3], 3: [2], 4: [4], 5: [5], 6: [7], 7: [8]}
        for k, rows in expected.items():
            got = t.lookup(k)
            assert list(reversed(got)) == rows, (k, got)
        assert t.lookup(999) == []


def test_fixed_table_insert_previous_kat(dfp):
    """fixed_table.rs:1411-1419: insert returns the previous value:
    (1,1)->None, (1,2)->1, (4023,4)->None, (1,5)->2, (4023,6)->4. Rows inserted in
    that order; chain_links gives each row's previous row with the same key."""
    keys = np.array([1, 1, 4023, 1, 4023], dtype=np.int64)
    values = [1, 2, 4, 5, 6]
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(keys)
        prev = t.chain_links(len(keys))
    got = [None if prev[i] < 0 else values[prev[i]] for i in range(len(keys))]
    assert got == [None, 1, None, 2, 4]


def test_zero_and_extreme_keys(dfp, oracle_mod, probe_mode):
    """fixed_table.rs:1399-1409 (zero hash storable) + the sentinel-colliding key."""
    bk = np.array([0, I64_MIN, np.iinfo(np.int64).max, -1, 0, I64_MIN], dtype=np.int64)
    pk = np.array([I64_MIN, 0, 5, -1, np.iinfo(np.int64).max, I64_MIN], dtype=np.int64)
    b, p, _ = gpu_join(dfp, bk, pk)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


def test_inner_join_with_nulls_kat(dfp, oracle_mod):
    """src/lib.rs:149-193: [1,2,NULL] join [NULL,2,3] -> only 2."""
    b, p, _ = gpu_join(dfp, np.array([1, 2, 0], np.int32), np.array([0, 2, 3], np.int32),
                       [True, True, False], [False, True, True], key_type="int32")
    assert list(b) == [1] and list(p) == [1]


def test_inner_join_without_matches_kat(dfp):
    """src/lib.rs:210-246: no matching keys -> 0 rows."""
    b, p, _ = gpu_join(dfp, np.array([1, 2, 0], np.int32), np.array([0, 4, 5], np.int32),
                       [True, True, False], [False, True, True], key_type="int32")
    assert len(b) == 0


def test_chain_order_across_partitions_kat(dfp):
    """src/utils/concurrent_self_hash_join_map.rs:321-373: rows of one key appended by
    two partitions; the chain lists every row newest first. Canonical numbering puts
    partition 0's rows first, so the chain is the descending list of all rows."""
    with dfp.HashTable(2, "int64", 0) as t:
        t.append(0, np.array([1, 7, 1, 1], np.int64))
        t.append(1, np.array([1, 1, 3, 1], np.int64))
        t.finish_all()
        assert t.partition_offset(1) == 4
        assert t.lookup(1) == [7, 5, 4, 3, 2, 0]


# ---- randomized parity vs the oracle -------------------------------------------

@pytest.mark.parametrize("nb,np_,krange,null_frac,key_type", [
    (0, 100, 10, 0.0, "int64"),
    (100, 0, 10, 0.0, "int64"),
    (1, 1, 1, 0.0, "int64"),
    (1000, 4095, 700, 0.0, "int64"),
    (4096, 4096, 3000, 0.1, "int64"),
    (5000, 4097, 10000, 0.2, "int32"),
    (100003, 300007, 60000, 0.05, "int64"),
    (50000, 123457, 20000, 0.0, "int32"),
    (200000, 1000000, 400000, 0.01, "int64"),
    (300000, 200000, 3000, 0.0, "int64"),  # dense, > 8192 rows per 8192-value block
])
def test_random_parity(dfp, oracle_mod, probe_mode, nb, np_, krange, null_frac, key_type):
    """Small key ranges take the direct-addressed layout's one-level build (hashed under
    the *-hashed modes)."""
    rng = np.random.default_rng(nb * 31 + np_)
    dt = np.int64 if key_type == "int64" else np.int32
    bk = rng.integers(-krange // 2, krange, nb).astype(dt)
    pk = rng.integers(-krange // 2, krange, np_).astype(dt)
    bv = rng.random(nb) >= null_frac if null_frac else None
    pv = rng.random(np_) >= null_frac if null_frac else None
    b, p, _ = gpu_join(dfp, bk, pk, bv, pv, key_type=key_type)
    ob, op = oracle_mod.inner_join(bk, pk, bv, pv)
    assert_same(b, p, ob, op)


def test_host_input_parity(dfp, oracle_mod):
    rng = np.random.default_rng(5)
    bk = rng.integers(0, 3000, 10000).astype(np.int64)
    pk = rng.integers(0, 6000, 20000).astype(np.int64)
    b, p, _ = gpu_join(dfp, bk, pk, device_input=False)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


def test_multi_partition_canonical_numbering(dfp, oracle_mod, probe_mode):
    rng = np.random.default_rng(11)
    bk = rng.integers(0, 5000, 30000).astype(np.int64)
    pk = rng.integers(0, 9000, 40000).astype(np.int64)
    parts = [0, 7000, 7000, 19000, 30000]  # includes an empty partition
    b, p, _ = gpu_join(dfp, bk, pk, parts=parts)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


@pytest.mark.parametrize("dups", [17, 300, 5000, 70000])
def test_heavy_duplicates(dfp, oracle_mod, probe_mode, dups):
    """Segments > 16 rows (LDS sort) and > 4096 rows (ordered rescan)."""
    rng = np.random.default_rng(dups)
    hot = np.full(dups, 42, np.int64)
    other = rng.integers(0, 1000, 20000).astype(np.int64)
    bk = np.concatenate([other[:10000], hot, other[10000:]])
    rng.shuffle(bk)
    pk = np.array([42, 1, 42, 999, 5000, 42], np.int64)
    b, p, st = gpu_join(dfp, bk, pk)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)
    assert st["max_key_rows"] >= dups


def test_chain_links_match_reference_semantics(dfp):
    """Each valid row's link is the next older valid row with the same key (the
    reference's overflow chain at parallelism 1 with exact keys); nulls never chain."""
    rng = np.random.default_rng(3)
    bk = rng.integers(0, 2000, 20000).astype(np.int64)
    bv = rng.random(len(bk)) > 0.1
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(torch.from_numpy(bk).cuda(), bv)
        prev = t.chain_links(len(bk))
    last = {}
    want = np.full(len(bk), -1, np.int64)
    for i, (k, v) in enumerate(zip(bk.tolist(), bv.tolist())):
        if v:
            want[i] = last.get(k, -1)
            last[k] = i
    assert np.array_equal(prev, want)


def test_exponential_keys_parity(dfp, oracle_mod, probe_mode):
    """benches/exponential_distribution.rs key distribution (src/api_utils.rs:15-23)."""
    bk = oracle_mod.make_exponential_int_array(0, 200000).astype(np.int64)
    pk = oracle_mod.uniform_keys(500000, 0xC0FFEE, 200000)
    b, p, st = gpu_join(dfp, bk, pk)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)
    assert st["dup_keys"] > 0


def _run_keys(rng, nkeys=3000, maxrun=12):
    """Sorted build keys in runs of 1..maxrun rows (consecutive rows per key: run refs for
    2..9 rows, dup_rows segments beyond), a few keys whose rows are not consecutive, and
    probe keys over and beyond the build range."""
    lens = rng.integers(1, maxrun + 1, nkeys)
    bk = np.repeat(np.arange(nkeys, dtype=np.int64) * 3, lens)
    # keys whose rows are split (not a run): the same key again further on
    bk = np.concatenate([bk, bk[:: max(1, len(bk) // 50)]])
    pk = rng.integers(-5, nkeys * 3 + 5, 40000).astype(np.int64)
    return bk, pk


def test_run_refs_parity(dfp, oracle_mod, probe_mode):
    """Run refs (hj_device.h): keys with consecutive rows keep them in the ref (2..9 rows),
    longer or split ones keep their dup_rows segment; nulls break runs; two partitions
    number rows across the partition boundary. Bit-exact against the oracle under every
    probe strategy, table layout and tile size."""
    rng = np.random.default_rng(61)
    bk, pk = _run_keys(rng)
    b, p, st = gpu_join(dfp, bk, pk)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)
    assert st["max_key_rows"] >= 12
    bv = rng.random(len(bk)) > 0.05
    n = len(bk)
    b, p, _ = gpu_join(dfp, bk, pk, bvalid=bv, parts=[0, n // 3, n])
    ob, op = oracle_mod.inner_join(bk, pk, bv, None)
    assert_same(b, p, ob, op)


def test_run_refs_chain_links_and_stats(dfp):
    """hj_table_chain_links and hj_table_stats decode run refs: sorted keys in runs."""
    rng = np.random.default_rng(62)
    bk, _ = _run_keys(rng, nkeys=2000)
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(torch.from_numpy(bk).cuda())
        prev = t.chain_links(len(bk))
        st = t.stats()
    last = {}
    want = np.full(len(bk), -1, np.int64)
    for i, k in enumerate(bk.tolist()):
        want[i] = last.get(k, -1)
        last[k] = i
    assert np.array_equal(prev, want)
    vals, cnt = np.unique(bk, return_counts=True)
    assert st["distinct_keys"] == len(vals) and st["dup_keys"] == int((cnt > 1).sum())
    assert st["dup_rows"] == int(cnt[cnt > 1].sum()) and st["max_key_rows"] == int(cnt.max())


@pytest.mark.parametrize("pmode", [4, 3])
def test_run_refs_rows_past_2_24(dfp, oracle_mod, pmode):
    """Runs whose top row is >= 2^24 keep their dup_rows segment (the run ref holds 24
    bits): a 17.5 M-row sorted build with keys in pairs, probed across the 2^24 boundary."""
    L = dfp.load()
    old = L.hj_set_probe_mode(pmode)
    try:
        nb = 17_500_000
        bk = np.arange(nb, dtype=np.int64) // 2
        pk = np.concatenate([np.arange(8_300_000, 8_450_000, dtype=np.int64),
                             np.arange(0, 10_000, dtype=np.int64), np.array([nb // 2 - 1, nb // 2 + 3])])
        b, p, st = gpu_join(dfp, bk, pk)
    finally:
        L.hj_set_probe_mode(old)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


@pytest.mark.parametrize("frag_t", ["512", "1024"])
def test_frag_build_workgroup_sizes(dfp, oracle_mod, monkeypatch, frag_t):
    """Both forms of the dense frag build (DFP_HJ_FRAG_T: 512 threads x 16 rows, the
    default, or 1024 x 8): exponential keys (duplicate passes in most blocks), a block
    with more rows than the registers hold (the spill path) and nulls, against the oracle."""
    monkeypatch.setenv("DFP_HJ_FRAG_T", frag_t)
    rng = np.random.default_rng(int(frag_t))
    bk = np.concatenate([oracle_mod.make_exponential_int_array(0, 300000).astype(np.int64),
                         np.full(20000, 123457, np.int64)])
    rng.shuffle(bk)
    bv = rng.random(len(bk)) > 0.02
    pk = oracle_mod.uniform_keys(400000, 0xBEEF, 320000)
    pk[::1000] = 123457
    b, p, st = gpu_join(dfp, bk, pk, bvalid=bv)
    ob, op = oracle_mod.inner_join(bk, pk, bv, None)
    assert_same(b, p, ob, op)
    assert st["buckets"] == 0 and st["dup_keys"] > 0 and st["max_key_rows"] >= 19000


@pytest.mark.parametrize("layout", [0, 1, 2])
def test_stats(dfp, layout):
    L = dfp.load()
    old = L.hj_set_build_mode(layout)
    try:
        bk = np.array([5, 5, 5, 6, 7, 7], np.int64)
        with dfp.HashTable(1, "int64", 0) as t:
            t.build(bk, np.array([1, 1, 1, 1, 1, 0], bool))
            s = t.stats()
    finally:
        L.hj_set_build_mode(old)
    assert s["build_rows"] == 6 and s["inserted_rows"] == 5
    assert s["distinct_keys"] == 3 and s["dup_keys"] == 1 and s["dup_rows"] == 3 and s["max_key_rows"] == 3
    # layouts 0 and 2 choose the direct-addressed table for this dense range (3 values, 6 rows)
    assert (s["buckets"] == 0) == (layout != 1)


# ---- full-size properties (BASELINE configs) -------------------------------------

def test_c2_full_size_properties(dfp, oracle_mod):
    """C2 (10^7 unique build keys x 10^8 uniform probe keys over 2*10^7): every probe key
    < 10^7 matches exactly once, at build row k * inv(7368787) mod 10^7; check count,
    order and a sample of values against the closed form."""
    B, P, R = 10**7, 10**8, 2 * 10**7
    dev = torch.device("cuda", 0)
    lib = dfp.load()
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, s) == 0
    assert lib.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, R, s) == 0
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        b, p = t.probe(pk, device_output=True)
    expected = int((pk < B).sum().item())
    assert b.numel() == expected
    # probe indices strictly ascending (unique build keys -> at most one match per row)
    assert bool((p[1:] > p[:-1]).all().item())
    # every emitted pair has equal keys
    assert bool((bk[b] == pk[p.long()]).all().item())
    inv = pow(7368787, -1, B)
    sample = torch.randint(0, b.numel(), (10000,), device=dev)
    keys = pk[p[sample].long()].cpu().numpy().astype(object)
    want = np.array([(int(k) * inv) % B for k in keys], dtype=np.int64)
    assert np.array_equal(b[sample].cpu().numpy(), want)


@pytest.mark.parametrize("layout", [0, 1])
def test_c1b_full_pairs(dfp, oracle_mod, layout):
    """C1b (BASELINE.json configs[0] shape): 2^20 unique build keys x 2^20 probe keys over
    2^21, every pair against the oracle, in both table layouts (auto probe strategy)."""
    L = dfp.load()
    old = L.hj_set_build_mode(layout)
    try:
        n = 1 << 20
        bk = oracle_mod.perm_keys(n, 7368787, n)
        pk = oracle_mod.uniform_keys(n, 0xC0FFEE, 2 * n)
        b, p, st = gpu_join(dfp, bk, pk)
        assert (st["buckets"] == 0) == (layout == 0)
        ob, op = oracle_mod.inner_join(bk, pk)
        assert_same(b, p, ob, op)
    finally:
        L.hj_set_build_mode(old)


MIX_MUL_I64 = 0x9E3779B97F4A7C15 - (1 << 64)  # odd: k -> k * M (mod 2^64) is a bijection


def test_c2h_full_size_equals_c2(dfp):
    """C2h = C2 with both sides' keys mapped by the bijection k -> k * M (mod 2^64): the
    keys spread over the int64 domain, so the build takes the hashed bucket table and
    the probe its sliced hashed pipeline (auto choice), yet the pairs must be exactly
    C2's (direct-addressed table, sliced probe): same count, same order, same values."""
    B, P, R = 10**7, 10**8, 2 * 10**7
    dev = torch.device("cuda", 0)
    lib = dfp.load()
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, s) == 0
    assert lib.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, R, s) == 0
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        assert t.stats()["buckets"] == 0
        b0, p0 = t.probe(pk, device_output=True)
    bk.mul_(MIX_MUL_I64)
    pk.mul_(MIX_MUL_I64)
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        st = t.stats()
        assert st["buckets"] > 0 and st["buckets"] <= 2047 * 2048  # hashed, within the sliced limit
        b1, p1 = t.probe(pk, device_output=True)
    assert b1.numel() == b0.numel() == 49_999_816
    assert torch.equal(p0, p1) and torch.equal(b0, b1)


@pytest.mark.parametrize("nb,np_,dup_frac,null_frac,key_type", [
    (2_000_000, 3_000_001, 0.0, 0.0, "int64"),   # ~390 slices, ragged last tile
    (1_500_000, 2_000_000, 0.3, 0.01, "int64"),  # duplicated keys (inline meta counts and more)
    (800_000, 1_000_000, 0.1, 0.02, "int32"),    # int32 keys over the whole int32 domain
])
def test_hashed_sliced_auto(dfp, oracle_mod, nb, np_, dup_frac, null_frac, key_type):
    """Keys over the whole integer domain (hashed table), probe side large enough for the
    auto choice to take the sliced hashed pipeline; INT64_MIN / zero included."""
    L = dfp.load()
    old_p, old_b = L.hj_set_probe_mode(0), L.hj_set_build_mode(0)
    try:
        rng = np.random.default_rng(nb + np_)
        info = np.iinfo(np.int64 if key_type == "int64" else np.int32)
        dt = np.int64 if key_type == "int64" else np.int32
        distinct = rng.integers(info.min, info.max, nb, dtype=np.int64).astype(dt)
        bk = distinct.copy()
        nd = int(nb * dup_frac)
        if nd:
            bk[:nd] = distinct[rng.integers(nd, nb, nd)]  # repeated keys
            bk[nd:nd + 70] = distinct[-1]                 # one key with > 63 rows
        bk[-2:] = [info.min, 0]
        pk = np.concatenate([bk[rng.integers(0, nb, np_ // 2)],
                             rng.integers(info.min, info.max, np_ - np_ // 2, dtype=np.int64).astype(dt)])
        rng.shuffle(pk)
        pk[:3] = [info.min, 0, info.max]
        bv = rng.random(nb) >= null_frac if null_frac else None
        pv = rng.random(np_) >= null_frac if null_frac else None
        b, p, st = gpu_join(dfp, bk, pk, bv, pv, key_type=key_type)
        assert st["buckets"] > 0
        ob, op = oracle_mod.inner_join(bk, pk, bv, pv)
        assert_same(b, p, ob, op)
    finally:
        L.hj_set_probe_mode(old_p)
        L.hj_set_build_mode(old_b)


@pytest.mark.parametrize("lf,dup_frac", [(0.75, 0.0), (0.8, 0.25)])
def test_hashed_sliced_high_load(dfp, oracle_mod, monkeypatch, lf, dup_frac):
    """Hashed table at a high load factor: many home buckets were passed full, so many
    probe rows continue past them — the sliced lookup queues those per wave and flushes the
    queue mid-window when it fills (r05); displaced keys with duplicated rows (counts in the
    bucket meta or the segment header) and key 0 among them. Same pairs as the oracle."""
    monkeypatch.setenv("DFP_HJ_LOAD_FACTOR", str(lf))
    L = dfp.load()
    old_p = L.hj_set_probe_mode(4)  # the sliced probe
    try:
        rng = np.random.default_rng(int(lf * 100))
        distinct = rng.integers(-(2**63), 2**63 - 1, 1_200_000, dtype=np.int64)
        bk = distinct.copy()
        nd = int(len(bk) * dup_frac)
        if nd:
            bk[:nd] = distinct[rng.integers(nd, len(bk), nd)]
            bk[nd:nd + 90] = distinct[-1]  # one key with > 63 rows
        bk[-1] = 0
        pk = np.concatenate([bk[rng.integers(0, len(bk), 1_500_000)],
                             rng.integers(-(2**63), 2**63 - 1, 1_500_000, dtype=np.int64)])
        rng.shuffle(pk)
        pk[:2] = [0, 0]
        b, p, st = gpu_join(dfp, bk, pk)
        assert st["buckets"] > 0
        ob, op = oracle_mod.inner_join(bk, pk)
        assert_same(b, p, ob, op)
    finally:
        L.hj_set_probe_mode(old_p)


@pytest.mark.parametrize("layout", [0, 2])
def test_hashed_build_every_key_twice(dfp, oracle_mod, layout):
    """Hashed table whose every key has two rows (plus a few with 3..40): each 1024-bucket
    build slice then has more duplicated keys than its LDS directory holds, so the frag
    build keeps those directories in the spill pool (layout 0); layout 2 is the histogram
    path. Same pairs as the oracle."""
    L = dfp.load()
    old = L.hj_set_build_mode(layout)
    try:
        rng = np.random.default_rng(41)
        d = rng.integers(-(2**63), 2**63 - 1, 700_000, dtype=np.int64)
        bk = np.concatenate([d, d, d[:1000], np.full(40, d[7])])
        rng.shuffle(bk)
        pk = np.concatenate([d[rng.integers(0, len(d), 900_000)], rng.integers(-(2**63), 2**63 - 1, 300_000)])
        b, p, st = gpu_join(dfp, bk, pk)
        assert st["buckets"] > 0 and st["dup_keys"] == 700_000
        ob, op = oracle_mod.inner_join(bk, pk)
        assert_same(b, p, ob, op)
    finally:
        L.hj_set_build_mode(old)


@pytest.mark.parametrize("lo_pad,hi_pad", [(0, 0), (1000, 7), (10**12, 10**12)])
def test_build_key_range_hint(dfp, oracle_mod, lo_pad, hi_pad):
    """hj_build_key_range: the caller's range (exact, a little wider, far wider -> the
    hashed layout) replaces the key-range reduction; pairs equal the oracle's."""
    rng = np.random.default_rng(lo_pad % 97)
    bk = rng.integers(-5000, 400_000, 300_000).astype(np.int64)
    pk = rng.integers(-6000, 410_000, 1_000_000).astype(np.int64)
    with dfp.HashTable(1, "int64", 0) as t:
        t.append(0, torch.from_numpy(bk).cuda())
        t.key_range(int(bk.min()) - lo_pad, int(bk.max()) + hi_pad)
        t.finish(0)
        st = t.stats()
        b, p = t.probe(torch.from_numpy(pk).cuda(), device_output=True)
    assert (st["buckets"] == 0) == (lo_pad < 10**6)  # far wider than 8x the rows: hashed
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob)
    assert np.array_equal(p.cpu().numpy().view(np.uint32), op)


@pytest.mark.parametrize("base", [0, -(2**62), 2**62 - 10**6, 123_456_789_012])
def test_build_key_base(dfp, oracle_mod, base):
    """hj_build_key_base: an int32 table built from offsets key - base (with duplicates and
    nulls) takes int64 probe keys afterwards; pairs equal the oracle's over the int64 keys,
    and get_iter answers int64 keys."""
    rng = np.random.default_rng(abs(base) % 1000)
    off = rng.integers(0, 400_000, 300_000)
    bk = off + base
    pk = rng.integers(-50_000, 450_000, 1_000_000) + base
    valid = rng.random(off.size) > 0.05
    with dfp.HashTable(1, "int32", 0) as t:
        t.append(0, torch.from_numpy(off.astype(np.int32)).cuda(), valid=torch.from_numpy(valid).cuda())
        t.key_range(0, int(off.max()))
        t.key_base(base)
        t.finish(0)
        assert t.stats()["buckets"] == 0  # direct-addressed
        b, p = t.probe(torch.from_numpy(pk).cuda(), device_output=True)
        k0 = int(bk[valid][0])
        rows = t.lookup(k0)
    ob, op = oracle_mod.inner_join(bk, pk, valid)
    assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob)
    assert np.array_equal(p.cpu().numpy().view(np.uint32), op)
    want = np.nonzero((bk == k0) & valid)[0][::-1]
    assert rows == [int(x) for x in want]


def test_build_key_base_needs_dense(dfp):
    """A key range wider than 8 x the rows cannot be re-keyed: the build fails loudly."""
    from datafusion_parallelism_amd import HjError

    off = np.arange(0, 10_000 * 100, 100, dtype=np.int32)
    t = dfp.HashTable(1, "int32", 0)
    try:
        t.append(0, torch.from_numpy(off).cuda())
        t.key_base(5)
        with pytest.raises(HjError, match="direct-addressed"):
            t.finish(0)
    finally:
        t.close()


def test_c3_full_size_digest(dfp, oracle_mod):
    """C3 (10^7 exponential build keys x 10^8 uniform probe keys): the pair count and
    per-probe-row match counts against the closed form multiplicity of each key."""
    B, P = 10**7, 10**8
    bk_np = oracle_mod.make_exponential_int_array(0, B).astype(np.int64)
    mult = np.bincount(bk_np, minlength=B)
    dev = torch.device("cuda", 0)
    lib = dfp.load()
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    assert lib.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, B, torch.cuda.current_stream().cuda_stream) == 0
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(torch.from_numpy(bk_np).cuda())
        st = t.stats()
        b, p = t.probe(pk, device_output=True)
    assert st["distinct_keys"] == 6603254 and st["max_key_rows"] == 6
    expected = int(torch.from_numpy(mult).cuda()[pk].sum().item())
    assert b.numel() == expected
    assert bool((torch.from_numpy(bk_np).cuda()[b] == pk[p.long()]).all().item())
    # canonical order: probe ascending, build strictly descending within a probe row
    pl = p.long()
    assert bool((pl[1:] >= pl[:-1]).all().item())
    same = pl[1:] == pl[:-1]
    assert bool((b[1:][same] < b[:-1][same]).all().item())


@pytest.mark.parametrize("ids_u31", [False, True])
@pytest.mark.parametrize("dups", [1, 300, 5000])
def test_explicit_build_ids(dfp, oracle_mod, probe_mode, ids_u31, dups):
    """Explicit (global) build ids, as the multi-GPU exchange hands them over: pairs carry
    the ids, ordered by id descending within a probe row. ids_u31 stores the ids in place
    of row numbers (HJ_IDS_U31); without it they are gathered from the id array. Covers
    segments sorted in registers, in LDS and by the ordered rescan (> 4096 rows)."""
    rng = np.random.default_rng(dups + ids_u31)
    bk = np.concatenate([rng.integers(0, 3000, 20000), np.full(dups, 77)]).astype(np.int64)
    rng.shuffle(bk)
    bv = rng.random(len(bk)) > 0.05
    ids = np.cumsum(rng.integers(1, 50, len(bk))).astype(np.int64) + 10**6  # ascending, sparse
    pk = np.concatenate([rng.integers(0, 4000, 30000), [77, 77]]).astype(np.int64)
    with dfp.HashTable(2, "int64", 0) as t:
        h = len(bk) // 2
        t.append(0, torch.from_numpy(bk[:h].copy()).cuda(), bv[:h], ids=torch.from_numpy(ids[:h].copy()).cuda(),
                 ids_u31=ids_u31)
        t.append(1, torch.from_numpy(bk[h:].copy()).cuda(), bv[h:], ids=torch.from_numpy(ids[h:].copy()).cuda(),
                 ids_u31=ids_u31)
        t.finish_all()
        b, p = t.probe(torch.from_numpy(pk).cuda())
    ob, op = oracle_mod.inner_join(bk, pk, bv, None)
    assert_same(b, p, ids[ob.astype(np.int64)].astype(np.uint64), op)


@pytest.mark.parametrize("pmode", [0, 4])
def test_large_build_120m_rows(dfp, pmode):
    """A 1.2e8-row build (past the 5.9e7-row limit of round-1's first table geometry):
    size-independent properties on the GPU - every pair has equal keys, every probe key
    below N matches exactly its one build row (a permutation build side), canonical
    order, no pair for keys >= N. pmode 4: the sliced probe over its 3663 slices (two
    passes over slice ranges); 0: the auto choice."""
    L = dfp.load()
    old_p = L.hj_set_probe_mode(pmode)
    try:
        _large_build_120m(dfp)
    finally:
        L.hj_set_probe_mode(old_p)


def _large_build_120m(dfp):
    L = dfp.load()
    N, P = 120_000_000, 10_000_000
    s = torch.cuda.current_stream().cuda_stream
    bk = torch.empty(N, dtype=torch.int64, device="cuda")
    assert L.hj_gen_perm_keys(bk.data_ptr(), N, 7368787, N, s) == 0
    pk = torch.empty(P, dtype=torch.int64, device="cuda")
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 99, 2 * N, s) == 0
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        b, p = t.probe(pk, device_output=True)
        st = t.stats()
    assert st["distinct_keys"] == N and st["dup_keys"] == 0
    want = int((pk < N).sum())
    assert b.numel() == want
    pl = p.to(torch.int64)
    assert bool((bk[b] == pk[pl]).all())
    assert bool((pl[1:] > pl[:-1]).all())  # unique build keys: one pair per matched row, ascending
    del bk, pk, b, p
    torch.cuda.empty_cache()


@pytest.mark.parametrize("bmode", [0, 2])
@pytest.mark.parametrize("nb,krange", [(2_200_000, 17_600_000), (2_000_000, 16_000_000)])
def test_dense_build_levels(dfp, oracle_mod, nb, krange, bmode):
    """Direct-addressed builds on both sides of the one-level limit (2048 blocks of 8192
    key values): 17.6 M values take the two-level partition, 16 M the one-level one (the
    tile-local partition under build mode 0, histogram + scatter under mode 2)."""
    L = dfp.load()
    old = L.hj_set_build_mode(bmode)
    try:
        _dense_build_levels(dfp, oracle_mod, nb, krange)
    finally:
        L.hj_set_build_mode(old)


def _dense_build_levels(dfp, oracle_mod, nb, krange):
    rng = np.random.default_rng(nb)
    bk = rng.integers(0, krange, nb)
    bk[:3] = [0, krange - 1, krange - 1]
    pk = rng.integers(-1000, krange + 1000, 1_000_000)
    b, p, st = gpu_join(dfp, bk, pk)
    assert st["buckets"] == 0  # direct-addressed
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


# ---- sliced probe (LDS lookups, hj_set_probe_mode 4) --------------------------------

@pytest.fixture(params=[14, 15], ids=["t14", "t15"])
def sliced_mode(dfp, request):
    """The sliced probe with 2^14- and 2^15-row probe tiles (hj_set_probe_tile_log)."""
    L = dfp.load()
    old_p = L.hj_set_probe_mode(4)
    old_b = L.hj_set_build_mode(0)
    old_t = L.hj_set_probe_tile_log(request.param)
    yield
    L.hj_set_probe_mode(old_p)
    L.hj_set_build_mode(old_b)
    L.hj_set_probe_tile_log(old_t)


@pytest.mark.parametrize("nb,krange,np_,null_frac,key_type", [
    (9_000_000, 2047 * 32768, 2_000_000, 0.0, "int64"),     # 2047 slices: the largest sliced table
    (9_000_000, 2048 * 32768, 1_000_000, 0.0, "int64"),     # 2048 slices: past round 2's 2047-slice limit
    (17_000_000, 4100 * 32768, 2_000_000, 0.01, "int64"),   # 4100 slices: two passes over slice ranges, nulls
    (5_000_000, 2047 * 16384, 2_000_000, 0.0, "int64"),     # ~1024 slices
    (300_000, 1_000_000, 3_000_001, 0.02, "int32"),         # nulls, ragged last tile
    (2_000_000, 600_000, 1_500_000, 0.0, "int64"),          # duplicated keys (counts <= 15 and more)
])
def test_sliced_probe_parity(dfp, oracle_mod, sliced_mode, nb, krange, np_, null_frac, key_type):
    rng = np.random.default_rng(nb + np_)
    dt = np.int64 if key_type == "int64" else np.int32
    bk = rng.integers(0, krange, nb).astype(dt)
    bk[:2] = [0, krange - 1]
    if krange < nb:  # a few keys with > 15 rows (count read from dup_rows)
        bk[2:2 + 40] = 17
        bk[100:100 + 300] = krange // 2
    pk = rng.integers(-1000, krange + 1000, np_).astype(dt)
    bv = rng.random(nb) >= null_frac if null_frac else None
    pv = rng.random(np_) >= null_frac if null_frac else None
    b, p, st = gpu_join(dfp, bk, pk, bv, pv, key_type=key_type)
    assert st["buckets"] == 0  # direct-addressed
    ob, op = oracle_mod.inner_join(bk, pk, bv, pv)
    assert_same(b, p, ob, op)


@pytest.mark.parametrize("nb,np_,dup_frac", [(12_000_000, 2_000_000, 0.0), (11_000_000, 1_500_001, 0.2),
                                               (22_000_000, 2_000_000, 0.05)])
def test_sliced_hashed_multipass_parity(dfp, oracle_mod, sliced_mode, nb, np_, dup_frac):
    """Hashed tables past round 2's 2047 slices of 2048 buckets (12 M keys at load 0.5 =
    2344 slices: one pass of up to 4095), and past one pass (22 M keys = 4297 slices: two
    passes over slice ranges, appending to the tiles' entries, one emission); duplicated
    keys and key 0 (the side bucket, slice 0) included."""
    rng = np.random.default_rng(nb)
    distinct = rng.integers(-(2**63), 2**63 - 1, nb, dtype=np.int64)
    bk = distinct.copy()
    nd = int(nb * dup_frac)
    if nd:
        bk[:nd] = distinct[rng.integers(nd, nb, nd)]
    bk[-1] = 0
    pk = np.concatenate([bk[rng.integers(0, nb, np_ // 2)], rng.integers(-(2**63), 2**63 - 1, np_ - np_ // 2)])
    pk[:2] = [0, bk[5]]
    b, p, st = gpu_join(dfp, bk, pk)
    assert st["buckets"] > 2047 * 2048  # beyond round 2's sliced limit
    ob, op = oracle_mod.inner_join(bk, pk)
    assert_same(b, p, ob, op)


@pytest.mark.parametrize("pmode", [4, 0])
def test_c2h_40m_multipass_closed_form(dfp, pmode):
    """A 4*10^7-key hashed build (16 M buckets = 7813 slices) probed with 10^8 rows: C2's
    closed form under the bijection k -> k * M — probe keys below B match exactly the row
    k * inv(7368787) mod B; count, order, values. pmode 4: the sliced probe in two passes
    over slice ranges; 0: the auto choice (the fused probe for a two-pass hashed table)."""
    lib = dfp.load()
    old_p = lib.hj_set_probe_mode(pmode)
    try:
        _c2h_40m(dfp)
    finally:
        lib.hj_set_probe_mode(old_p)


def _c2h_40m(dfp):
    B, P = 40_000_000, 10**8
    dev = torch.device("cuda", 0)
    lib = dfp.load()
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, s) == 0
    assert lib.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, s) == 0
    expected = int((pk < B).sum().item())
    sample = torch.randint(0, P, (20000,), device=dev)
    raw = pk[sample].cpu().numpy()
    bk.mul_(MIX_MUL_I64)
    pk.mul_(MIX_MUL_I64)
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        st = t.stats()
        assert st["buckets"] > 4095 * 2048  # two passes of up to 4095 slices
        b, p = t.probe(pk, device_output=True)
    assert b.numel() == expected
    pl = p.long()
    assert bool((pl[1:] > pl[:-1]).all().item())  # one pair per matched row, ascending
    assert bool((bk[b] == pk[pl]).all().item())
    # closed form on a sample of probe rows: row r matches iff raw key < B, at k * inv mod B
    inv = pow(7368787, -1, B)
    hit = torch.zeros(P, dtype=torch.int64, device=dev).index_fill_(0, pl, 1)
    where = torch.full((P,), -1, dtype=torch.int64, device=dev).index_copy_(0, pl, b)
    h, w = hit[sample].cpu().numpy(), where[sample].cpu().numpy()
    for k, hh, ww in zip(raw.tolist(), h.tolist(), w.tolist()):
        assert hh == (k < B)
        if k < B:
            assert ww == (k * inv) % B
    del bk, pk, b, p, hit, where
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", [4, 3])
def test_probe_overlaps_build_on_other_stream(dfp, oracle_mod, mode):
    """Build on stream A, probe launched at once on stream B (no host or stream sync in
    between): the probe orders itself after the build only at its first table read (the
    sliced probe's partition runs while the build may still be running). Several
    back-to-back tables, as the bench's pipeline does."""
    L = dfp.load()
    old_p = L.hj_set_probe_mode(mode)
    try:
        rng = np.random.default_rng(5 + mode)
        dev = torch.device("cuda", 0)
        nb, krange, np_ = 3_000_000, 4_000_000, 4_000_000
        sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        ws = torch.empty(dfp.HashTable.workspace_bytes(np_), dtype=torch.uint8, device=dev)
        for it in range(3):
            bk = rng.integers(0, krange, nb).astype(np.int64)
            pk = rng.integers(-1000, krange + 1000, np_).astype(np.int64)
            bk_d, pk_d = torch.from_numpy(bk).to(dev), torch.from_numpy(pk).to(dev)
            torch.cuda.synchronize(dev)
            cap = 2 * np_
            ob = torch.empty(cap, dtype=torch.int64, device=dev)
            op = torch.empty(cap, dtype=torch.int32, device=dev)
            dt = torch.zeros(1, dtype=torch.int64, device=dev)
            torch.cuda.synchronize(dev)
            with dfp.HashTable(1, "int64", 0) as t:
                with torch.cuda.stream(sa):
                    t.append(0, bk_d)
                    t.finish(0)
                t.probe_async(pk_d.data_ptr(), np_, ob.data_ptr(), op.data_ptr(), cap, dt.data_ptr(),
                              ws.data_ptr(), sb.cuda_stream)
                sb.synchronize()
                total = int(dt.item())
                b = ob[:total].cpu().numpy().astype(np.uint64)
                p = op[:total].cpu().numpy().view(np.uint32)
            xb, xp = oracle_mod.inner_join(bk, pk)
            assert_same(b, p, xb, xp)
    finally:
        L.hj_set_probe_mode(old_p)


def test_sliced_probe_ids_unaligned(dfp, oracle_mod, sliced_mode):
    """hj_probe_async_ids (explicit probe ids, the multi-GPU path) on a key pointer that
    is 8- but not 16-byte aligned (scalar key loads), with explicit build ids."""
    rng = np.random.default_rng(77)
    nb, krange, np_ = 400_000, 2_000_000, 1_000_003
    bk = rng.integers(0, krange, nb).astype(np.int64)
    ids = np.cumsum(rng.integers(1, 9, nb)).astype(np.int64)
    pk = rng.integers(0, krange, np_ + 1).astype(np.int64)
    pids = rng.integers(0, 2**32 - 1, np_, dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda", 0)
    with dfp.HashTable(1, "int64", 0) as t:
        t.append(0, torch.from_numpy(bk).to(dev), None, ids=torch.from_numpy(ids).to(dev))
        t.finish_all()
        pk_d = torch.from_numpy(pk).to(dev)
        keys_ptr = pk_d.data_ptr() + 8  # rows 1..np_
        assert keys_ptr % 16 == 8
        pid_d = torch.from_numpy(pids.view(np.int32)).to(dev)
        cap = 2 * np_
        ob = torch.empty(cap, dtype=torch.int64, device=dev)
        op = torch.empty(cap, dtype=torch.int32, device=dev)
        dt = torch.zeros(1, dtype=torch.int64, device=dev)
        ws = torch.empty(t.workspace_bytes(np_), dtype=torch.uint8, device=dev)
        t.probe_async(keys_ptr, np_, ob.data_ptr(), op.data_ptr(), cap, dt.data_ptr(), ws.data_ptr(),
                      probe_ids_ptr=pid_d.data_ptr())
        total = int(dt.item())
        b = ob[:total].cpu().numpy().astype(np.uint64)
        p = op[:total].cpu().numpy().view(np.uint32)
    xb, xp = oracle_mod.inner_join(bk, pk[1:])
    assert_same(b, p, ids[xb.astype(np.int64)].astype(np.uint64), pids[xp.astype(np.int64)])


def _probe_async_base(dfp, t, pk, base):
    """hj_probe_async_base on device buffers -> (build idx, probe idx) as numpy."""
    n = len(pk)
    keys = torch.from_numpy(np.ascontiguousarray(pk)).cuda()
    cap = max(4 * n, 16)
    ob = torch.empty(cap, dtype=torch.int64, device="cuda")
    op = torch.empty(cap, dtype=torch.int32, device="cuda")
    ws = torch.empty(dfp.HashTable.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    dt = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    t.probe_async(keys.data_ptr(), n, ob.data_ptr(), op.data_ptr(), cap, dt.data_ptr(), ws.data_ptr(), s,
                  probe_base=base)
    m = int(dt.item())
    assert m <= cap
    return ob[:m].cpu().numpy().astype(np.uint64), op[:m].cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("base", [1, 3_000_000_000])
def test_probe_base(dfp, oracle_mod, probe_mode, base):
    """hj_probe_async_base: probe_idx = probe_base + row (a rank's or a batch's rows of a
    longer probe stream), identical pairs otherwise; a base past 2^32 - n is refused."""
    rng = np.random.default_rng(base % 1000)
    bk = rng.integers(0, 400_000, 300_000).astype(np.int64)
    pk = rng.integers(-1000, 450_000, 1_000_003).astype(np.int64)
    ob, op = oracle_mod.inner_join(bk, pk)
    with dfp.HashTable(1, "int64", 0) as t:
        t.append(0, torch.from_numpy(bk).cuda())
        t.finish(0)
        b, p = _probe_async_base(dfp, t, pk, base)
        assert np.array_equal(b, ob)
        assert np.array_equal(p, (op.astype(np.uint64) + base).astype(np.uint32))
        with pytest.raises(dfp.HjError):
            _probe_async_base(dfp, t, pk, 2**32 - 10)


def test_probe_capacity_truncates(dfp, oracle_mod, probe_mode):
    """include/hj.h hj_probe_async: min(total, capacity) pairs are written - the first ones
    of the canonical order - and the total still comes back; nothing past the capacity is
    touched. Build keys with single rows, runs (sorted duplicates) and scattered
    duplicates, so count-free steps, run windows and segment windows all meet the bound."""
    rng = np.random.default_rng(7)
    runs = np.repeat(np.arange(0, 40_000, dtype=np.int64), rng.integers(1, 6, 40_000))
    scattered = rng.integers(40_000, 120_000, 150_000).astype(np.int64)
    bk = np.concatenate([runs, scattered])
    pk = rng.integers(-100, 125_000, 400_001).astype(np.int64)
    ob, op = oracle_mod.inner_join(bk, pk)
    m = len(ob)
    n = len(pk)
    keys = torch.from_numpy(pk).cuda()
    ws = torch.empty(dfp.HashTable.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    with dfp.HashTable(1, "int64", 0) as t:
        t.append(0, torch.from_numpy(bk).cuda())
        t.finish(0)
        for cap in (1, 63, 64, 65, 12_345, m // 2, m - 1, m):
            ob_d = torch.full((m + 64,), -7, dtype=torch.int64, device="cuda")
            op_d = torch.full((m + 64,), -7, dtype=torch.int32, device="cuda")
            dt = torch.zeros(1, dtype=torch.int64, device="cuda")
            t.probe_async(keys.data_ptr(), n, ob_d.data_ptr(), op_d.data_ptr(), cap, dt.data_ptr(), ws.data_ptr(), s)
            assert int(dt.item()) == m, cap
            b = ob_d.cpu().numpy()
            p = op_d.cpu().numpy()
            assert np.array_equal(b[:cap].astype(np.uint64), ob[:cap]), cap
            assert np.array_equal(p[:cap].view(np.uint32), op[:cap]), cap
            assert (b[cap:] == -7).all() and (p[cap:] == -7).all(), cap


# ---- the range-free dense build (the partition learns the key range) -------------

@pytest.mark.parametrize("case", ["aligned", "straddle", "negative", "near_min", "max_blocks", "past_blocks",
                                  "dups_parts", "nulls"])
def test_range_free_dense_build(dfp, oracle_mod, case):
    """The dense build's partition bins rows by absolute 8192-value key block modulo 2048 and
    reduces the key range itself; the table starts at the minimum rounded down to a block.
    Key sets at the edges of that map — a minimum on / off a block boundary, negative keys,
    keys at INT64_MIN, exactly 2048 blocks, more blocks than 2048 (the build falls back to
    the key-range pass), several partitions with duplicates, null rows — give the oracle's
    pairs."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    n = 200_000
    bvalid = None
    parts = None
    if case == "aligned":
        bk = rng.integers(0, 8192 * 40, n) + 8192 * 7
    elif case == "straddle":
        bk = rng.integers(0, 8192 * 40, n) + 8192 * 7 + 5000
    elif case == "negative":
        bk = rng.integers(-8192 * 30 - 17, 8192 * 10, n)
    elif case == "near_min":
        bk = rng.integers(0, 600_000, n) + I64_MIN
        bk[:3] = [I64_MIN, I64_MIN, I64_MIN + 1]
    elif case == "max_blocks":  # [al, al + 2048 blocks): the last block ends the range
        lo = 8192 * 3 + 100
        bk = rng.integers(lo, 8192 * 3 + 2048 * 8192, 2_100_000)
        bk[:2] = [lo, 8192 * 3 + 2048 * 8192 - 1]
    elif case == "past_blocks":  # 2049 blocks: the key-range pass path
        lo = 8192 * 3 + 100
        bk = rng.integers(lo, 8192 * 3 + 2049 * 8192, 2_100_000)
        bk[:2] = [lo, 8192 * 3 + 2049 * 8192 - 1]
    elif case == "dups_parts":
        bk = rng.integers(1000, 1000 + 50_000, n)
        parts = [0, 50_000, 50_000, 120_000, n]
    else:
        bk = rng.integers(-5000, 300_000, n)
        bvalid = rng.random(n) > 0.1
    bk = bk.astype(np.int64)
    span = int(bk.max()) - int(bk.min()) + 1
    plo = max(int(bk.min()) - 50, int(I64_MIN))
    pk = np.concatenate([rng.choice(bk, 300_000), rng.integers(plo, int(bk.min()) + span + 50, 300_000)])
    pk = pk.astype(np.int64)
    b, p, st = gpu_join(dfp, bk, pk, bvalid=bvalid, parts=parts)
    assert st["buckets"] == 0, "a direct-addressed table"
    ob, op = oracle_mod.inner_join(bk, pk, None if bvalid is None else np.asarray(bvalid, bool))
    assert_same(b, p, ob, op)


# ---- the speculative build (the key range stays on the device) --------------------

@pytest.mark.parametrize("case", ["dense_edge", "hashed_edge", "wide", "all_null", "single_key", "int32"])
def test_spec_build_layouts(dfp, oracle_mod, case):
    """hj_build_finish launches the dense frag build before the host has read the key range
    (its kernels resolve the geometry from the reduction's result in device memory); the
    host reads the range when the table is first used, and a range that takes another
    layout is built then. At the layout edges — a range of exactly 8 x rows (dense) and one
    value more (hashed), keys over the whole int64 domain, every key null, one key value,
    int32 keys — the table takes the layout the range gives and the oracle's pairs."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    n = 100_000
    bvalid = None
    key_type = "int64"
    want_dense = True
    if case == "dense_edge":
        bk = rng.integers(0, 8 * n, n) - 12345
        bk[:2] = [-12345, 8 * n - 1 - 12345]
    elif case == "hashed_edge":
        bk = rng.integers(0, 8 * n + 1, n) - 12345
        bk[:2] = [-12345, 8 * n - 12345]
        want_dense = False
    elif case == "wide":
        bk = rng.integers(I64_MIN, np.iinfo(np.int64).max, n, dtype=np.int64)
        want_dense = False
    elif case == "all_null":
        bk = rng.integers(0, 1000, n)
        bvalid = np.zeros(n, bool)
        want_dense = None
    elif case == "single_key":
        bk = np.full(n, 77, np.int64)
    else:
        bk = rng.integers(-2**31, 2**31 - 8 * n, 1)[0] + rng.integers(0, 4 * n, n)
        key_type = "int32"
    bk = np.asarray(bk, np.int64 if key_type == "int64" else np.int32)
    pk = np.concatenate([rng.choice(bk, 50_000), rng.integers(int(bk.min()) - 10, int(bk.min()) + 4 * n, 50_000)])
    pk = pk.astype(bk.dtype)
    b, p, st = gpu_join(dfp, bk, pk, bvalid=bvalid, key_type=key_type)
    if want_dense is not None:
        assert (st["buckets"] == 0) == want_dense, st
    ob, op = oracle_mod.inner_join(bk, pk, None if bvalid is None else bvalid)
    assert_same(b, p, ob, op)


@pytest.mark.parametrize("case", ["dense", "hashed"])
def test_spec_build_concurrent_first_probes(dfp, oracle_mod, case):
    """Several threads probe a freshly built table at once (the operator's partitions do):
    the first caller settles a speculative build — for wide keys by building the hashed
    table — and the others wait for it; every probe gives the oracle's pairs."""
    import threading

    rng = np.random.default_rng(11 if case == "dense" else 12)
    n = 200_000
    bk = (rng.integers(0, 4 * n, n) if case == "dense"
          else rng.integers(I64_MIN, np.iinfo(np.int64).max, n, dtype=np.int64)).astype(np.int64)
    pks = [np.concatenate([rng.choice(bk, 40_000), rng.integers(0, 4 * n, 40_000)]).astype(np.int64)
           for _ in range(4)]
    want = [oracle_mod.inner_join(bk, pk) for pk in pks]
    for _ in range(3):
        with dfp.HashTable(1, "int64", 0) as t:
            t.append(0, torch.from_numpy(bk).cuda())
            t.finish(0)
            got, errs = [None] * 4, []

            def run(i):
                try:
                    got[i] = t.probe(torch.from_numpy(pks[i]).cuda())
                except Exception as e:  # noqa: BLE001 - reported below
                    errs.append(e)

            th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errs, errs
            for (b, p), (ob, op) in zip(got, want):
                assert_same(b, p, ob, op)
            assert (t.stats()["buckets"] == 0) == (case == "dense")


@pytest.mark.parametrize("case", ["dense", "hashed"])
def test_spec_build_two_partitions_first_probes(dfp, oracle_mod, case):
    """The shape of the round-4 fault (gpurun_out/r04p): the operator's two
    partitions each append half of the build side and call hj_build_finish (the last one
    launches the speculative build), then both probe at once with device output and a
    validity bitmap — composite keys are 64-bit hashes, so the table is hashed and the first
    probe builds it while the other must wait for the settled geometry."""
    import threading

    rng = np.random.default_rng(21 if case == "dense" else 22)
    n = 120_000
    bk = (rng.integers(0, 4 * n, n) if case == "dense"
          else rng.integers(I64_MIN, np.iinfo(np.int64).max, n, dtype=np.int64)).astype(np.int64)
    pks = [np.concatenate([rng.choice(bk, 30_000), rng.integers(0, 4 * n, 30_000)]).astype(np.int64) for _ in range(2)]
    pvalid = [rng.random(pk.size + 5) > 0.05 for pk in pks]  # bit 5 of the bitmap is row 0
    want = [oracle_mod.inner_join(bk, pk, None, v[5:]) for pk, v in zip(pks, pvalid)]
    halves = [bk[: n // 2], bk[n // 2:]]
    for _ in range(3):
        with dfp.HashTable(2, "int64", 0) as t:
            got, errs = [None] * 2, []

            def part(i):
                try:
                    t.append(i, torch.from_numpy(halves[i]).cuda())
                    t.finish(i)
                    bits = torch.from_numpy(np.packbits(pvalid[i], bitorder="little")).cuda()
                    b, p = t.probe(torch.from_numpy(pks[i]).cuda(), valid=bits, device_output=True, valid_offset=5)
                    got[i] = (b.cpu().numpy().astype(np.uint64), p.cpu().numpy().astype(np.uint32))
                except Exception as e:  # noqa: BLE001 - reported below
                    errs.append(e)

            th = [threading.Thread(target=part, args=(i,)) for i in range(2)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errs, errs
            for (b, p), (ob, op) in zip(got, want):
                assert_same(b, p, ob, op)
            assert (t.stats()["buckets"] == 0) == (case == "dense")
