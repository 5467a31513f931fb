"""GPU parity of the multi-GPU table (hj_build_begin_multi) through the
C ABI against the oracle. The box has one GPU, so the shards are placed on the same
device several times ([0, 0], [0, 0, 0, 0]): every exchange is a same-device copy, but the
sharding, the per-shard global ids, the row-range split (broadcast) and the canonical merge
of the shards' pairs (radix) run exactly as over xGMI."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _multi_join(dfp, devices, plan, bk, pk, bvalid=None, pvalid=None, parts=1, key_type="int64", host_probe=False):
    with dfp.HashTable(parts, key_type, devices=devices, plan=plan) as t:
        bounds = np.linspace(0, len(bk), parts + 1).astype(int)
        for p in range(parts):
            lo, hi = bounds[p], bounds[p + 1]
            t.append(p, torch.from_numpy(bk[lo:hi].copy()).cuda(), None if bvalid is None else bvalid[lo:hi])
        t.finish_all()
        st = t.stats()
        if host_probe:
            b, pp = t.probe(pk, pvalid)
        else:
            b, pp = t.probe(torch.from_numpy(pk.copy()).cuda(), pvalid, device_output=True)
            b, pp = b.cpu().numpy().astype(np.uint64), pp.cpu().numpy().view(np.uint32)
        lookups = {int(k): t.lookup(int(k)) for k in bk[:5]}
        return np.asarray(b, np.uint64), np.asarray(pp, np.uint32), st, lookups


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("nb,np_,krange,null_frac,parts", [
    (1000, 3000, 600, 0.0, 1),
    (200_000, 500_001, 150_000, 0.02, 3),      # duplicates, nulls, several partitions
    (2_000_000, 3_000_000, 4_000_000, 0.0, 2), # direct-addressed shards, sliced probes
])
def test_multi_table_parity(dfp, oracle_mod, plan, devices, nb, np_, krange, null_frac, parts):
    rng = np.random.default_rng(nb + len(devices))
    bk = rng.integers(-5, krange, nb).astype(np.int64)
    pk = rng.integers(-10, krange + 10, np_).astype(np.int64)
    bv = rng.random(nb) >= null_frac if null_frac else None
    pv = rng.random(np_) >= null_frac if null_frac else None
    b, p, st, lk = _multi_join(dfp, devices, plan, bk, pk, bv, pv, parts=parts)
    ob, op = oracle_mod.inner_join(bk, pk, bv, pv)
    assert len(b) == len(ob)
    assert np.array_equal(p, op) and np.array_equal(b, ob)
    assert st["build_rows"] == nb
    for k, rows in lk.items():  # get_iter: the key's rows, newest first
        valid = np.ones(nb, bool) if bv is None else bv
        assert rows == sorted(np.nonzero((bk == k) & valid)[0].tolist(), reverse=True)


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
def test_multi_table_host_probe_int32(dfp, oracle_mod, plan):
    rng = np.random.default_rng(9)
    bk = rng.integers(-2**31, 2**31 - 1, 300_000).astype(np.int32)
    bk[:1000] = bk[1000:2000]  # duplicated keys
    pk = np.concatenate([bk[rng.integers(0, len(bk), 200_000)], rng.integers(-2**31, 2**31 - 1, 100_000).astype(np.int32)])
    b, p, _, _ = _multi_join(dfp, [0, 0], plan, bk, pk, key_type="int32", host_probe=True)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(p, op) and np.array_equal(b, ob)


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
def test_multi_table_probe_base(dfp, oracle_mod, plan):
    """hj_probe_async_base on a multi table: the broadcast plan's shards take their row
    ranges' bases (no id arrays); the radix plan adds the base after the merge."""
    rng = np.random.default_rng(17)
    bk = rng.integers(0, 100_000, 80_000).astype(np.int64)
    pk = rng.integers(0, 120_000, 250_001).astype(np.int64)
    base = 123_456_789
    ob, op = oracle_mod.inner_join(bk, pk)
    with dfp.HashTable(1, "int64", devices=[0, 0, 0, 0], plan=plan) as t:
        t.append(0, torch.from_numpy(bk).cuda())
        t.finish_all()
        n = len(pk)
        keys = torch.from_numpy(pk).cuda()
        cap = 4 * n
        b = torch.empty(cap, dtype=torch.int64, device="cuda")
        p = torch.empty(cap, dtype=torch.int32, device="cuda")
        ws = torch.empty(dfp.HashTable.workspace_bytes(n), dtype=torch.uint8, device="cuda")
        dt = torch.zeros(1, dtype=torch.int64, device="cuda")
        t.probe_async(keys.data_ptr(), n, b.data_ptr(), p.data_ptr(), cap, dt.data_ptr(), ws.data_ptr(),
                      torch.cuda.current_stream().cuda_stream, probe_base=base)
        m = int(dt.item())
        assert np.array_equal(b[:m].cpu().numpy().astype(np.uint64), ob)
        assert np.array_equal(p[:m].cpu().numpy().view(np.uint32), (op.astype(np.uint64) + base).astype(np.uint32))


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
def test_multi_table_staging_copies(dfp, oracle_mod, plan, monkeypatch):
    """DFP_HJ_MULTI_STAGE=1 treats every shard's device as foreign: the cross-device
    branches (keys / ids copied into the shard's HBM, the validity bitmap re-based at
    voff & 7, the broadcast probe's per-shard key and bitmap copies) run on one GPU."""
    monkeypatch.setenv("DFP_HJ_MULTI_STAGE", "1")
    rng = np.random.default_rng(23)
    nb, np_ = 150_003, 400_009
    bk = rng.integers(0, 90_000, nb).astype(np.int64)
    pk = rng.integers(-50, 100_000, np_).astype(np.int64)
    bv = rng.random(nb) >= 0.03
    pv = rng.random(np_) >= 0.03
    import pyarrow as pa

    devices = [0, 0, 0] if plan == "broadcast" else [0, 0]  # radix: a power of two
    # host Arrow slices at odd offsets: the appended bitmaps start at voff & 7 != 0
    arr = pa.array(np.concatenate([np.zeros(5, np.int64), bk]), mask=~np.concatenate([np.ones(5, bool), bv]))
    bounds = [0, 40_001, 97_000, nb]
    with dfp.HashTable(3, "int64", devices=devices, plan=plan) as t:
        for q in range(3):
            t.append(q, arr.slice(5 + bounds[q], bounds[q + 1] - bounds[q]))
        t.finish_all()
        b, p = t.probe(torch.from_numpy(pk).cuda(), pv, device_output=True)
        b, p = b.cpu().numpy().astype(np.uint64), p.cpu().numpy().view(np.uint32)
        assert t.stats()["build_rows"] == nb
    ob, op = oracle_mod.inner_join(bk, pk, bv, pv)
    assert np.array_equal(p, op) and np.array_equal(b, ob)


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
def test_multi_table_injected_shard_failure(dfp, oracle_mod, plan, monkeypatch):
    """A shard that fails after earlier shards' builds were enqueued: the error reaches the
    caller, every queued shard stream is drained before the scratch returns to the cache,
    and the next join on the same device is exact."""
    rng = np.random.default_rng(29)
    bk = rng.integers(0, 400_000, 600_000).astype(np.int64)
    pk = rng.integers(0, 500_000, 900_000).astype(np.int64)
    monkeypatch.setenv("DFP_HJ_INJECT_SHARD_FAIL", "2")
    t = dfp.HashTable(1, "int64", devices=[0, 0, 0, 0], plan=plan)
    t.append(0, torch.from_numpy(bk).cuda())
    with pytest.raises(dfp.HjError, match="injected shard failure"):
        t.finish(0)
    t.close()
    monkeypatch.delenv("DFP_HJ_INJECT_SHARD_FAIL")
    b, p, _, _ = _multi_join(dfp, [0, 0, 0, 0], plan, bk, pk)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(p, op) and np.array_equal(b, ob)


@pytest.mark.parametrize("plan", ["broadcast", "radix"])
def test_multi_table_probe_argument_checks(dfp, plan):
    """The multi-table probes run the single-GPU probe's checks before dispatching (u32
    probe numbering: base + rows <= 2^32)."""
    with dfp.HashTable(1, "int64", devices=[0, 0], plan=plan) as t:
        t.append(0, torch.arange(1000, dtype=torch.int64, device="cuda"))
        t.finish_all()
        n = 1000
        keys = torch.arange(n, dtype=torch.int64, device="cuda")
        b = torch.empty(n, dtype=torch.int64, device="cuda")
        p = torch.empty(n, dtype=torch.int32, device="cuda")
        ws = torch.empty(dfp.HashTable.workspace_bytes(n), dtype=torch.uint8, device="cuda")
        dt = torch.zeros(1, dtype=torch.int64, device="cuda")
        with pytest.raises(dfp.HjError, match="probe_base"):
            t.probe_async(keys.data_ptr(), n, b.data_ptr(), p.data_ptr(), n, dt.data_ptr(), ws.data_ptr(),
                          torch.cuda.current_stream().cuda_stream, probe_base=2**32 - 10)
        with pytest.raises(ValueError):
            t.probe_async(keys.data_ptr(), n, b.data_ptr(), p.data_ptr(), n, dt.data_ptr(), ws.data_ptr(),
                          torch.cuda.current_stream().cuda_stream, probe_ids_ptr=keys.data_ptr(), probe_base=5)
