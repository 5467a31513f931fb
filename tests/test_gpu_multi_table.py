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
