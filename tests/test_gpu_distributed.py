"""GPU: the multi-GPU path (radix partition kernel + RCCL all-to-all + local build/probe
with global ids) run as one RCCL rank on the box's GPU, against the oracle; and the
partition kernel against its host restatement. (N > 1 ranks: the driver's 8-GPU runs;
the exchange logic at world_size 2 is covered on CPU by test_distributed_gloo.py.)"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
from conftest import init_one_rank_nccl

pytestmark = pytest.mark.gpu


def _mix64(k):
    with np.errstate(over="ignore"):
        k = k.astype(np.uint64)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xFF51AFD7ED558CCD)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xC4CEB9FE1A85EC53)
        k ^= k >> np.uint64(33)
        return k


@pytest.mark.parametrize("nparts", [1, 2, 8, 64])
@pytest.mark.parametrize("id_dtype", [torch.int64, torch.int32])
@pytest.mark.parametrize("narrow", [False, True])
def test_radix_partition_kernel(dfp, nparts, id_dtype, narrow):
    """Stable multi-split by the low hash bits; narrow: keys written as int32(key - off)."""
    from datafusion_parallelism_amd.distributed import gpu_radix_partition

    rng = np.random.default_rng(nparts)
    k = rng.integers(-10**12, 10**12, 100003) if not narrow else rng.integers(5 * 10**9, 9 * 10**9, 100003)
    off = 5 * 10**9 + 2**31 if narrow else None
    out_k, out_i, counts = gpu_radix_partition(torch.from_numpy(k).cuda(), None, 1000, nparts, id_dtype=id_dtype,
                                               key_offset=off)
    dest = (_mix64(k) & np.uint64(nparts - 1)).astype(np.int64)
    order = np.argsort(dest, kind="stable")  # stable multi-split
    assert np.array_equal(counts.cpu().numpy(), np.bincount(dest, minlength=nparts))
    want_k = k[order] if not narrow else (k[order] - off).astype(np.int32)
    assert out_k.dtype == (torch.int32 if narrow else torch.int64)
    assert np.array_equal(out_k.cpu().numpy(), want_k)
    assert np.array_equal(out_i.cpu().numpy(), order + 1000)


@pytest.mark.parametrize("nparts", [1, 2, 8, 64])
@pytest.mark.parametrize("by_range,lo,hi", [(True, 0, 99999), (True, -(2**63), 2**63 - 1), (False, 2000, 60000),
                                            (True, 2000, 60000), (True, -(2**40), 2**40 + 3)])
def test_partition_spec_kernel(dfp, nparts, by_range, lo, hi):
    """hj_partition_rows: keys outside [lo, hi] dropped, range or hash map, stable; the
    host restatement PartSpec.part_of gives the same destinations."""
    from datafusion_parallelism_amd.distributed import PartSpec, gpu_radix_partition

    rng = np.random.default_rng(nparts + 7)
    k = rng.integers(-(2**41), 2**41, 50007) if lo < -1000 else rng.integers(-500, 100500, 50007)
    k[:5] = [lo, hi, max(lo - 1, -(2**63)), min(hi + 1, 2**63 - 1), (lo + hi) // 2]
    spec = PartSpec(by_range, lo, hi)
    out_k, out_i, counts = gpu_radix_partition(torch.from_numpy(k).cuda(), None, 0, nparts, spec=spec)
    rdest, keep = spec.part_of(k, nparts)
    dest = rdest if by_range else (_mix64(k) & np.uint64(nparts - 1)).astype(np.int64)
    idx = np.nonzero(keep)[0]
    order = idx[np.argsort(dest[idx], kind="stable")]
    tot = int(counts.sum())
    assert np.array_equal(counts.cpu().numpy(), np.bincount(dest[idx], minlength=nparts))
    assert np.array_equal(out_k[:tot].cpu().numpy(), k[order])
    assert np.array_equal(out_i[:tot].cpu().numpy(), order)
    if by_range:  # contiguous key ranges: destination non-decreasing in the key
        srt = idx[np.argsort(k[idx], kind="stable")]
        assert (np.diff(dest[srt]) >= 0).all()


@pytest.mark.parametrize("chunks", [1, 3])
def test_distributed_join_one_rank(dfp, oracle_mod, chunks):
    """One RCCL rank (the exchange is a self-copy): pairs equal the oracle's; with
    chunks > 1 the probe side is pipelined (one rank keeps the global order)."""
    from datafusion_parallelism_amd.distributed import DistributedHashJoin

    init_one_rank_nccl()
    try:
        rng = np.random.default_rng(4)
        bk = rng.integers(0, 30000, 100000)
        pk = rng.integers(0, 50000, 300000)
        b, p = DistributedHashJoin(chunks=chunks).run(torch.from_numpy(bk).cuda(), 0, torch.from_numpy(pk).cuda(), 0)
        ob, op = oracle_mod.inner_join(bk, pk)
        assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob)
        assert np.array_equal(p.cpu().numpy().astype(np.uint32), op)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("keys", ["dense", "sparse", "dense_far"])
def test_broadcast_join_one_rank(dfp, oracle_mod, keys):
    """The broadcast plan on one RCCL rank: a dense build domain travels as int32 offsets
    (broadcast_key_plan + hj_build_key_base), a sparse one as int64 keys; far from zero
    (offsets from 2^62) too. Pairs equal the oracle's, probe ids = probe_base + row."""
    from datafusion_parallelism_amd.distributed import DistributedHashJoin, broadcast_key_plan

    init_one_rank_nccl()
    try:
        rng = np.random.default_rng(7)
        off = 2**62 if keys == "dense_far" else 0
        if keys == "sparse":
            bk = rng.integers(-(2**50), 2**50, 200_000)
            pk = np.concatenate([rng.choice(bk, 300_000), rng.integers(-(2**50), 2**50, 300_000)])
        else:
            bk = rng.integers(0, 150_000, 200_000) + off
            pk = rng.integers(-1000, 200_000, 600_000) + off
        tb, tp = torch.from_numpy(bk).cuda(), torch.from_numpy(pk).cuda()
        plan = broadcast_key_plan(tb, bk.size)
        assert (plan is None) == (keys == "sparse")
        if plan is not None:
            assert plan == (int(bk.min()), int(bk.max() - bk.min() + 1))
        b, p = DistributedHashJoin().run_broadcast(tb, tp, 5)
        ob, op = oracle_mod.inner_join(bk, pk)
        assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob)
        assert np.array_equal(p.cpu().numpy().astype(np.uint32), op + 5)
    finally:
        dist.destroy_process_group()


def test_large_exchange_one_rank(dfp):
    """A 1.3 GB exchange (above the size where single RCCL self-copies come back wrong,
    tools/debug_shuffle.py) runs in rounds and arrives exact."""
    from datafusion_parallelism_amd import distributed
    from datafusion_parallelism_amd.distributed import all_to_all_rows, gpu_radix_partition

    init_one_rank_nccl()
    try:
        n = 160_000_000
        dev = torch.device("cuda", 0)
        keys = torch.randint(-(2**40), 2**40, (n,), dtype=torch.int64, device=dev)
        k, perm, counts = gpu_radix_partition(keys, None, 0, 1, id_dtype=torch.int64)
        assert 8 * n > 4 * distributed.A2A_MAX_BYTES
        rk, ri, st = all_to_all_rows(k, perm, counts)
        assert st.recv_rows == n
        assert torch.equal(rk, keys)
        assert torch.equal(ri, torch.arange(n, device=dev))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nparts", [1, 2, 8, 64])
@pytest.mark.parametrize("n", [0, 1, 16383, 16384, 1_000_003])
@pytest.mark.parametrize("mode", ["hash", "range_narrow", "ids_u64_nulls"])
def test_partition_regions_kernel(dfp, nparts, n, mode):
    """hj_partition_regions (one pass, look-back over 16384-row tiles): region d holds the
    rows of destination d in source row order, with hj_partition_rows' map, filter,
    narrowing and ids; counts exact."""
    import ctypes

    from datafusion_parallelism_amd import _lib
    from datafusion_parallelism_amd.distributed import PartSpec

    L = _lib.load()
    rng = np.random.default_rng(n + nparts)
    k = rng.integers(-(2**40), 2**40, n) if mode != "range_narrow" else rng.integers(-500, 3 * 10**6, n)
    dev = torch.device("cuda", 0)
    keys = torch.from_numpy(k.astype(np.int64)).to(dev)
    spec, off, ids, valid_np = None, 0, None, np.ones(n, bool)
    if mode == "range_narrow":
        spec = PartSpec(True, 0, 2 * 10**6)
        off = 0 + 2**31
    id_base = 77
    if mode == "ids_u64_nulls":
        ids_np = rng.integers(0, 2**62, n).astype(np.uint64)
        ids = torch.from_numpy(ids_np.view(np.int64)).to(dev)
        valid_np = rng.random(n) > 0.1
    bitmap = torch.from_numpy(np.packbits(np.concatenate([np.zeros(3, bool), valid_np]), bitorder="little")).to(dev)
    cap = max(n, 1)
    ob = 4 if mode == "range_narrow" else 8
    out_k = torch.empty(nparts * cap, dtype=torch.int32 if ob == 4 else torch.int64, device=dev)
    idb = 8 if mode == "ids_u64_nulls" else 4
    out_i = torch.empty(nparts * cap, dtype=torch.int64 if idb == 8 else torch.int32, device=dev)
    counts = torch.full((nparts,), -1, dtype=torch.int64, device=dev)
    ws = torch.empty(L.hj_partition_regions_workspace_bytes(n, nparts), dtype=torch.uint8, device=dev)
    sp = ctypes.byref(_lib.HjPartSpec(1, spec.key_lo, spec.key_hi)) if spec else None
    _lib.check(L.hj_partition_regions(1, keys.data_ptr() if n else None, bitmap.data_ptr(), 3,
                                      ids.data_ptr() if ids is not None else None, id_base, n, nparts, sp,
                                      out_k.data_ptr(), ob, off, out_i.data_ptr(), idb, cap, counts.data_ptr(),
                                      ws.data_ptr(), None))
    torch.cuda.synchronize()
    assert int(ws[8:16].view(torch.int64).item()) == 0  # look-back never gave up
    keep = valid_np.copy()
    if spec is not None:
        dest, inr = spec.part_of(k, nparts)
        keep &= inr
    else:
        dest = (_mix64(k) & np.uint64(nparts - 1)).astype(np.int64)
    c = counts.cpu().numpy()
    assert np.array_equal(c, np.bincount(dest[keep], minlength=nparts))
    ok_, oi_ = out_k.cpu().numpy(), out_i.cpu().numpy()
    for d in range(nparts):
        rows = np.nonzero(keep & (dest == d))[0]  # ascending: stable
        want_k = k[rows] if ob == 8 else (k[rows] - off).astype(np.int32)
        assert np.array_equal(ok_[d * cap:d * cap + c[d]], want_k)
        want_i = ids_np[rows].view(np.int64) if ids is not None else (rows + id_base).astype(np.int32)
        assert np.array_equal(oi_[d * cap:d * cap + c[d]], want_i)


@pytest.mark.parametrize("n", [0, 1, 2, 4095, 4097, 3_000_001, 40_000_000])
@pytest.mark.parametrize("kind", ["i64", "i32", "i64_nulls"])
def test_key_minmax(dfp, n, kind):
    """hj_key_minmax (one launch, the last block reduces the partials): min and max of the
    valid keys, INT64_MAX / INT64_MIN for none; back-to-back calls reuse one workspace
    (the ticket counter is re-armed), against numpy."""
    from datafusion_parallelism_amd import _lib

    L = _lib.load()
    rng = np.random.default_rng(n)
    dev = torch.device("cuda", 0)
    dt = np.int32 if kind == "i32" else np.int64
    lo, hi = (-(2**31), 2**31 - 1) if kind == "i32" else (-(2**62), 2**62)
    k = rng.integers(lo, hi, n, dtype=dt)
    valid = rng.random(n) > 0.3 if kind == "i64_nulls" else np.ones(n, bool)
    keys = torch.from_numpy(k).to(dev)
    bitmap = torch.from_numpy(np.packbits(np.concatenate([np.zeros(5, bool), valid]), bitorder="little")).to(dev)
    ws = torch.empty(L.hj_key_minmax_workspace_bytes(), dtype=torch.uint8, device=dev)
    out = torch.empty(2, dtype=torch.int64, device=dev)
    kt = 0 if kind == "i32" else 1
    for _ in range(3):
        out.fill_(7)
        _lib.check(L.hj_key_minmax(kt, keys.data_ptr() if n else None,
                                   bitmap.data_ptr() if kind == "i64_nulls" else None, 5 if kind == "i64_nulls" else 0,
                                   n, out.data_ptr(), ws.data_ptr(), None))
        got = out.tolist()
        v = k[valid]
        want = [int(v.min()), int(v.max())] if v.size else [2**63 - 1, -(2**63)]
        assert got == want
