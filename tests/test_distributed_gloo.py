"""CPU, world_size 2 (gloo): the multi-GPU exchange logic of
datafusion_parallelism_amd.distributed — counts all-to-all, uneven-split row exchange,
global build/probe ids — joined per rank by the oracle (test-local stand-ins for the
HIP partition / local-join kernels, which need a GPU). Global pairs gathered from both
ranks must equal the single-process oracle join after canonical ordering."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rendezvous

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mix64(k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        k = k.astype(np.uint64)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xFF51AFD7ED558CCD)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xC4CEB9FE1A85EC53)
        k ^= k >> np.uint64(33)
        return k


def cpu_partition(keys, ids, id_base, nparts, spec=None):
    """Stable multi-split by the low hash bits, or by key range and dropping keys outside
    the spec's bounds (the semantics of hj_partition_rows)."""
    k = keys.numpy()
    i = np.arange(len(k), dtype=np.int64) + id_base if ids is None else ids.numpy()
    dest = (_mix64(k) & np.uint64(nparts - 1)).astype(np.int64)
    if spec is not None:
        rdest, keep = spec.part_of(k, nparts)
        if spec.by_range:
            dest = rdest
        k, i, dest = k[keep], i[keep], dest[keep]
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=nparts)
    n = len(keys)  # like the device kernel: full-length outputs, the first counts.sum() rows valid
    ok_ = np.zeros(n, dtype=k.dtype)
    oi_ = np.zeros(n, dtype=i.dtype)
    ok_[:len(order)] = k[order]
    oi_[:len(order)] = i[order]
    return torch.from_numpy(ok_), torch.from_numpy(oi_), torch.from_numpy(counts)


def oracle_local_join(bk, bi, pk, pi, cap=None):
    import oracle

    b, p = oracle.inner_join(bk.numpy(), pk.numpy())
    return torch.from_numpy(bi.numpy()[b.astype(np.int64)]), torch.from_numpy(pi.numpy()[p.astype(np.int64)])


class CpuLocalTable:
    """Test-local stand-in for GpuLocalTable (the oracle joins each received chunk)."""

    def __init__(self, bk, bi):
        self.bk, self.bi = bk, bi

    def probe(self, pk, pi, cap=None):
        b, p = oracle_local_join(self.bk, self.bi, pk, pi)
        return lambda: (b, p)

    def close(self):
        pass


def _canonical(b, p):
    pl = p.numpy().astype(np.int64)
    bl = b.numpy().astype(np.int64)
    same = pl[1:] == pl[:-1]
    return bool(np.all(pl[1:] >= pl[:-1]) and np.all(bl[1:][same] < bl[:-1][same]))


def _worker(rank, world, port, bks, pks, q, chunks=1, max_bytes=None, rfilter=True, plan="radix"):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    rendezvous.join(rank, world, port)
    from datafusion_parallelism_amd import distributed
    from datafusion_parallelism_amd.distributed import DistributedHashJoin

    if max_bytes:  # force the multi-round exchange path
        distributed.A2A_MAX_BYTES = max_bytes

    dj = DistributedHashJoin(partition_fn=cpu_partition, local_join_fn=oracle_local_join, chunks=chunks,
                             local_build_fn=CpuLocalTable, runtime_filter=rfilter)
    bbase = sum(len(x) for x in bks[:rank])
    pbase = sum(len(x) for x in pks[:rank])
    if plan == "broadcast":  # all_gather of the build shards, no probe exchange
        b, p = dj.run_broadcast(torch.from_numpy(bks[rank]), torch.from_numpy(pks[rank]), pbase)
        segs = [(b, p)]
    elif chunks == 1:
        b, p = dj.run(torch.from_numpy(bks[rank]), bbase, torch.from_numpy(pks[rank]), pbase)
        segs = [(b, p)]
    else:  # pipelined probe side: canonical per chunk
        plan = dj.prepare(torch.from_numpy(bks[rank]), torch.from_numpy(pks[rank]), bbase)
        allb = np.concatenate(bks)
        allp = np.concatenate(pks)
        span = allb.max() - allb.min() if rfilter else max(allb.max(), allp.max()) - min(allb.min(), allp.min())
        assert (plan.key_offset is None) == (span >= 2**32)
        assert plan.spec.by_range == (rfilter and allb.max() - allb.min() + 1 <= 8 * len(allb))
        bk, bi = dj.shard_build(torch.from_numpy(bks[rank]), bbase, plan)
        segs = dj.run_pipelined(bk, bi, torch.from_numpy(pks[rank]), pbase, plan)
        assert len(segs) == chunks
        b, p = torch.cat([x for x, _ in segs]), torch.cat([y for _, y in segs])
    # every rank's local output is canonical for its key subset (per chunk)
    ok = all(_canonical(x, y) for x, y in segs)
    pl = p.numpy().astype(np.int64)
    bl = b.numpy().astype(np.int64)
    sizes = [None] * world
    dist.all_gather_object(sizes, (bl.tolist(), pl.tolist(), ok))
    if rank == 0:
        q.put(sizes)
    dist.destroy_process_group()



@pytest.mark.parametrize("world,chunks,wide,max_bytes,rfilter", [
    (2, 1, False, None, True), (2, 3, False, None, True), (2, 3, True, None, True), (2, 1, False, 5000, True),
    (2, 3, True, 7000, True), (2, 3, False, None, False), (2, 1, True, None, False), (4, 1, False, 3000, True),
    (4, 2, True, None, False)])
def test_distributed_exchange_matches_single_join(oracle_mod, world, chunks, wide, max_bytes, rfilter):
    """rfilter: runtime min/max filter + range map for dense build domains (the default);
    off: every probe row travels, hash map."""
    """wide: keys spread over > 2^32 values, so they travel as full int64 (otherwise
    DistributedHashJoin.prepare narrows them to int32 offsets)."""
    rng = np.random.default_rng(9)
    bk = rng.integers(0, 3000, 9000).astype(np.int64)
    pk = rng.integers(0, 5000, 14000).astype(np.int64)
    if wide:
        bk, pk = bk * (2**33) - 2**40, pk * (2**33) - 2**40
    bb = [0, 4000, 9000] if world == 2 else [0, 1000, 4000, 4001, 9000]
    pb = [0, 9000, 14000] if world == 2 else [0, 5000, 5000, 11000, 14000]
    bks = [bk[bb[r]:bb[r + 1]] for r in range(world)]
    pks = [pk[pb[r]:pb[r + 1]] for r in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = rendezvous.parent_store()  # held until the ranks exit
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, world, port, bks, pks, q, chunks, max_bytes, rfilter)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    allb = np.concatenate([np.array(r[0], np.int64) for r in res]).astype(np.uint64)
    allp = np.concatenate([np.array(r[1], np.int64) for r in res]).astype(np.uint32)
    assert all(r[2] for r in res), "per-rank output not in canonical order"
    cb, cp = oracle_mod.canonical_pairs(allb, allp)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(cb, ob) and np.array_equal(cp.astype(np.uint32), op)


@pytest.mark.parametrize("world", [2, 3])
def test_broadcast_plan_is_canonical(oracle_mod, world):
    """Broadcast-build plan: the ranks' outputs, concatenated in rank
    order, ARE the single-process canonical output (no sort): the gathered build shards
    are the global row order and every rank probes a contiguous probe range."""
    rng = np.random.default_rng(21)
    bk = rng.integers(0, 2500, 7001).astype(np.int64)
    pk = rng.integers(-50, 4000, 12003).astype(np.int64)
    bb = np.linspace(0, len(bk), world + 1).astype(int)
    pb = np.linspace(0, len(pk), world + 1).astype(int)
    bks = [bk[bb[r]:bb[r + 1]] for r in range(world)]
    pks = [pk[pb[r]:pb[r + 1]] for r in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = rendezvous.parent_store()  # held until the ranks exit
    port = store.port
    procs = [ctx.Process(target=_worker, args=(r, world, port, bks, pks, q, 1, None, True, "broadcast"))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    allb = np.concatenate([np.array(r[0], np.int64) for r in res]).astype(np.uint64)
    allp = np.concatenate([np.array(r[1], np.int64) for r in res]).astype(np.uint32)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(allb, ob) and np.array_equal(allp, op)


def test_choose_plan():
    from datafusion_parallelism_amd.distributed import DistributedHashJoin

    assert DistributedHashJoin.choose_plan(10**7, 10**8, 8) == "broadcast"   # C2: 8e7 < 1.1e8
    assert DistributedHashJoin.choose_plan(10**8, 10**8, 8) == "radix"
    assert DistributedHashJoin.choose_plan(10**7, 10**8, 1) == "broadcast"


def test_check_counts_rejects_poisoned_counts():
    """A failed look-back in hj_partition_regions makes counts >= 2^60: every rank raises
    (poison bound on every row); a rank's own count above its region size raises too."""
    from datafusion_parallelism_amd import HjError
    from datafusion_parallelism_amd.distributed import check_counts

    check_counts([[3, 4], [10, 0]], 7, me=0)  # rank 1's 10 is within its own (larger) region
    with pytest.raises(HjError):
        check_counts([[3, 4], [-1, 0]], 7, me=0)
    with pytest.raises(HjError):
        check_counts([[3, 4], [1 << 60, 0]], 7, me=0)
    with pytest.raises(HjError):
        check_counts([[3, 9]], 7, me=0)


def test_sharded_ok_boundaries():
    """sharded_ok: a direct-addressed build domain within the widest dense range
    (DENSE_MAX_RANGE), u32 build ids and packed segment offsets; a range one value past
    DENSE_MAX_RANGE (dense by the 8 x rows criterion) takes the fallback instead of an
    exchange whose gathered table hj_table_wrap_dense would refuse."""
    from datafusion_parallelism_amd.distributed import (DENSE_MAX_RANGE, DistributedHashJoin, ExchangePlan,
                                                        PartSpec)

    def plan(rng, rows, by_range=True, ids=torch.int32):
        return ExchangePlan(build_id_dtype=ids, spec=PartSpec(by_range, 0, rng - 1), build_rows=rows,
                            build_lo=0, build_hi=rng - 1)

    ok = DistributedHashJoin.sharded_ok
    rows = 40_000_000  # 8 x rows > DENSE_MAX_RANGE, 2 x rows + 2G + 2 < 2^27
    assert ok(plan(DENSE_MAX_RANGE, rows), 8)
    assert not ok(plan(DENSE_MAX_RANGE + 1, rows), 8)
    assert ok(plan(8 * 1000, 1000), 4) and not ok(plan(8 * 1000 + 1, 1000), 4)  # density
    assert not ok(plan(1000, 1000, by_range=False), 2) and ok(plan(1000, 1000, by_range=False), 1)
    assert not ok(plan(1000, 1000, ids=torch.int64), 2)
    big = (2**27 - 2 * 8 - 2) // 2  # packed refs: 2B + 2G + 2 < 2^27
    assert ok(plan(big, big - 1), 8) and not ok(plan(big, big), 8)
    assert not ok(ExchangePlan(), 1)  # empty build side


def _plan_worker(rank, world, port, shards, rows, q):
    sys.path.insert(0, ROOT)
    rendezvous.join(rank, world, port)
    try:
        from datafusion_parallelism_amd.distributed import broadcast_key_plan

        plan = broadcast_key_plan(torch.from_numpy(shards[rank]), rows)
        q.put((rank, plan))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["dense", "sparse", "empty_shard", "all_empty"])
def test_broadcast_key_plan_world(case):
    """broadcast_key_plan over 3 gloo ranks: one MIN all-reduce over [min, ~max] gives every
    rank the global (base, range) of a dense build domain (the int32-offset gather), None
    for a sparse domain or no rows; an empty shard contributes nothing."""
    rng = np.random.default_rng(3)
    world = 3
    if case == "dense":
        shards = [rng.integers(10**12, 10**12 + 5000, 2000) for _ in range(world)]
    elif case == "sparse":
        shards = [rng.integers(-(2**50), 2**50, 2000) for _ in range(world)]
    elif case == "empty_shard":
        shards = [rng.integers(-7000, 7000, 3000), np.zeros(0, np.int64), rng.integers(-9000, 100, 3000)]
    else:
        shards = [np.zeros(0, np.int64) for _ in range(world)]
    shards = [s.astype(np.int64) for s in shards]
    rows = sum(len(s) for s in shards)
    allk = np.concatenate(shards)
    if rows and (allk.max() - allk.min() + 1) <= 8 * rows:
        want = (int(allk.min()), int(allk.max() - allk.min() + 1))
    else:
        want = None
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = rendezvous.parent_store()  # held until the ranks exit
    port = store.port
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, shards, rows, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(got[r] == want for r in range(world)), (got, want)
    assert (want is None) == (case in ("sparse", "all_empty"))


def _gather_worker(rank, world, port, lens, q):
    sys.path.insert(0, ROOT)
    rendezvous.join(rank, world, port)
    try:
        from datafusion_parallelism_amd.distributed import DistributedHashJoin

        dj = DistributedHashJoin()
        offs = [sum(lens[:d]) for d in range(world)]
        out = torch.full((sum(lens),), -7, dtype=torch.int32)
        mine = out.narrow(0, offs[rank], lens[rank])
        mine.copy_(torch.arange(lens[rank], dtype=torch.int32) + 1000 * rank)
        dj._allgather_var(out, offs, lens, mine)
        counts = dj._allgather_counts(torch.tensor([rank * 11 + 3], dtype=torch.int64))
        q.put((rank, out.numpy().copy(), counts))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lens", [[5, 5, 5], [6, 5, 4], [3, 0, 7], [4, 4]])
def test_sharded_plan_gathers(lens):
    """The sharded-build plan's collectives over gloo ranks: every rank's slice lands at its
    offset on every rank (even slices: one all-gather; uneven ones, as the range map cuts
    them: a padded all-gather and a copy to place), and the per-rank segment counts
    arrive in rank order."""
    world = len(lens)
    want = np.concatenate([np.arange(n, dtype=np.int32) + 1000 * r for r, n in enumerate(lens)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = rendezvous.parent_store()  # held until the ranks exit
    port = store.port
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, lens, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    for rank, out, counts in res:
        assert np.array_equal(out, want), rank
        assert counts == [r * 11 + 3 for r in range(world)]
