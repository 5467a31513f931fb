"""GPU: the multi-GPU plans of the C ABI (hj_dist.cpp) at world 2 / 4 / 8, through the C
entry points, with the ranks as threads of this process on the one GPU.

RCCL refuses two ranks on one device, so these tests use the test library
(lib/libdfp_hj_commtest.so = the product objects + the thread transport of
csrc/hj_comm_threads.cpp): the same hj_dist.cpp code — count matrices, point-to-point
exchanges, uneven all-gathers, the duplicate-segment rebase, the status words, the job
queue — with a host barrier and device copies in place of RCCL. The transport also checks
what RCCL would hang on (every rank issues the same collectives; each receive meets a send
of its size).

* hj_dist_build_sharded_async: every rank probes the whole build side's table with its own
  probe rows (hj_probe, probe idx + the rank's probe base); the ranks' outputs in rank order
  must equal the oracle's canonical pairs of the whole join. Kinds: dense,
  far from zero, duplicate-heavy, clustered (empty middle pieces), a sparse piece, sparse
  (the replicated fallback); int32 / int64 keys; nulls with a bitmap offset; a nonzero
  global build base; int32 probe keys against int64 build keys; two jobs queued back to back.
* hj_dist_join_radix: each rank's pairs are its share; concatenated and stably sorted by
  probe id they must equal the oracle's canonical pairs.
* failures: a rank that fails locally (test hook) makes every rank's job fail, none hangs,
  and the communicator keeps working for the next job.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _keys(kind, rng, nb, np_):
    off = 2**40 if kind == "dense_far" else 0
    if kind == "sparse":
        bk = rng.integers(-(2**50), 2**50, nb)
        pk = np.concatenate([rng.choice(bk, np_ // 2), rng.integers(-(2**50), 2**50, np_ - np_ // 2)])
    elif kind == "dups":  # heavy duplicates: segments in every piece, some keys > 15 rows
        bk = np.concatenate([rng.integers(0, nb // 8, nb - 400), np.full(400, nb // 16)])
        rng.shuffle(bk)
        pk = rng.integers(-50, nb // 8 + 50, np_)
    elif kind == "runs":  # sorted build keys: duplicated keys on consecutive (global) rows, run refs
        bk = np.repeat(np.arange(nb // 4, dtype=np.int64) * 2, 4)[:nb]
        pk = rng.integers(-20, nb // 2 + 20, np_)
    elif kind == "clustered":  # build keys at both ends of the range: middle pieces empty
        bk = np.concatenate([rng.integers(0, 1000, nb // 2), rng.integers(7 * nb, 7 * nb + 1000, nb - nb // 2)])
        pk = rng.integers(-10, 7 * nb + 1010, np_)
    elif kind == "sparse_piece":  # one piece holds a handful of rows over its whole key range
        bk = np.concatenate([rng.integers(0, 1000, nb - 7), rng.integers(7 * nb, 7 * nb + 1000, 7)])
        pk = np.concatenate([rng.choice(bk, np_ // 2), rng.integers(-10, 7 * nb + 1010, np_ - np_ // 2)])
    else:
        bk = rng.integers(0, nb + nb // 2, nb) + off
        pk = rng.integers(-1000, nb * 2, np_) + off
    return bk.astype(np.int64), pk.astype(np.int64)


@pytest.fixture(scope="module")
def ctl(dfp):
    import sys
    import os

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "datafusion-parallelism_amd")
    sys.path.insert(0, here)
    import build as hipbuild

    sys.path.pop(0)
    hipbuild.build_commtest()
    from datafusion_parallelism_amd import _lib

    return _lib.load_commtest()


class Ranks:
    """W rank threads over one hub; run(fn) calls fn(rank, comm) on every rank thread and
    returns the per-rank results (exceptions re-raised after all threads ended)."""

    def __init__(self, L, world, timeout_s=60.0, fail_at=None):
        import ctypes

        from datafusion_parallelism_amd._lib import check
        from datafusion_parallelism_amd.distributed import NativeComm

        self.L, self.world = L, world
        self.hub = L.hj_test_hub_create(world, timeout_s)
        assert self.hub
        self.comms = []
        dev = torch.device("cuda", 0)
        for r in range(world):
            h = ctypes.c_void_p()
            check(L.hj_test_comm_create(self.hub, r, 0, ctypes.byref(h)), L)
            self.comms.append(NativeComm(dev, lib=L, handle=h))
        if fail_at is not None:
            rank, job, step = fail_at
            L.hj_test_comm_fail_at(self.comms[rank]._h, job, step)

    def run(self, fn):
        out, errs = [None] * self.world, [None] * self.world

        def body(r):
            try:
                torch.cuda.set_device(0)
                out[r] = fn(r, self.comms[r])
            except BaseException as e:  # noqa: BLE001 - reported by the caller
                errs[r] = e

        ths = [threading.Thread(target=body, args=(r,)) for r in range(self.world)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=180)
            assert not t.is_alive(), "a rank thread hung"
        return out, errs

    def close(self):
        for c in self.comms:
            c.close()
        self.L.hj_test_hub_free(self.hub)


def _split(n, world, r):
    return n * r // world, n * (r + 1) // world


def _sharded_rank(r, comm, world, bk, pk, valid, key_dtype, probe_dtype, base0, steps=1):
    """One rank: `steps` sharded build-side jobs queued back to back, each table probed by
    the rank's own probe rows -> list of (build, probe) numpy pairs per step."""
    from datafusion_parallelism_amd.distributed import NativeJob  # noqa: F401

    b0, b1 = _split(bk.size, world, r)
    p0, p1 = _split(pk.size, world, r)
    keys = torch.from_numpy(bk[b0:b1].astype(key_dtype)).cuda()
    vbits = None
    if valid is not None:  # bit 5 of the bitmap is row b0
        v = np.concatenate([np.zeros(5, bool), valid[b0:b1]])
        vbits = torch.from_numpy(np.packbits(v, bitorder="little")).cuda()
    probe = pk[p0:p1].astype(probe_dtype)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    jobs = [comm.build_sharded_async(keys, base0 + b0, s.cuda_stream, valid=vbits, valid_offset=5,
                                     probe_dtype=torch.int64 if probe_dtype == np.int64 else torch.int32)
            for _ in range(steps)]
    res = []
    for job in jobs:
        table, info = job.table()
        job.close()
        try:
            b, p = table.probe(probe)
        finally:
            table.close()
        res.append((b, p.astype(np.uint64) + p0, info.build_rows, info.sharded))
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("kind", ["dense", "dups", "runs", "clustered", "sparse_piece", "sparse", "dense_far"])
def test_sharded_threads(ctl, oracle_mod, world, kind):
    rng = np.random.default_rng(world * 100 + len(kind))
    bk, pk = _keys(kind, rng, 60_000, 200_000)
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _sharded_rank(r, c, world, bk, pk, None, np.int64, np.int64, 0, steps=2))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    ob, op = oracle_mod.inner_join(bk, pk)
    for step in range(2):
        b = np.concatenate([o[step][0] for o in out])
        p = np.concatenate([o[step][1] for o in out])
        assert np.array_equal(b, ob), (kind, step)
        assert np.array_equal(p, op.astype(np.uint64)), (kind, step)
        assert all(o[step][2] == bk.size for o in out)
        assert all(o[step][3] == (kind != "sparse") for o in out)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("key_type", ["int32", "int64"])
@pytest.mark.parametrize("kind", ["dense", "dups", "sparse"])
def test_sharded_threads_nulls_base(ctl, oracle_mod, world, key_type, kind):
    """Nulls through a bitmap with an offset, a nonzero global build base, int32 keys."""
    rng = np.random.default_rng(7 + world)
    bk, pk = _keys(kind, rng, 50_000, 150_000)
    if key_type == "int32":
        bk, pk = (bk % (2**31)).astype(np.int32).astype(np.int64), (pk % (2**31)).astype(np.int32).astype(np.int64)
    valid = rng.random(bk.size) > 0.1
    kd = np.int32 if key_type == "int32" else np.int64
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _sharded_rank(r, c, world, bk, pk, valid, kd, kd, 1000))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    ob, op = oracle_mod.inner_join(bk, pk, valid, None)
    assert np.array_equal(np.concatenate([o[0][0] for o in out]), ob + 1000)
    assert np.array_equal(np.concatenate([o[0][1] for o in out]), op.astype(np.uint64))
    assert all(o[0][2] == 1000 + bk.size for o in out)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_threads_int32_probe_of_int64_build(ctl, oracle_mod, world):
    """A dense int64 build side probed with int32 keys: the table is keyed in the probe
    keys' type (hj_dist_build_sharded's probe_key_type)."""
    rng = np.random.default_rng(3)
    bk, pk = _keys("dups", rng, 40_000, 120_000)
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _sharded_rank(r, c, world, bk, pk, None, np.int64, np.int32, 0))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(np.concatenate([o[0][0] for o in out]), ob)
    assert np.array_equal(np.concatenate([o[0][1] for o in out]), op.astype(np.uint64))


def _radix_rank(r, comm, world, bk, pk, key_dtype, steps=1, base=0):
    b0, b1 = _split(bk.size, world, r)
    p0, p1 = _split(pk.size, world, r)
    keys = torch.from_numpy(bk[b0:b1].astype(key_dtype)).cuda()
    probe = torch.from_numpy(pk[p0:p1].astype(key_dtype)).cuda()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    jobs = [comm.join_radix(keys, base + b0, probe, p0, s.cuda_stream) for _ in range(steps)]
    res = []
    for job in jobs:
        b, p = job.pairs()
        res.append((b.cpu().numpy().astype(np.uint64) - base, p.cpu().numpy().astype(np.uint32)))
        t = job.times()
        assert all(x >= 0 for x in t)
        del b, p
        job.close()
    return res


def _merge(parts):
    b = np.concatenate([x[0] for x in parts])
    p = np.concatenate([x[1] for x in parts])
    o = np.argsort(p, kind="stable")
    return b[o], p[o]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("kind", ["dense", "dups", "runs", "clustered", "sparse"])
def test_radix_threads(ctl, oracle_mod, world, kind):
    rng = np.random.default_rng(world * 31 + len(kind))
    bk, pk = _keys(kind, rng, 60_000, 200_000)
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _radix_rank(r, c, world, bk, pk, np.int64, steps=2))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    ob, op = oracle_mod.inner_join(bk, pk)
    for step in range(2):
        b, p = _merge([o[step] for o in out])
        assert np.array_equal(b, ob), (kind, step)
        assert np.array_equal(p, op), (kind, step)
        # each rank's share is itself in canonical order (probe ascending)
        for o in out:
            assert np.all(np.diff(o[step][1].astype(np.int64)) >= 0)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_radix_threads_int32_and_empty(ctl, oracle_mod, world):
    """int32 keys; and a build side with no rows on some ranks (a rank with nothing)."""
    rng = np.random.default_rng(world)
    bk, pk = _keys("dups", rng, 30_000, 90_000)
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _radix_rank(r, c, world, bk, pk, np.int32))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    b, p = _merge([o[0] for o in out])
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(b, ob) and np.array_equal(p, op)
    # an empty build side everywhere: no pairs, no error
    ranks = Ranks(ctl, world)
    try:
        out, errs = ranks.run(lambda r, c: _radix_rank(r, c, world, bk[:0], pk, np.int64))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    assert sum(o[0][0].size for o in out) == 0


@pytest.mark.parametrize("base", [0, 5000])
def test_radix_one_rank_paths(ctl, oracle_mod, base):
    """One rank: base 0 takes the identity path (the build in place, the probe with
    probe_base), a nonzero global build base the whole plan; both give the oracle's pairs,
    also with duplicate-heavy keys (more pairs than probe rows: the job's re-probe)."""
    rng = np.random.default_rng(base + 1)
    bk = np.concatenate([rng.integers(0, 2000, 20_000), np.full(300, 77)]).astype(np.int64)
    pk = np.concatenate([rng.integers(-10, 2010, 30_000), np.full(50, 77)]).astype(np.int64)
    ranks = Ranks(ctl, 1)
    try:
        out, errs = ranks.run(lambda r, c: _radix_rank(r, c, 1, bk, pk, np.int64, steps=2, base=base))
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    ob, op = oracle_mod.inner_join(bk, pk)
    for step in range(2):
        b, p = out[0][step]
        assert b.size > pk.size  # the re-probe ran
        assert np.array_equal(b, ob) and np.array_equal(p, op)


@pytest.mark.parametrize("plan", ["sharded", "radix"])
@pytest.mark.parametrize("step", [0, 1, 2])
def test_rank_failure_is_collective(ctl, oracle_mod, plan, step):
    """Rank 1's job 0 fails locally at `step` (test hook): every rank's job 0 returns an
    error (the failing rank its own, the others HJ_ERR_RCCL 'a peer rank failed'), no rank
    hangs, and job 1 on the same communicators is correct."""
    from datafusion_parallelism_amd._lib import HJ_ERR_INVALID, HJ_ERR_RCCL, HjError

    world = 4
    rng = np.random.default_rng(step)
    bk, pk = _keys("dups", rng, 40_000, 100_000)
    ranks = Ranks(ctl, world, timeout_s=30, fail_at=(1, 0, step))

    def body(r, comm):
        b0, b1 = _split(bk.size, world, r)
        p0, p1 = _split(pk.size, world, r)
        keys = torch.from_numpy(bk[b0:b1]).cuda()
        probe = torch.from_numpy(pk[p0:p1]).cuda()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        if plan == "sharded":
            jobs = [comm.build_sharded_async(keys, b0, s.cuda_stream) for _ in range(2)]
        else:
            jobs = [comm.join_radix(keys, b0, probe, p0, s.cuda_stream) for _ in range(2)]
        status = None
        try:
            jobs[0].wait()
        except HjError as e:
            status = (e.status, str(e))
        if plan == "sharded":
            table, _ = jobs[1].table()
            try:
                b, p = table.probe(pk[p0:p1])
            finally:
                table.close()
            res = (b, p.astype(np.uint32) + p0)
        else:
            b, p = jobs[1].pairs()
            res = (b.cpu().numpy().astype(np.uint64), p.cpu().numpy().astype(np.uint32))
            del b, p
        for j in jobs:
            j.close()
        return status, res

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for r, (status, _) in enumerate(out):
        assert status is not None, f"rank {r}'s job 0 did not fail"
        if r == 1:
            assert status[0] == HJ_ERR_INVALID and "injected" in status[1]
        else:
            assert status[0] == HJ_ERR_RCCL and "peer rank failed" in status[1]
    ob, op = oracle_mod.inner_join(bk, pk)
    if plan == "sharded":
        b = np.concatenate([o[1][0] for o in out])
        p = np.concatenate([o[1][1] for o in out])
    else:
        b, p = _merge([o[1] for o in out])
    assert np.array_equal(b, ob) and np.array_equal(p, op)


def test_radix_probe_ids_past_32_bits_fail_collectively(ctl, oracle_mod):
    """a rank whose probe ids (probe_base + row) pass 2^32 notes the
    error before the plan's first status exchange, so every rank's job returns it (the others
    'a peer rank failed') instead of that rank returning alone while its peers block in the
    next collective; the next job on the same communicators is correct."""
    from datafusion_parallelism_amd._lib import HJ_ERR_INVALID, HJ_ERR_RCCL, HjError

    world = 4
    rng = np.random.default_rng(11)
    bk, pk = _keys("dense", rng, 20_000, 60_000)
    ranks = Ranks(ctl, world, timeout_s=30)

    def body(r, comm):
        b0, b1 = _split(bk.size, world, r)
        p0, p1 = _split(pk.size, world, r)
        keys = torch.from_numpy(bk[b0:b1]).cuda()
        probe = torch.from_numpy(pk[p0:p1]).cuda()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        bad = (1 << 32) - 10 if r == world - 1 else p0
        j0 = comm.join_radix(keys, b0, probe, bad, s.cuda_stream)
        j1 = comm.join_radix(keys, b0, probe, p0, s.cuda_stream)
        status = None
        try:
            j0.wait()
        except HjError as e:
            status = (e.status, str(e))
        b, p = j1.pairs()
        res = (b.cpu().numpy().astype(np.uint64), p.cpu().numpy().astype(np.uint32))
        del b, p
        j0.close()
        j1.close()
        return status, res

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for r, (status, _) in enumerate(out):
        assert status is not None, f"rank {r}'s job 0 did not fail"
        if r == world - 1:
            assert status[0] == HJ_ERR_INVALID and "32 bits" in status[1]
        else:
            assert status[0] == HJ_ERR_RCCL and "peer rank failed" in status[1]
    b, p = _merge([o[1] for o in out])
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(b, ob) and np.array_equal(p, op)


def test_radix_pairs_outlive_consumer_after_job_free(ctl, oracle_mod):
    """the pairs' tensors sit on job-owned blocks that return to the
    library's (not stream-ordered) cache when the job is freed. A consumer queued on the
    caller's stream behind a long kernel, then the tensors dropped and the job freed, then a
    new join started at once: the consumer still reads the first join's pairs."""
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    rng = np.random.default_rng(5)
    bk, pk = _keys("dense", rng, 200_000, 400_000)
    pk2 = (pk + 7) % max(int(bk.max()), 1)
    ranks = Ranks(ctl, 1)

    def body(r, comm):
        keys = torch.from_numpy(bk).cuda()
        probe = torch.from_numpy(pk).cuda()
        probe2 = torch.from_numpy(pk2).cuda()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            j0 = comm.join_radix(keys, 0, probe, 0, s.cuda_stream)
            b, p = j0.pairs()
            torch.cuda._sleep(200_000_000)  # the consumer waits behind a long kernel
            cb, cp = b.clone(), p.clone()
            del b, p
            j0.close()
            j1 = comm.join_radix(keys, 0, probe2, 0, s.cuda_stream)
            b1, p1 = j1.pairs()
            torch.cuda.synchronize()
            res = (cb.cpu().numpy().astype(np.uint64), cp.cpu().numpy().astype(np.uint32),
                   b1.cpu().numpy().astype(np.uint64), p1.cpu().numpy().astype(np.uint32))
            del b1, p1
            j1.close()
        return res

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    cb, cp, b1, p1 = out[0]
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(cb, ob) and np.array_equal(cp, op)
    ob2, op2 = oracle_mod.inner_join(bk, pk2)
    assert np.array_equal(b1, ob2) and np.array_equal(p1, op2)


# ---- relational exchanges behind the C ABI (hj_dist_shuffle / hj_dist_gather) -----------

def _dest(keys, world):
    """hj_partition_rows' hash map restated on the host (mix64 low bits)."""
    from test_distributed_gloo import _mix64

    return (_mix64(np.asarray(keys, np.int64)) & np.uint64(world - 1)).astype(np.int64)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("key_dtype", [np.int64, np.int32])
def test_shuffle_threads(ctl, world, key_dtype):
    """Every rank's received (keys, payload) = the rows of every source rank whose key hashes
    to it, ordered by (source rank, source row); payload columns of 8, 4, 2 and 1 bytes; an
    empty rank; two jobs back to back."""
    rng = np.random.default_rng(world * 7 + (key_dtype == np.int32))
    sizes = [int(x) for x in rng.integers(1000, 30000, world)]
    if world > 1:
        sizes[1] = 0
    keys = [rng.integers(-(2**31), 2**31 - 1, n).astype(key_dtype) for n in sizes]
    pay = [(rng.integers(-(2**62), 2**62, n), rng.integers(0, 2**31, n).astype(np.int32),
            rng.integers(-(2**15), 2**15, n).astype(np.int16), rng.integers(-128, 128, n).astype(np.int8))
           for n in sizes]
    ranks = Ranks(ctl, world)

    def body(r, comm):
        k = torch.from_numpy(keys[r]).cuda()
        cols = [torch.from_numpy(c).cuda() for c in pay[r]]
        torch.cuda.synchronize()
        jobs = [comm.shuffle(k, cols) for _ in range(2)]
        out = []
        for j in jobs:
            rk, rc = j.columns()
            out.append((rk.cpu().numpy(), [c.cpu().numpy() for c in rc]))
            del rk, rc
            j.close()
        return out

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for me in range(world):
        sel = [_dest(keys[s], world) == me if world > 1 else np.ones(len(keys[s]), bool) for s in range(world)]
        want_k = np.concatenate([keys[s][sel[s]] for s in range(world)])
        want_c = [np.concatenate([pay[s][i][sel[s]] for s in range(world)]) for i in range(4)]
        for step in range(2):
            got_k, got_c = out[me][step]
            assert np.array_equal(got_k, want_k), (me, step)
            for i in range(4):
                assert got_c[i].dtype == want_c[i].dtype and np.array_equal(got_c[i], want_c[i]), (me, step, i)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_gather_threads(ctl, world):
    """Every rank receives all ranks' rows in rank order (uneven, one empty rank)."""
    rng = np.random.default_rng(world)
    sizes = [int(x) for x in rng.integers(0, 5000, world)]
    sizes[0] = 0
    a = [rng.integers(-(2**62), 2**62, n) for n in sizes]
    b = [rng.integers(0, 100, n).astype(np.int8) for n in sizes]
    ranks = Ranks(ctl, world)

    def body(r, comm):
        cols = [torch.from_numpy(a[r]).cuda(), torch.from_numpy(b[r]).cuda()]
        torch.cuda.synchronize()
        j = comm.gather(cols)
        _, (ga, gb) = j.columns()
        res = (ga.cpu().numpy(), gb.cpu().numpy())
        del ga, gb
        j.close()
        return res

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for r in range(world):
        assert np.array_equal(out[r][0], np.concatenate(a)) and np.array_equal(out[r][1], np.concatenate(b))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tpch_plans_over_exchange_jobs(ctl, world):
    """C4/C5's plans with every exchange a job of the C ABI (tpch.q3_dist / q9_dist with a
    NativeExchange over the thread transport): each rank generates its block of the tables,
    and every rank's answer equals the one-GPU plan's on the whole tables."""
    from datafusion_parallelism_amd import tpch
    from datafusion_parallelism_amd.distributed import NativeExchange

    sf = 0.05
    whole = tpch.generate(sf, "cuda", seed=11, q9=True)
    want3 = tpch.q3(whole)
    want9 = tpch.q9(whole)
    del whole
    ranks = Ranks(ctl, world)

    def body(r, comm):
        t = tpch.generate(sf, "cuda", seed=11, q9=True, rank=r, world=world)
        ex = NativeExchange(comm, world)
        return tpch.q3_dist(t, exchange=ex), tpch.q9_dist(t, exchange=ex)

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for r in range(world):
        q3r, q9r = out[r]
        assert q3r == want3, (r, q3r, want3)
        assert q9r == want9, r


def test_exchange_failure_is_collective(ctl):
    """A rank whose shuffle fails locally (test hook at the partition) makes every rank's job
    fail, none hangs, and the next exchange on the same communicators is correct."""
    from datafusion_parallelism_amd._lib import HJ_ERR_INVALID, HJ_ERR_RCCL, HjError

    world = 4
    rng = np.random.default_rng(3)
    keys = [rng.integers(0, 10**6, 5000) for _ in range(world)]
    ranks = Ranks(ctl, world, timeout_s=30, fail_at=(2, 0, 1))

    def body(r, comm):
        k = torch.from_numpy(keys[r]).cuda()
        torch.cuda.synchronize()
        j0 = comm.shuffle(k, [k])
        j1 = comm.shuffle(k, [k])
        status = None
        try:
            j0.columns()
        except HjError as e:
            status = (e.status, str(e))
        rk, (rc,) = j1.columns()
        res = (rk.cpu().numpy(), rc.cpu().numpy())
        del rk, rc
        j0.close()
        j1.close()
        return status, res

    try:
        out, errs = ranks.run(body)
    finally:
        ranks.close()
    assert all(e is None for e in errs), errs
    for r, (status, (rk, rc)) in enumerate(out):
        assert status is not None
        if r == 2:
            assert status[0] == HJ_ERR_INVALID and "injected" in status[1]
        else:
            assert status[0] == HJ_ERR_RCCL and "peer rank failed" in status[1]
        want = np.concatenate([keys[s][_dest(keys[s], world) == r] for s in range(world)])
        assert np.array_equal(rk, want) and np.array_equal(rc, want)
