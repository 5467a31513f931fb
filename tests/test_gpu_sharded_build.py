"""GPU: the sharded-build broadcast plan (DistributedHashJoin.join_sharded): each rank builds
the direct-addressed table of its own key range from the build rows the range exchange
brought it, the pieces (and their duplicate segments, re-pointed) are all-gathered into
one table, and each rank probes its own probe rows against it.

* one RCCL rank on the box's GPU, against the oracle (dense, far-from-zero, duplicate-heavy
  and sparse = the whole-build fallback);
* 2, 4 and 8 ranks as threads on the one GPU: the plan's own code with its three
  communication steps (range all-reduce, build exchange, variable all-gather) done by a
  thread barrier instead of RCCL, so the piece boundaries, the duplicate-segment rebase and
  empty pieces run at world > 1. The ranks' outputs in rank order must equal the oracle's
  canonical pairs of the whole join.
"""
import os
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
from conftest import init_one_rank_nccl

pytestmark = pytest.mark.gpu


def _keys(kind, rng, nb, np_):
    off = 2**62 if kind == "dense_far" else 0
    if kind == "sparse":
        bk = rng.integers(-(2**50), 2**50, nb)
        pk = np.concatenate([rng.choice(bk, np_ // 2), rng.integers(-(2**50), 2**50, np_ - np_ // 2)])
    elif kind == "dups":  # heavy duplicates: segments in every piece, some keys > 15 rows
        bk = np.concatenate([rng.integers(0, nb // 8, nb - 400), np.full(400, nb // 16)])
        rng.shuffle(bk)
        pk = rng.integers(-50, nb // 8 + 50, np_)
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


def _init_one_rank():
    init_one_rank_nccl()


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("kind", ["dense", "dense_far", "dups", "sparse"])
def test_sharded_build_one_rank(dfp, oracle_mod, kind, native):
    """native: the build side through the C entry point hj_dist_build_sharded (RCCL inside
    the library, the path a Rust host drives); else the torch.distributed steps."""
    from datafusion_parallelism_amd.distributed import DistributedHashJoin

    _init_one_rank()
    dj = None
    try:
        rng = np.random.default_rng(11)
        bk, pk = _keys(kind, rng, 150_000, 500_000)
        dj = DistributedHashJoin(native=native)
        side = torch.cuda.Stream()
        for _ in range(2):  # the second step reuses the communicator (and its deferred scratch)
            table, result = dj.join_sharded(torch.from_numpy(bk).cuda(), 0, torch.from_numpy(pk).cuda(), 7,
                                            build_stream=side)
            assert dj.last_native == native
            try:
                b, p = result()
            finally:
                table.close()
            ob, op = oracle_mod.inner_join(bk, pk)
            assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob)
            assert np.array_equal(p.cpu().numpy().astype(np.uint32), op + 7)
    finally:
        if dj is not None:
            dj.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["dense", "dups", "sparse"])
@pytest.mark.parametrize("key_type", ["int64", "int32"])
def test_native_build_sharded_nulls_and_base(dfp, oracle_mod, kind, key_type):
    """hj_dist_build_sharded directly (one rank): a validity bitmap with an offset, a
    nonzero build_base (global ids = base + row), int32 and int64 keys; the table probed
    with hj_probe_async_base equals the oracle with the ids shifted."""
    from datafusion_parallelism_amd import HashTable
    from datafusion_parallelism_amd.distributed import NativeComm

    _init_one_rank()
    comm = None
    try:
        rng = np.random.default_rng(5)
        bk, pk = _keys(kind, rng, 100_000, 300_000)
        if key_type == "int32":
            if kind == "sparse":
                bk, pk = (bk % (2**31)).astype(np.int32), (pk % (2**31)).astype(np.int32)
            else:
                bk, pk = bk.astype(np.int32), pk.astype(np.int32)
        valid = rng.random(bk.size + 3) > 0.1  # bit 3 is row 0
        bits = torch.from_numpy(np.packbits(valid, bitorder="little")).cuda()
        comm = NativeComm(torch.device("cuda", 0))
        s = torch.cuda.current_stream()
        table, info = comm.build_sharded(torch.from_numpy(bk).cuda(), 1000, s.cuda_stream, valid=bits,
                                         valid_offset=3)
        assert info.build_rows == 1000 + bk.size and info.sharded == (kind != "sparse")
        try:
            b, p = table.probe(torch.from_numpy(pk).cuda(), device_output=True)
            assert isinstance(table, HashTable)
        finally:
            table.close()
        ob, op = oracle_mod.inner_join(bk, pk, valid[3:], None)
        assert np.array_equal(b.cpu().numpy().astype(np.uint64), ob + 1000)
        assert np.array_equal(p.cpu().numpy().astype(np.uint32), op)
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


class _ThreadComm:
    """The collectives of W ranks that are threads of one process on one GPU."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slot = [None] * world

    def share(self, rank, value):
        """-> every rank's value (rank order); every rank's device work is finished first."""
        torch.cuda.synchronize()
        self.slot[rank] = value
        self.bar.wait()
        out = list(self.slot)
        self.bar.wait()
        return out


def _threaded_join(world, comm, rank, bk, pk, out, errs):
    from datafusion_parallelism_amd.distributed import DistributedHashJoin

    class Rank(DistributedHashJoin):
        def __init__(self):  # no process group: rank and world of the thread
            self.group, self.world, self.rank = None, world, rank
            self.partition_fn = None
            self.chunks, self.compress_keys, self.runtime_filter = 1, True, True
            self.events, self.prepare_stream = None, None

        def _partition(self, keys, id_base, id_dtype, key_offset, spec=None):
            from datafusion_parallelism_amd.distributed import gpu_partition_regions

            return gpu_partition_regions(keys, None, id_base, self.world, id_dtype=id_dtype, key_offset=key_offset,
                                         spec=spec)

        def _allreduce_range(self, lo, hi):
            all_ = comm.share(rank, (lo.tolist(), hi.tolist()))
            return ([min(v[0][j] for v in all_) for j in range(lo.numel())],
                    [max(v[1][j] for v in all_) for j in range(hi.numel())])

        def _exchange_build(self, bk_r, bi_r, bc, bcap):
            all_ = comm.share(rank, (bk_r, bi_r, bc.tolist(), bcap))
            ks = [k[rank * cap:rank * cap + c[rank]] for k, _, c, cap in all_]
            ids = [i[rank * cap:rank * cap + c[rank]] for _, i, c, cap in all_]
            return torch.cat(ks).contiguous(), torch.cat(ids).contiguous()

        def _allgather_var(self, out, offs, lens, src):
            all_ = comm.share(rank, src.clone())
            for d in range(world):
                out.narrow(0, offs[d], lens[d]).copy_(all_[d])

        def _allgather_counts(self, t):
            return [int(v) for v in comm.share(rank, int(t.item()))]

    try:
        B, P = bk.size, pk.size
        b0, b1 = B * rank // world, B * (rank + 1) // world
        p0, p1 = P * rank // world, P * (rank + 1) // world
        dj = Rank()
        table, result = dj.join_sharded(torch.from_numpy(bk[b0:b1]).cuda(), b0, torch.from_numpy(pk[p0:p1]).cuda(), p0)
        try:
            b, p = result()
            out[rank] = (b.cpu().numpy().astype(np.uint64), p.cpu().numpy().astype(np.uint32))
        finally:
            table.close()
    except BaseException as e:  # noqa: BLE001 - reported by the test
        errs.append((rank, repr(e)))
        comm.bar.abort()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("kind", ["dense", "dups", "clustered", "sparse_piece"])
def test_sharded_build_threads(dfp, oracle_mod, world, kind):
    rng = np.random.default_rng(world * 10 + len(kind))
    bk, pk = _keys(kind, rng, 120_000, 400_000)
    comm = _ThreadComm(world)
    out, errs = [None] * world, []
    ths = [threading.Thread(target=_threaded_join, args=(world, comm, r, bk, pk, out, errs)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs, errs
    assert all(o is not None for o in out)
    ob, op = oracle_mod.inner_join(bk, pk)
    assert np.array_equal(np.concatenate([o[0] for o in out]), ob)
    assert np.array_equal(np.concatenate([o[1] for o in out]), op)
