"""Multi-GPU hash join: one process per GPU, build side radix-sharded across ranks.

SURVEY.md §8(e): both sides are partitioned by hash bits so that rank g owns the keys
with ``mix64(key) & (G-1) == g`` (the reference's nearest relative is the high-bit shard
function of src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16; here the LOW
hash bits pick the rank because the table index uses the high 32 bits). The one
exchange step is an all-to-all of ``(key, global row id)`` over RCCL (torch.distributed
backend "nccl" on ROCm = RCCL over xGMI); each rank then builds and probes its shard
independently with the single-GPU kernels, emitting global ``(build_row, probe_row)``
pairs. There is no other collective on the data path.

The partition and local-join steps are pluggable only so that the exchange logic can be
exercised by world_size-2 ``gloo`` tests on a machine without a GPU; the default (and
only product) implementations are the HIP kernels.
"""
from __future__ import annotations

import contextlib
import ctypes
from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.distributed as dist

from . import _lib
from ._lib import HJ_ERR_RCCL, HJ_INT32, HJ_INT64, HjError, check
from .table import HashTable


@dataclass(frozen=True)
class PartSpec:
    """hj_part_spec: rows with keys outside [key_lo, key_hi] are dropped before the
    exchange; by_range maps contiguous key ranges to ranks (else the mix64 hash)."""
    by_range: bool = False
    key_lo: int = -(2**63)
    key_hi: int = 2**63 - 1

    def part_of(self, keys, nparts: int):
        """Host restatement of the device map (tests / host stand-ins): -> (dest, keep)."""
        import numpy as np

        k = np.asarray(keys).astype(np.int64)
        keep = (k >= self.key_lo) & (k <= self.key_hi)
        if not self.by_range:
            return None, keep
        rng = (self.key_hi - self.key_lo) + 1
        mul = min((nparts << 64) // rng, 2**64 - 1)
        off = [(int(x) - self.key_lo) % 2**64 for x in k.tolist()]
        return np.array([(o * mul) >> 64 for o in off], dtype=np.int64), keep


def gpu_radix_partition(keys: torch.Tensor, ids: torch.Tensor | None, id_base: int, nparts: int,
                        stream: int | None = None, id_dtype: torch.dtype = torch.int64,
                        key_offset: int | None = None, spec: PartSpec | None = None):
    """hj_partition_rows on device tensors -> (keys grouped by destination, ids
    (int64 = u64 build ids, int32 = u32 probe ids), counts[nparts] int64 device tensor).
    key_offset (int64 keys): the keys come out as int32(key - key_offset); spec: the
    destination map and runtime filter (default: hash map, nothing dropped). Dropped
    rows are not written: the outputs hold counts.sum() rows."""
    L = _lib.load()
    n = keys.numel()
    kt = HJ_INT64 if keys.dtype == torch.int64 else HJ_INT32
    narrow = key_offset is not None and keys.dtype == torch.int64
    out_k = torch.empty(n, dtype=torch.int32 if narrow else keys.dtype, device=keys.device)
    out_i = torch.empty(n, dtype=id_dtype, device=keys.device)
    counts = torch.zeros(nparts, dtype=torch.int64, device=keys.device)
    ws = torch.empty(max(L.hj_partition_workspace_bytes(n, nparts), 8), dtype=torch.uint8, device=keys.device)
    s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
    sp = None
    if spec is not None and spec != PartSpec():
        sp = ctypes.byref(_lib.HjPartSpec(int(spec.by_range), spec.key_lo, spec.key_hi))
    check(L.hj_partition_rows(kt, keys.data_ptr(), None, 0, None if ids is None else ids.data_ptr(), id_base, n,
                              nparts, sp, out_k.data_ptr(), out_k.element_size(), key_offset if narrow else 0,
                              out_i.data_ptr(), 8 if id_dtype == torch.int64 else 4, counts.data_ptr(),
                              ws.data_ptr(), s))
    return out_k, out_i, counts


def gpu_partition_regions(keys: torch.Tensor, ids: torch.Tensor | None, id_base: int, nparts: int,
                          cap: int | None = None, id_dtype: torch.dtype = torch.int64, key_offset: int | None = None,
                          spec: PartSpec | None = None, stream: int | None = None):
    """hj_partition_regions on device tensors: one pass over the rows into per-destination
    regions -> (keys, ids, counts[nparts] int64 device tensor, cap): region d's rows are
    keys[d * cap : d * cap + counts[d]] (source row order), likewise ids. cap defaults to
    the row count (any distribution fits)."""
    L = _lib.load()
    n = keys.numel()
    cap = max(n, 1) if cap is None else max(int(cap), 1)
    kt = HJ_INT64 if keys.dtype == torch.int64 else HJ_INT32
    narrow = key_offset is not None and keys.dtype == torch.int64
    out_k = torch.empty(nparts * cap, dtype=torch.int32 if narrow else keys.dtype, device=keys.device)
    out_i = torch.empty(nparts * cap, dtype=id_dtype, device=keys.device)
    counts = torch.empty(nparts, dtype=torch.int64, device=keys.device)
    ws = torch.empty(max(L.hj_partition_regions_workspace_bytes(n, nparts), 8), dtype=torch.uint8,
                     device=keys.device)
    s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
    sp = None
    if spec is not None and spec != PartSpec():
        sp = ctypes.byref(_lib.HjPartSpec(int(spec.by_range), spec.key_lo, spec.key_hi))
    check(L.hj_partition_regions(kt, keys.data_ptr(), None, 0, None if ids is None else ids.data_ptr(), id_base, n,
                                 nparts, sp, out_k.data_ptr(), out_k.element_size(), key_offset if narrow else 0,
                                 out_i.data_ptr(), 8 if id_dtype == torch.int64 else 4, cap, counts.data_ptr(),
                                 ws.data_ptr(), s))
    return out_k, out_i, counts, cap


def regions_from_grouped(k: torch.Tensor, i: torch.Tensor, counts: torch.Tensor, nparts: int):
    """Destination-grouped partition output (hj_partition_rows' layout, or a host stand-in's)
    as regions of cap = len(k) rows (tests' stand-ins feed the region exchange this way)."""
    cap = max(k.numel(), 1)
    rk = torch.zeros(nparts * cap, dtype=k.dtype, device=k.device)
    ri = torch.zeros(nparts * cap, dtype=i.dtype, device=i.device)
    c = [int(x) for x in counts.tolist()]
    at = 0
    for d in range(nparts):
        rk[d * cap:d * cap + c[d]] = k[at:at + c[d]]
        ri[d * cap:d * cap + c[d]] = i[at:at + c[d]]
        at += c[d]
    return rk, ri, counts, cap


class GpuLocalTable:
    """One rank's shard table (global build ids held in place of row numbers when they
    fit 31 bits and ascend, HJ_IDS_U31) and asynchronous probes of received chunks."""

    def __init__(self, build_keys: torch.Tensor, build_ids: torch.Tensor, ids_u31: bool | None = None,
                 key_range: tuple[int, int] | None = None, dense: bool = False):
        """ids_u31: the caller knows the ids ascend and are < 2^31 (DistributedHashJoin:
        stable partition, ranks in order, global build side < 2^31 rows); None checks.
        key_range: every build key lies in it (hj_build_key_range: no key-range reduction);
        dense: direct-addressed over key_range whatever the density (hj_build_dense)."""
        dev = build_keys.device
        kt = "int64" if build_keys.dtype == torch.int64 else "int32"
        # received build ids ascend (stable partition, ranks in order): when they also
        # fit 31 bits the table keeps them in place of row numbers (no id gather per pair)
        nbi = build_ids.numel()
        u31 = ids_u31
        if u31 is None:
            u31 = nbi == 0 or bool(((build_ids[-1] < 2**31) & (build_ids[0] >= 0) &
                                    (nbi < 2 or bool((build_ids[1:] > build_ids[:-1]).all()))).item())
        self.table = HashTable(1, kt, dev.index or 0)
        self.table.append(0, build_keys, ids=build_ids, ids_u31=u31)
        if key_range is not None and nbi:
            self.table.key_range(*key_range)
            if dense:
                self.table.dense()
        self.table.finish(0)
        self.device = dev

    def probe(self, probe_keys: torch.Tensor, probe_ids: torch.Tensor, capacity: int | None = None):
        """Enqueue the probe on the current stream (no host sync); returns a finaliser
        that waits and yields (build_idx int64 [u64 values], probe_idx int32 [u32])."""
        dev = self.device
        n = probe_keys.numel()
        pid32 = probe_ids if probe_ids.dtype == torch.int32 else probe_ids.to(torch.int32)
        ws = torch.empty(HashTable.workspace_bytes(n), dtype=torch.uint8, device=dev)
        d_total = torch.empty(1, dtype=torch.int64, device=dev)  # written by the probe
        cap = max(capacity or n, 1)
        s = torch.cuda.current_stream(dev).cuda_stream

        def launch(c):
            ob = torch.empty(c, dtype=torch.int64, device=dev)
            op = torch.empty(c, dtype=torch.int32, device=dev)
            self.table.probe_async(probe_keys.data_ptr(), n, ob.data_ptr(), op.data_ptr(), c, d_total.data_ptr(),
                                   ws.data_ptr(), s, probe_ids_ptr=pid32.data_ptr())
            return ob, op

        ob, op = launch(cap)
        read_total = host_read_async(d_total)  # waits for this probe only, not later work

        def result(total: int | None = None):
            """total: d_total already read by the caller (one host sync for many probes)."""
            nonlocal ob, op
            total = int(read_total()[0]) if total is None else total
            if total > cap:  # rare (duplicate-heavy keys): once more with the exact size
                ob, op = launch(total)
                total = int(d_total.item())
            return ob[:total], op[:total]

        result.d_total = d_total
        return result

    def close(self):
        self.table.close()


def gpu_local_join(build_keys: torch.Tensor, build_ids: torch.Tensor, probe_keys: torch.Tensor,
                   probe_ids: torch.Tensor, capacity_hint: int | None = None):
    """Build this rank's shard with explicit global build ids and probe it with global
    probe ids -> (build_idx int64 [u64 values], probe_idx int32 [u32 values])."""
    t = GpuLocalTable(build_keys, build_ids)
    try:
        return t.probe(probe_keys, probe_ids, capacity_hint)()
    finally:
        t.close()


@dataclass
class ExchangePlan:
    """What the exchange narrows and filters (DistributedHashJoin.prepare): keys travel
    as int32(key - key_offset) when key_offset is set, build ids as build_id_dtype;
    both sides use `spec` (probe rows outside the global build key range are dropped
    before the exchange; a dense build key domain is split into contiguous ranges)."""
    key_offset: int | None = None
    build_id_dtype: torch.dtype = torch.int64
    spec: PartSpec = field(default_factory=PartSpec)
    build_rows: int | None = None  # global build rows (received ids are checked against it)
    build_lo: int | None = None    # global build key range (None: unknown / empty)
    build_hi: int | None = None

    def local_key_range(self, rank: int, world: int) -> tuple[int, int] | None:
        """The key range of `rank`'s received build rows, in the travelling key domain
        (after narrowing): the rank's contiguous share of [build_lo, build_hi] under a range
        map (the partition kernel's multiply-high map, restated exactly), the whole range
        under the hash map; None when unknown."""
        if self.build_lo is None:
            return None
        lo, hi = self.build_lo, self.build_hi
        if self.spec.by_range and world > 1:
            rng = hi - lo + 1
            mul = min((world << 64) // rng, 2**64 - 1)
            first = lambda r: -(-(r << 64) // mul)  # smallest offset x with (x * mul) >> 64 >= r
            a, b = first(rank), first(rank + 1) - 1
            lo, hi = lo + a, min(hi, lo + b)
            if lo > hi:
                return None
        if self.key_offset is not None:
            lo, hi = lo - self.key_offset, hi - self.key_offset
        return lo, hi


@dataclass
class ExchangeStats:
    sent_rows: int = 0
    recv_rows: int = 0


# Bytes one rank sends or receives per all_to_all_single call. RCCL self-copies above
# ~800 MB come back wrong on this stack (tools/debug_shuffle.py: 1.6 GB -> the second
# half differs), so larger exchanges run in rounds of at most this size.
A2A_MAX_BYTES = 256 << 20


def concurrent_stream(device, avoid: torch.cuda.Stream | None = None, tries: int = 8,
                      priority: int = 0) -> torch.cuda.Stream:
    """A torch pool stream whose work runs concurrently with `avoid` (default: the current
    stream). HIP multiplexes streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 here)
    in creation order, and two streams on one queue run one after the other: a side stream
    that lands on the current stream's queue serializes every overlap a pipeline counts on
    (seen in kernel traces: the plan's key-range read queued behind the previous probe).
    Tested, not assumed: a spin kernel on `avoid`, a tiny one on the candidate, and the
    candidate must finish while the spin still runs. -> the first candidate that does (else
    the last one tried). priority: the HIP stream priority (-1 high, 0 normal)."""
    avoid = avoid or torch.cuda.current_stream(device)
    cand = None
    for _ in range(tries):
        cand = torch.cuda.Stream(device, priority=priority)
        if cand.cuda_stream == avoid.cuda_stream:
            continue
        spin_done = torch.cuda.Event()
        with torch.cuda.stream(avoid):
            torch.cuda._sleep(20_000_000)
            spin_done.record(avoid)
        mark = torch.cuda.Event()
        with torch.cuda.stream(cand):
            torch.cuda._sleep(1000)
            mark.record(cand)
        mark.synchronize()
        overlapped = not spin_done.query()
        spin_done.synchronize()
        if overlapped:
            return cand
    return cand


def host_read_async(t: torch.Tensor) -> Callable[[], list]:
    """Start reading a small device tensor to the host without blocking the stream: a
    non-blocking copy into pinned memory and an event, enqueued now (work the caller
    enqueues afterwards does not delay it). -> a callable that waits for the event only and
    returns t.tolist(). Host tensors are read at once."""
    if not t.is_cuda:
        vals = t.tolist()
        return lambda: vals
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()

    def get():
        ev.synchronize()
        return h.tolist()
    return get


def _count_matrix_async(counts: torch.Tensor, group=None) -> Callable[[], list[list[int]]]:
    """m[s][d] = rows rank s sends to rank d: one all_gather of G int64 (enqueued now; one
    rank: no collective) and an asynchronous host read. -> a callable that waits for the
    read only: every rank learns its receive sizes and everyone's, so all ranks agree on
    the number of exchange rounds without another collective."""
    world = dist.get_world_size(group)
    if world == 1:
        get = host_read_async(counts)
        return lambda: [get()]
    parts = [torch.empty_like(counts) for _ in range(world)]
    dist.all_gather(parts, counts, group=group)
    return host_read_async(torch.stack(parts))


def _count_matrix(counts: torch.Tensor, group=None) -> list[list[int]]:
    return _count_matrix_async(counts, group)()


def key_minmax(k: torch.Tensor, out: torch.Tensor) -> None:
    """out[0], out[1] = min, max of k (INT64_MAX, INT64_MIN when empty) into a device int64
    tensor: hj_key_minmax, one launch on the current stream (host tensors: torch)."""
    if not k.is_cuda:
        if k.numel():
            mn, mx = torch.aminmax(k.to(torch.int64))
            out[0], out[1] = mn, mx
        else:
            out[0], out[1] = 2**63 - 1, -(2**63)
        return
    L = _lib.load()
    ws = torch.empty(L.hj_key_minmax_workspace_bytes(), dtype=torch.uint8, device=k.device)
    kt = HJ_INT64 if k.dtype == torch.int64 else HJ_INT32
    check(L.hj_key_minmax(kt, k.data_ptr(), None, 0, k.numel(), out.data_ptr(), ws.data_ptr(),
                          torch.cuda.current_stream(k.device).cuda_stream))


def _exchange_cols(cols: list[torch.Tensor], m: list[list[int]], group=None, async_op: bool = False):
    """all_to_all_single of destination-grouped columns with the split sizes of count
    matrix m. -> (received columns, works still in flight). Exchanges larger than
    A2A_MAX_BYTES per rank run in rounds (each round moves the same fraction of every
    peer's segment; all ranks derive the round count from m)."""
    me = dist.get_rank(group)
    world = len(m)
    send = m[me]
    recv = [m[s][me] for s in range(world)]
    cols = [c[:sum(send)] for c in cols]  # rows the partition dropped are not sent
    widest = max(c.element_size() for c in cols) if cols else 1
    peak = max(max(sum(m[r]), sum(m[s][r] for s in range(world))) for r in range(world)) * widest
    rounds = max(1, -(-peak // A2A_MAX_BYTES))
    outs = [torch.empty(sum(recv), dtype=c.dtype, device=c.device) for c in cols]
    if rounds == 1:
        works = [dist.all_to_all_single(o, c, output_split_sizes=recv, input_split_sizes=send, group=group,
                                        async_op=async_op) for o, c in zip(outs, cols)]
        return outs, works
    s_off = [sum(send[:p]) for p in range(world)]
    r_off = [sum(recv[:p]) for p in range(world)]

    def piece(n, j):
        return n * j // rounds, n * (j + 1) // rounds

    for j in range(rounds):
        sj = [piece(send[p], j) for p in range(world)]
        rj = [piece(recv[p], j) for p in range(world)]
        ssz = [b - a for a, b in sj]
        rsz = [b - a for a, b in rj]
        for o, c in zip(outs, cols):
            tin = torch.cat([c[s_off[p] + a:s_off[p] + b] for p, (a, b) in enumerate(sj)])
            tout = torch.empty(sum(rsz), dtype=c.dtype, device=c.device)
            dist.all_to_all_single(tout, tin, output_split_sizes=rsz, input_split_sizes=ssz, group=group)
            q = 0
            for p, (a, b) in enumerate(rj):
                o[r_off[p] + a:r_off[p] + b].copy_(tout[q:q + b - a])
                q += b - a
    return outs, []


def check_counts(m: list[list[int]], cap: int, me: int = 0) -> None:
    """A region partition's counts (count matrix m: row s = rank s's counts) must be sane
    before anything is exchanged: hj_partition_regions reports a failed look-back (never
    expected) by counts of 2^60 or more, and a count above the region size means rows were
    not written. This rank's row is checked against its own region size `cap`, every row
    against the poison bound (each rank sees the same matrix, so all ranks raise together
    instead of exchanging wrong regions)."""
    for s, row in enumerate(m):
        for d, c in enumerate(row):
            if c < 0 or c >= 1 << 59 or (s == me and c > cap):
                raise HjError(_lib.HJ_ERR_HIP, f"region partition of rank {s}: count {c} for destination {d} "
                                               f"outside [0, {cap if s == me else '2^59'}] (device look-back "
                                               f"failure or region overflow)")


def exchange_regions(cols: list[torch.Tensor], cap: int, m: list[list[int]], group=None, async_op: bool = False):
    """Exchange per-destination regions (gpu_partition_regions' layout) with point-to-point
    sends and receives (RCCL ncclSend/ncclRecv in one group; xGMI links are point to point,
    so the per-peer messages of one rank use its links in parallel): -> (received columns,
    each the concatenation of the sources' rows in source-rank order, works in flight).
    The rank's own region is copied on the device (one rank: it is returned as is, no
    copy). Messages above A2A_MAX_BYTES travel in pieces (both sides derive the same
    split from the count matrix)."""
    me = dist.get_rank(group)
    world = len(m)
    check_counts(m, cap, me)
    recv = [m[s][me] for s in range(world)]
    if world == 1:
        return [c[:recv[0]] for c in cols], []
    r_off = [sum(recv[:p]) for p in range(world)]
    outs = [torch.empty(sum(recv), dtype=c.dtype, device=c.device) for c in cols]
    ops = []

    def pieces(nrows, esz):
        rounds = max(1, -(-nrows * esz // A2A_MAX_BYTES))
        return [(nrows * j // rounds, nrows * (j + 1) // rounds) for j in range(rounds)]

    peer_rank = (lambda p: dist.get_global_rank(group, p)) if group is not None else (lambda p: p)
    for c, o in zip(cols, outs):
        esz = c.element_size()
        if recv[me]:
            o[r_off[me]:r_off[me] + recv[me]].copy_(c[me * cap:me * cap + recv[me]])
        for p in range(world):
            if p == me:
                continue
            for a, b in pieces(m[me][p], esz):
                if b > a:
                    ops.append(dist.P2POp(dist.isend, c[p * cap + a:p * cap + b], peer_rank(p), group))
            for a, b in pieces(m[p][me], esz):
                if b > a:
                    ops.append(dist.P2POp(dist.irecv, o[r_off[p] + a:r_off[p] + b], peer_rank(p), group))
    works = dist.batch_isend_irecv(ops) if ops else []
    if not async_op:
        for w in works:
            w.wait()
        works = []
    return outs, works


def check_ids(ids: torch.Tensor, bound: int, what: str = "ids") -> None:
    """Raise if any of `ids` (received over an exchange, about to index something) lies
    outside [0, bound): the check runs on the device (min/max), one host read."""
    if ids.numel() == 0:
        return
    lo, hi = torch.aminmax(ids.to(torch.int64) if ids.dtype != torch.int64 else ids)
    lo, hi = int(lo.item()), int(hi.item())
    if lo < 0 or hi >= bound:
        raise HjError(HJ_ERR_RCCL, f"{what} out of range [0, {bound}) after the exchange: [{lo}, {hi}]")


def all_to_all_rows(keys_by_dest: torch.Tensor, ids_by_dest: torch.Tensor, counts: torch.Tensor,
                    group=None, async_op: bool = False):
    """Exchange destination-grouped rows: counts first (all_gather of G int64, host
    sync for the split sizes), then keys and ids with uneven splits (all_to_all_single).
    -> (keys, ids, stats[, works]); with async_op the row exchanges are left in flight
    (wait on `works` before using keys / ids)."""
    m = _count_matrix(counts, group)
    me = dist.get_rank(group)
    (rk, ri), works = _exchange_cols([keys_by_dest, ids_by_dest], m, group, async_op)
    st = ExchangeStats(sum(m[me]), sum(r[me] for r in m))
    if async_op:
        return rk, ri, st, works
    return rk, ri, st


def check_l(L, status: int) -> None:
    check(status, L)


class _DevArray:
    """A device buffer owned by a native job, exported to torch without a copy
    (``__cuda_array_interface__``): the tensor torch.as_tensor makes holds this object,
    which holds the job, so the job's memory lives as long as the tensor."""

    def __init__(self, ptr: int, n: int, typestr: str, owner):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr or 0, False),
                                         "version": 2}


_TYPESTR = {torch.int64: "<i8", torch.int32: "<i4", torch.int16: "<i2", torch.int8: "|i1", torch.uint8: "|u1",
            torch.bool: "|b1", torch.float64: "<f8", torch.float32: "<f4"}


def _tensor_any(ptr: int | None, n: int, dtype: torch.dtype, device: torch.device, owner) -> torch.Tensor:
    """A device tensor of `dtype` over a job-owned buffer (the owner lives as long as it)."""
    if n == 0 or not ptr:
        return torch.empty(0, dtype=dtype, device=device)
    return torch.as_tensor(_DevArray(ptr, n, _TYPESTR[dtype], owner), device=device)


def _tensor_of(ptr: int, n: int, dtype: torch.dtype, device: torch.device, owner) -> torch.Tensor:
    if n == 0 or not ptr:
        return torch.empty(0, dtype=dtype, device=device)
    ts = {torch.int64: "<i8", torch.int32: "<i4"}[dtype]
    return torch.as_tensor(_DevArray(ptr, n, ts, owner), device=device)


class NativeJob:
    """An hj_dist_job (one multi-GPU plan step queued on the communicator's worker thread):
    the caller's thread returns at once; table() / pairs() wait for the job's host steps."""

    def __init__(self, L, handle: ctypes.c_void_p, device: torch.device, keep=(), key_type: int = HJ_INT64):
        self._L, self._h, self.device, self._keep, self.key_type = L, handle, device, list(keep), key_type
        self._consumers = []  # torch streams current when pairs() handed out the job's buffers
        self.key_dtype, self.col_dtypes = None, []  # exchange jobs: the received columns' dtypes

    def wait(self):
        info = _lib.HjDistInfo()
        check_l(self._L, self._L.hj_dist_job_wait(self._h, ctypes.byref(info)))
        return info

    def table(self):
        """The job's table (the sharded build side: the whole build side) -> (HashTable,
        HjDistInfo); the table keeps the job's inputs alive."""
        h = ctypes.c_void_p()
        info = _lib.HjDistInfo()
        check_l(self._L, self._L.hj_dist_job_table(self._h, ctypes.byref(h), ctypes.byref(info)))
        return HashTable.from_handle(h, self.device.index or 0, self.key_type, keep=self._keep, lib=self._L), info

    def pairs(self):
        """A radix job's pairs -> (build_idx int64 [u64 values], probe_idx int32 [u32
        values]) as device tensors over the job's buffers (no copy)."""
        b, p, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check_l(self._L, self._L.hj_dist_job_pairs(self._h, ctypes.byref(b), ctypes.byref(p), ctypes.byref(n)))
        cur = torch.cuda.current_stream(self.device)
        if all(c != cur for c in self._consumers):
            self._consumers.append(cur)
        return (_tensor_of(b.value, n.value, torch.int64, self.device, self),
                _tensor_of(p.value, n.value, torch.int32, self.device, self))

    def columns(self):
        """An exchange job's received rows (hj_dist_job_columns; torch's current stream waits
        for the exchange) -> (keys or None, [columns]) as device tensors over the job's
        buffers (no copy), in the dtypes of the submitted columns."""
        n = len(self.col_dtypes)
        k = ctypes.c_void_p()
        cols = (ctypes.c_void_p * max(n, 1))()
        rows = ctypes.c_int64()
        stream = torch.cuda.current_stream(self.device)
        check_l(self._L, self._L.hj_dist_job_columns(self._h, stream.cuda_stream or None, ctypes.byref(k), cols, n,
                                                     ctypes.byref(rows)))
        if all(c != stream for c in self._consumers):
            self._consumers.append(stream)
        keys = None if self.key_dtype is None else _tensor_any(k.value, rows.value, self.key_dtype, self.device, self)
        return keys, [_tensor_any(cols[i], rows.value, dt, self.device, self) for i, dt in enumerate(self.col_dtypes)]

    def times(self) -> tuple[float, float, float]:
        """(build_ms, exchange_ms, probe_ms) of the finished job's device stages."""
        v = [ctypes.c_double() for _ in range(3)]
        check_l(self._L, self._L.hj_dist_job_times(self._h, *[ctypes.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def close(self):
        if getattr(self, "_h", None):
            # hj_dist_job_free returns the pairs' blocks to the library's cache, which is not
            # stream-ordered (the next job may reuse them at once): first wait for what the
            # consumers queued on the streams that held the tensors (the stream current at
            # pairs() and the one current now; a consumer on another stream must hold the
            # tensors, i.e. this job, until its work is done)
            streams = list(self._consumers)
            if torch.cuda.is_available():
                cur = torch.cuda.current_stream(self.device)
                if all(c != cur for c in streams):
                    streams.append(cur)
            for st in streams:
                ev = torch.cuda.Event()
                ev.record(st)
                ev.synchronize()
            self._L.hj_dist_job_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _JobRef:
    """What join() returns in place of a table on the native radix path: close() drops this
    reference only; the job (and the pairs' buffers) is freed once no result tensor refers
    to it."""

    def __init__(self, job):
        self.job = job

    def close(self):
        self.job = None


class NativeComm:
    """An hj_comm — the multi-GPU plans behind the C ABI (hj_dist.cpp, RCCL inside) — for
    the ranks of `group`: rank 0 makes the 128-byte unique id (hj_comm_unique_id), the group
    broadcasts it (the out-of-band channel a Rust host would provide itself), every rank
    creates the communicator on its GPU (hj_comm_create, collective). `lib` / `handle`:
    an already-made communicator of another library build (tests: the thread transport)."""

    def __init__(self, device: torch.device, group=None, lib=None, handle=None):
        self.device = device
        if handle is not None:
            self._L, self._h = lib, handle
            return
        L = self._L = _lib.load()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        idb = torch.zeros(_lib.HJ_COMM_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            check_l(L, L.hj_comm_unique_id(idb.data_ptr()))
        if self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            t = idb.to(device) if dist.get_backend(group) == "nccl" else idb
            dist.broadcast(t, src=src, group=group)
            idb = t.cpu()
        h = ctypes.c_void_p()
        check_l(L, L.hj_comm_create(self.rank, self.world, idb.data_ptr(), device.index or 0, ctypes.byref(h)))
        self._h = h

    @staticmethod
    def _kt(t: torch.Tensor | torch.dtype) -> int:
        dt = t if isinstance(t, torch.dtype) else t.dtype
        return HJ_INT64 if dt == torch.int64 else HJ_INT32

    def build_sharded_async(self, keys: torch.Tensor, build_base: int, stream: int, valid: torch.Tensor | None = None,
                            valid_offset: int = 0, probe_dtype: torch.dtype | None = None) -> NativeJob:
        """hj_dist_build_sharded_async on this rank's build keys (enqueued on `stream` by the
        worker) -> a NativeJob whose table() is the whole build side's table, keyed in the
        probe keys' type (default: the build keys')."""
        h = ctypes.c_void_p()
        pkt = self._kt(probe_dtype or keys.dtype)
        check_l(self._L, self._L.hj_dist_build_sharded_async(self._h, self._kt(keys), keys.data_ptr() if keys.numel() else None,
                                                  None if valid is None else valid.data_ptr(), valid_offset,
                                                  keys.numel(), build_base, pkt, stream or None, ctypes.byref(h)))
        return NativeJob(self._L, h, keys.device, keep=[keys, valid], key_type=pkt)

    def build_sharded(self, keys: torch.Tensor, build_base: int, stream: int, valid: torch.Tensor | None = None,
                      valid_offset: int = 0, probe_dtype: torch.dtype | None = None):
        """The same, waiting -> (the whole build side's table, HjDistInfo)."""
        job = self.build_sharded_async(keys, build_base, stream, valid, valid_offset, probe_dtype)
        try:
            return job.table()
        finally:
            job.close()

    def join_radix(self, build_keys: torch.Tensor, build_base: int, probe_keys: torch.Tensor, probe_base: int,
                   stream: int, build_valid: torch.Tensor | None = None, build_valid_offset: int = 0,
                   probe_valid: torch.Tensor | None = None, probe_valid_offset: int = 0) -> NativeJob:
        """hj_dist_join_radix: one radix-plan step -> a NativeJob whose pairs() are this
        rank's share of the join (global ids)."""
        h = ctypes.c_void_p()
        check_l(self._L, self._L.hj_dist_join_radix(
            self._h, self._kt(build_keys), build_keys.data_ptr() if build_keys.numel() else None,
            None if build_valid is None else build_valid.data_ptr(), build_valid_offset, build_keys.numel(), build_base,
            self._kt(probe_keys), probe_keys.data_ptr() if probe_keys.numel() else None,
            None if probe_valid is None else probe_valid.data_ptr(), probe_valid_offset, probe_keys.numel(), probe_base,
            stream or None, ctypes.byref(h)))
        return NativeJob(self._L, h, probe_keys.device, keep=[build_keys, probe_keys, build_valid, probe_valid])

    def shuffle(self, keys: torch.Tensor, payload: list[torch.Tensor], stream: int | None = None) -> NativeJob:
        """hj_dist_shuffle: hash repartition of `keys` (int32 / int64) with fixed-width payload
        columns -> a NativeJob whose columns() are the received (keys, payload), ordered by
        (source rank, source row)."""
        keys = keys.contiguous()
        payload = [p.contiguous() for p in payload]
        for p in payload:
            assert p.numel() == keys.numel(), "shuffle: payload columns of the keys' length"
        n = len(payload)
        ptrs = (ctypes.c_void_p * max(n, 1))(*[p.data_ptr() if p.numel() else None for p in payload])
        widths = (ctypes.c_int * max(n, 1))(*[p.element_size() for p in payload])
        s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
        h = ctypes.c_void_p()
        check_l(self._L, self._L.hj_dist_shuffle(self._h, self._kt(keys), keys.data_ptr() if keys.numel() else None,
                                                 keys.numel(), n, ptrs, widths, s or None, ctypes.byref(h)))
        job = NativeJob(self._L, h, keys.device, keep=[keys] + payload)
        job.key_dtype, job.col_dtypes = keys.dtype, [p.dtype for p in payload]
        return job

    def gather(self, cols: list[torch.Tensor], stream: int | None = None) -> NativeJob:
        """hj_dist_gather: every rank receives all ranks' rows of `cols` in rank order ->
        a NativeJob whose columns() are (None, the gathered columns)."""
        cols = [c.contiguous() for c in cols]
        n = cols[0].numel()
        for c in cols:
            assert c.numel() == n, "gather: columns of one length"
        ptrs = (ctypes.c_void_p * len(cols))(*[c.data_ptr() if c.numel() else None for c in cols])
        widths = (ctypes.c_int * len(cols))(*[c.element_size() for c in cols])
        s = stream if stream is not None else torch.cuda.current_stream(cols[0].device).cuda_stream
        h = ctypes.c_void_p()
        check_l(self._L, self._L.hj_dist_gather(self._h, n, len(cols), ptrs, widths, s or None, ctypes.byref(h)))
        job = NativeJob(self._L, h, cols[0].device, keep=cols)
        job.col_dtypes = [c.dtype for c in cols]
        return job

    def close(self):
        if getattr(self, "_h", None):
            self._L.hj_comm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


DENSE_FACTOR = 8                 # hj_api.cpp kDenseFactor: direct-addressed when range <= 8 x rows
DENSE_MAX_RANGE = 131071 << 11   # kMaxChunks << kDenseShift: the widest direct-addressed range


def gather_sizes(n: int, dev, group=None) -> list[int]:
    """Every rank's row count (one all_gather of one int64 and a host read)."""
    world = dist.get_world_size(group)
    if world == 1:
        return [int(n)]
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(ns, t, group=group)
    return [int(x) for x in torch.cat(ns).tolist()]


def broadcast_key_plan(build_keys: torch.Tensor, global_rows: int, group=None) -> tuple[int, int] | None:
    """(base, range) when the global int64 build keys make a direct-addressed table
    (range <= 8 x global rows, within the widest dense range): the broadcast plan then
    gathers int32 offsets key - base (half the exchange bytes and half the build's key
    reads) and builds with hj_build_key_range(0, range - 1) + hj_build_key_base(base), a
    table keyed by the int64 keys again. One hj_key_minmax launch on the shard, one 16-byte
    all-reduce (MIN over [min, ~max]) and a host read that waits for this stream only.
    None: keep int64 keys."""
    if build_keys.dtype != torch.int64 or global_rows <= 0:
        return None
    mm = torch.empty(2, dtype=torch.int64, device=build_keys.device)
    key_minmax(build_keys, mm)
    mm[1:].bitwise_not_()  # ~max is order-reversing: one MIN all-reduce gives both ends
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group)
    lo, nhi = host_read_async(mm)()
    hi = ~nhi
    if lo > hi:
        return None
    rng = hi - lo + 1
    if rng > DENSE_FACTOR * global_rows or rng > DENSE_MAX_RANGE:
        return None
    return lo, rng


class DistributedHashJoin:
    """Inner equi-join of a build and a probe column that are each spread over the ranks
    (rank r holds rows [base_r, base_r + n_r) of the global column).

    chunks > 1 pipelines the probe side: the all-to-all of chunk c runs (RCCL stream)
    while chunk c-1 is probed (compute stream); each rank's output is then canonical
    per chunk (the concatenation of the chunks' canonical outputs). `local_build_fn(bk,
    bi) -> table` with `table.probe(pk, pi, cap) -> result()` and `table.close()`
    default to GpuLocalTable."""

    def __init__(self, group=None, partition_fn: Callable | None = None, local_join_fn: Callable | None = None,
                 chunks: int = 1, local_build_fn: Callable | None = None, compress_keys: bool = True,
                 runtime_filter: bool = True, native: bool | None = None, comms: int | None = None):
        """native: run the plans through the C entry points (hj_dist_build_sharded_async,
        hj_dist_join_radix: RCCL inside the library, one job per step on a communicator's
        worker thread) instead of the torch.distributed steps below; None = when the group's
        backend is nccl (RCCL) and the world is a power of two. comms: native communicators
        used in turn, one step each, so that consecutive steps' host reads overlap (each has
        its own worker and streams); None = 2 on one rank, 1 on more. Two communicators'
        workers issue their collectives in an order that differs between ranks, and HIP
        multiplexes the communicators' streams onto GPU_MAX_HW_QUEUES hardware queues that
        run in submission order: a collective of one communicator queued behind the other's
        on one rank, and the reverse on another, would wait for each other. With one
        communicator every rank issues its collectives in job order on one stream."""
        self.group = group
        self.native = native
        self._comm: NativeComm | None = None
        self._comms: list[NativeComm] = []
        self.world = dist.get_world_size(group)
        self._ncomms = max(1, int(comms)) if comms is not None else (2 if self.world == 1 else 1)
        self._turn = 0
        self.last_native = False  # the latest join / join_sharded ran the C entry point
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.partition_fn = partition_fn or gpu_radix_partition
        self.local_join_fn = local_join_fn or gpu_local_join
        self.local_build_fn = local_build_fn or GpuLocalTable
        self.chunks = max(1, int(chunks))
        self.compress_keys = compress_keys
        self.runtime_filter = runtime_filter
        # optional stage events (bench): torch.cuda.Event objects recorded by join() /
        # join_sharded() when present: "build_start" / "build_end" bracket the build side on
        # its stream, "partitioned" / "exchanged" the exchange, "probe_start" the probe's
        # launch on the probe stream
        self.events: dict | None = None
        # prepare()'s key-range reads and its host read run on this stream when set. Only for
        # callers whose build keys are complete with respect to it (inputs resident before a
        # pipeline of joins starts): the next join's plan is then read while the previous
        # join's probe still runs, instead of queueing behind it on the current stream with
        # the device idle during the host read and the plan.
        self.prepare_stream: torch.cuda.Stream | None = None

    def prepare(self, build_keys: torch.Tensor, probe_keys: torch.Tensor, build_base: int) -> ExchangePlan:
        """Plan the exchange from the global key ranges (one hj_key_minmax launch per side,
        two 16-byte all-reduces and one host read; one rank: no collective):

        * runtime filter: probe rows outside the global build key range [bmin, bmax]
          cannot match and are dropped by the partition kernel before they travel;
        * range map: when the build key domain is dense (bmax - bmin + 1 <= 8 x the
          global build rows, the direct-addressed table's criterion), ranks own
          contiguous key ranges, so every local table is direct-addressed over 1/G of
          the domain (else the mix64 hash map);
        * narrowing: when the travelling keys span < 2^32 values they are written as
          int32(key - min - 2^31) (a bijection, so equality and the join are unchanged;
          the local tables then use int32 keys); build ids travel as u32 when the
          global build side has < 2^31 rows."""
        plan = ExchangePlan()
        if not (self.compress_keys or self.runtime_filter):
            return plan
        dev = build_keys.device
        # with the runtime filter only build-range keys travel: the probe range is not needed
        sides = (build_keys,) if self.runtime_filter else (build_keys, probe_keys)
        ps = self.prepare_stream if build_keys.is_cuda else None
        with torch.cuda.stream(ps) if ps is not None else contextlib.nullcontext():
            mm = torch.empty(2 * len(sides), dtype=torch.int64, device=dev)  # build min, max[, probe min, max]
            for j, k in enumerate(sides):
                key_minmax(k, mm[2 * j:2 * j + 2])
            bend = build_base + build_keys.numel()
            if self.world > 1:
                lo = mm[0::2].contiguous()  # [build min[, probe min]]
                hi = torch.cat([mm[1::2], torch.tensor([bend], dtype=torch.int64, device=dev)])
                vlo, vhi = self._allreduce_range(lo, hi)
                bmin, bmax, bend = vlo[0], vhi[0], vhi[-1]
                pmin, pmax = (vlo[1], vhi[1]) if len(sides) == 2 else (2**63 - 1, -(2**63))
            else:
                v = host_read_async(mm)()
                bmin, bmax = v[0], v[1]
                pmin, pmax = (v[2], v[3]) if len(sides) == 2 else (2**63 - 1, -(2**63))
        plan.build_rows = bend
        if bend < 2**31:
            plan.build_id_dtype = torch.int32
        if bmin > bmax:  # empty build side: nothing can match, nothing to plan
            return plan
        plan.build_lo, plan.build_hi = bmin, bmax
        if self.runtime_filter:
            dense = (bmax - bmin + 1) <= 8 * bend
            plan.spec = PartSpec(bool(dense and self.world > 1), bmin, bmax)
            gmin, gmax = bmin, bmax  # only keys in the build range travel
        else:
            gmin, gmax = min(bmin, pmin), max(bmax, pmax)
        if self.compress_keys and build_keys.dtype == torch.int64 and gmax - gmin < 2**32:
            plan.key_offset = gmin + 2**31
        return plan

    def _mark(self, name: str, stream=None) -> None:
        """Record stage event `name` (if the caller asked for it) on `stream` (default: the
        current stream)."""
        ev = self.events
        if ev is not None and name in ev:
            ev[name].record(stream)

    def _partition(self, keys: torch.Tensor, id_base: int, id_dtype: torch.dtype, key_offset: int | None,
                   spec: PartSpec | None = None):
        """-> per-destination regions (keys, ids, counts, cap) of gpu_partition_regions."""
        if self.partition_fn is gpu_radix_partition:
            return gpu_partition_regions(keys, None, id_base, self.world, id_dtype=id_dtype, key_offset=key_offset,
                                         spec=spec)
        # host stand-ins (tests): a grouped partition of the original keys, as regions
        if spec is not None and spec != PartSpec():
            k, i, c = self.partition_fn(keys, None, id_base, self.world, spec=spec)
        else:
            k, i, c = self.partition_fn(keys, None, id_base, self.world)
        if key_offset is not None and k.dtype == torch.int64:
            k = (k - key_offset).to(torch.int32)
        return regions_from_grouped(k, i.to(id_dtype), c, self.world)

    def shard(self, keys: torch.Tensor, id_base: int, id_dtype: torch.dtype = torch.int64, async_op: bool = False,
              key_offset: int | None = None, spec: PartSpec | None = None):
        """Partition by destination rank and exchange: -> (keys, global ids, stats[, works]).
        Build rows carry u64 ids (int64), probe rows u32 ids (int32, the reference's
        UInt32 probe index): 16 resp. 12 bytes per int64-key row on the wire, 8 with a
        narrowing plan (prepare)."""
        k, i, c, cap = self._partition(keys, id_base, id_dtype, key_offset, spec)
        m = _count_matrix(c, self.group)
        (rk, ri), works = exchange_regions([k, i], cap, m, self.group, async_op)
        me = self.rank
        st = ExchangeStats(sum(m[me]), sum(r[me] for r in m))
        if async_op:
            return rk, ri, st, works
        return rk, ri, st

    def shard_build(self, build_keys: torch.Tensor, build_base: int, plan: ExchangePlan,
                    global_rows: int | None = None):
        """The build side's exchange under `plan`: -> (keys, int64 global ids). With
        `global_rows`, the received ids are checked to lie in [0, global_rows) (one device
        reduction): a corrupted exchange raises instead of yielding out-of-range pair
        indices that a caller's gather would fault on."""
        bk, bi, _ = self.shard(build_keys, build_base, plan.build_id_dtype, key_offset=plan.key_offset,
                               spec=plan.spec)
        bi = bi.to(torch.int64) if bi.dtype != torch.int64 else bi
        if global_rows is not None:
            check_ids(bi, global_rows, "received build ids")
        return bk, bi

    def _local_table(self, bk: torch.Tensor, bi: torch.Tensor, plan: ExchangePlan):
        if self.local_build_fn is GpuLocalTable:
            # ids < 2^31 ascend (stable partition, ranks in order): held in place of rows;
            # the rank's key range is known from the plan: no key-range reduction
            return GpuLocalTable(bk, bi, ids_u31=True if plan.build_id_dtype == torch.int32 else None,
                                 key_range=plan.local_key_range(self.rank, self.world))
        return self.local_build_fn(bk, bi)

    @staticmethod
    def _order_build_stream(build_stream, cur, inputs_ready) -> None:
        """The side stream must not read the inputs before their producers wrote them: it
        waits for `inputs_ready` (an event the caller recorded after producing the keys),
        else for everything enqueued on the current stream so far (safe, but it then also
        waits for a previous join's probe there)."""
        if build_stream is None or cur is None:
            return
        if inputs_ready is not None:
            build_stream.wait_event(inputs_ready)
        else:
            build_stream.wait_stream(cur)

    def join(self, build_keys: torch.Tensor, build_base: int, probe_keys: torch.Tensor, probe_base: int,
             capacity_hint: int | None = None, check: bool = True, build_stream: torch.cuda.Stream | None = None,
             inputs_ready: torch.cuda.Event | None = None):
        """The radix plan, one pass per side: plan (one host read), both sides partitioned
        into per-destination regions, ONE count exchange for both (one host read), the
        build side's regions exchanged and built (asynchronously: a direct-addressed build
        overlaps the probe side's exchange), the probe side's exchanged and probed once.
        build_stream: the plan and the build side (partition, exchange, local build) run
        there, beside the probe side's partition on the current stream; the probe waits for
        the table only (its build event). The side stream first waits for `inputs_ready`
        (recorded by the caller once the keys exist), or without it for the current stream.
        -> (table, result): result() waits and yields this rank's pairs (canonical for
        its keys); close the table afterwards."""
        if self._use_native(build_keys) and self.compress_keys and self.runtime_filter:
            # (the C plan always narrows keys and filters probe rows by the build range)
            return self._join_native(build_keys, build_base, probe_keys, probe_base)
        self.last_native = False
        ev = self.events  # optional stage events (bench): partitioned, exchanged
        cur = torch.cuda.current_stream(probe_keys.device) if probe_keys.is_cuda else None
        self._order_build_stream(build_stream, cur, inputs_ready)
        bside = torch.cuda.stream(build_stream) if build_stream is not None else contextlib.nullcontext()
        with bside:
            self._mark("build_start")
            plan = self.prepare(build_keys, probe_keys, build_base)
            # build ids leave the partition as int64 (the table's id type: no widening pass; the
            # build side is the small one, 4 more bytes per row on the wire)
            bk_r, bi_r, bc, bcap = self._partition(build_keys, build_base, torch.int64, plan.key_offset, plan.spec)
            # each side's counts travel and are read as soon as its partition ends: the host
            # waits for the build side's counts while the probe side's partition runs, and for the
            # probe side's while the build runs, so the device does not idle on either read
            mb = _count_matrix_async(bc, self.group)
        pk_r, pi_r, pc, pcap = self._partition(probe_keys, probe_base, torch.int32, plan.key_offset, plan.spec)
        mp = _count_matrix_async(pc, self.group)
        if ev is not None:
            ev["partitioned"].record()
        with bside:
            (bk, bi), _ = exchange_regions([bk_r, bi_r], bcap, mb(), self.group)
            bi = bi.to(torch.int64) if bi.dtype != torch.int64 else bi
            if check and plan.build_rows is not None:
                check_ids(bi, plan.build_rows, "received build ids")
            table = self._local_table(bk, bi, plan)
            self._mark("build_end")
        (pk, pi), works = exchange_regions([pk_r, pi_r], pcap, mp(), self.group, async_op=True)
        for wk in works:
            if wk is not None:
                wk.wait()
        if ev is not None:
            ev["exchanged"].record()
        self._mark("probe_start")
        result = self._probe_chunk(table, pk, pi, [], capacity_hint)
        return table, result

    def _join_native(self, build_keys, build_base, probe_keys, probe_base):
        """The radix plan through the C entry point hj_dist_join_radix (RCCL inside the
        library): one job on the communicator's worker; the build side's kernels and the
        collectives on its side stream, the probe side's on the current stream. -> (job,
        result) as join()'s: result() waits and yields this rank's pairs (device tensors
        over the job's buffers, valid while they are referenced)."""
        self.last_native = True
        cur = torch.cuda.current_stream(probe_keys.device)
        job = self._next_comm(probe_keys.device).join_radix(build_keys, build_base, probe_keys, probe_base,
                                                            cur.cuda_stream)

        def result(total=None):
            return job.pairs()  # tensors over the job's buffers: they keep the job alive

        result.job = job
        return _JobRef(job), result

    def run(self, build_keys: torch.Tensor, build_base: int, probe_keys: torch.Tensor, probe_base: int,
            capacity_hint: int | None = None):
        """-> this rank's share of the global pairs (build_idx, probe_idx)."""
        if self.chunks <= 1:
            table, result = self.join(build_keys, build_base, probe_keys, probe_base, capacity_hint)
            try:
                return result()
            finally:
                table.close()
        plan = self.prepare(build_keys, probe_keys, build_base)
        bk, bi = self.shard_build(build_keys, build_base, plan, global_rows=plan.build_rows)
        outs = self.run_pipelined(bk, bi, probe_keys, probe_base, plan)
        return torch.cat([b for b, _ in outs]), torch.cat([p for _, p in outs])

    def run_pipelined(self, bk: torch.Tensor, bi: torch.Tensor, probe_keys: torch.Tensor, probe_base: int,
                      plan: ExchangePlan | None = None):
        """Local build, then the probe side in `chunks` slices. Every slice is partitioned
        up front and their counts travel in one all_gather (one host sync); then the
        exchange of slice c is in flight (RCCL P2P) while slice c-1 is probed (compute
        stream). -> list of per-chunk (build_idx, probe_idx)."""
        plan = plan or ExchangePlan()
        table = self._local_table(bk, bi, plan)
        try:
            n = probe_keys.numel()
            w = self.world
            bounds = [n * c // self.chunks for c in range(self.chunks + 1)]
            parts = [self._partition(probe_keys[bounds[c]:bounds[c + 1]], probe_base + bounds[c], torch.int32,
                                     plan.key_offset, plan.spec) for c in range(self.chunks)]
            mats = _count_matrix(torch.cat([p[2] for p in parts]), self.group)  # rank s: [chunk c, dest d]
            results, pending = [], None
            for c in range(self.chunks):
                m = [[row[c * w + d] for d in range(w)] for row in mats]
                (rk, ri), works = exchange_regions([parts[c][0], parts[c][1]], parts[c][3], m, self.group,
                                                   async_op=True)
                if pending is not None:
                    results.append(self._probe_chunk(table, *pending))
                pending = (rk, ri, works)
            results.append(self._probe_chunk(table, *pending))
            if all(hasattr(r, "d_total") for r in results):  # every chunk's match count in one host read
                totals = torch.cat([r.d_total for r in results]).tolist()
                return [r(t) for r, t in zip(results, totals)]
            return [r() for r in results]
        finally:
            table.close()

    # -- sharded-build broadcast plan --------------------------------------------------
    @staticmethod
    def sharded_ok(plan: ExchangePlan, world: int) -> bool:
        """The sharded-build plan needs a direct-addressed build domain split by key range
        (prepare's range map; one rank: the whole range), build ids held in place of rows
        (< 2^31 rows) and every piece's segment offsets, rebased, inside the packed refs'
        27 bits (2·B + 2·G + 2 < 2^27). The gathered table is one direct-addressed array
        over the whole build key range, so that range must also be within the widest
        direct-addressed range (DENSE_MAX_RANGE, as broadcast_key_plan requires): a wider
        one would be refused by hj_table_wrap_dense after the exchange."""
        if plan.build_lo is None or plan.build_rows is None or plan.build_id_dtype != torch.int32:
            return False
        rng = plan.build_hi - plan.build_lo + 1
        dense = rng <= DENSE_FACTOR * plan.build_rows and rng <= DENSE_MAX_RANGE
        return dense and (world == 1 or plan.spec.by_range) and 2 * plan.build_rows + 2 * world + 2 < 2**27

    def join_sharded(self, build_keys: torch.Tensor, build_base: int, probe_keys: torch.Tensor, probe_base: int,
                     capacity_hint: int | None = None, build_stream: torch.cuda.Stream | None = None,
                     inputs_ready: torch.cuda.Event | None = None, pending=None):
        """The sharded-build broadcast plan: the build side goes through the radix plan's
        range partition and exchange, each rank builds the direct-addressed table of its
        own contiguous key range (global build ids in place of rows), the ranks all-gather
        those pieces (and their duplicate segments, re-pointed at their place in the
        concatenated segment array) into one table, and each rank probes its own probe rows
        against it with the global probe ids base + row. No probe-side exchange and no
        replicated build: per rank 1/G of the build and B·4 bytes of table received, against
        the broadcast plan's whole build and B·4 bytes of keys. The ranks' outputs in rank
        order are the canonical output. build_stream: the build side (plan, partition,
        exchange, local build, gather) runs there and the probe on the current stream
        waits for the gathered table only (the side stream first waits for `inputs_ready`,
        or without it for the current stream). Falls back to run_broadcast's shape (whole
        build per rank) when sharded_ok is false. On the native path the build side is a
        job on the communicator's worker (start_sharded; `pending`: a job the caller started
        earlier for these build keys).
        -> (table, result): result() waits and yields this rank's pairs; close the table
        afterwards."""
        cur = torch.cuda.current_stream(probe_keys.device)
        if pending is None:
            pending = self.start_sharded(build_keys, build_base, build_stream, inputs_ready, probe_keys.dtype)
        if pending is not None:  # the native build side (a job queued on the communicator's worker)
            self.last_native = True
            table, _ = pending.table()  # waits for the job's host steps only
            pending.close()
            self._mark("probe_start", cur)
            return table, self._probe_own(table, probe_keys, probe_base, capacity_hint, cur)
        self.last_native = False
        bs = build_stream or cur
        with torch.cuda.stream(bs):
            self._mark("build_start", bs)
            plan = self.prepare(build_keys, probe_keys, build_base)
            if not self.sharded_ok(plan, self.world):
                return self._broadcast_table(build_keys, probe_keys, probe_base, capacity_hint, bs, cur)
            table = self._gather_pieces(build_keys, build_base, plan, probe_keys.dtype, bs)
            self._mark("build_end", bs)
        self._mark("probe_start", cur)
        result = self._probe_own(table, probe_keys, probe_base, capacity_hint, cur)
        return table, result

    def start_sharded(self, build_keys: torch.Tensor, build_base: int, build_stream: torch.cuda.Stream | None = None,
                      inputs_ready: torch.cuda.Event | None = None, probe_dtype: torch.dtype | None = None):
        """Queue the sharded plan's build side as a native job (hj_dist_build_sharded_async:
        the communicator's worker runs its host steps, the caller's thread returns at once)
        -> a NativeJob to hand to join_sharded(pending=...), or None when the native path
        is off (join_sharded then runs the torch.distributed steps itself). A caller that
        pipelines steps starts step k + 1's build side before step k's probe: its host
        reads then wait on the worker while the device runs the probe."""
        if not self._use_native(build_keys):
            return None
        cur = torch.cuda.current_stream(build_keys.device)
        self._order_build_stream(build_stream, cur, inputs_ready)
        bs = build_stream or cur
        return self._next_comm(build_keys.device).build_sharded_async(build_keys, build_base, bs.cuda_stream,
                                                                      probe_dtype=probe_dtype)

    def _next_comm(self, device) -> "NativeComm":
        """The native communicator of the next step (created on first use, collectively:
        every rank makes its communicators in the same order)."""
        if not hasattr(self, "_comms"):  # test doubles that skip __init__
            self._comms, self._ncomms, self._turn = [], 1, 0
        if len(self._comms) < self._ncomms:
            self._comms.append(NativeComm(device, self.group))
            self._comm = self._comms[0]
        c = self._comms[self._turn % len(self._comms)]
        self._turn += 1
        return c

    def _use_native(self, build_keys: torch.Tensor) -> bool:
        native = getattr(self, "native", None)
        if native is not None:
            return bool(native)
        if not build_keys.is_cuda or self.partition_fn is not gpu_radix_partition:
            return False
        if type(self)._exchange_build is not DistributedHashJoin._exchange_build:  # test doubles
            return False
        return dist.get_backend(self.group) == "nccl" and (self.world & (self.world - 1)) == 0

    def close(self) -> None:
        """Release the native communicators (if any were made)."""
        for c in getattr(self, "_comms", []):
            c.close()
        self._comms = []
        self._comm = None

    def _gather_pieces(self, build_keys, build_base, plan: ExchangePlan, probe_dtype, bs):
        dev = build_keys.device
        W, me = self.world, self.rank
        bk_r, bi_r, bc, bcap = self._partition(build_keys, build_base, torch.int64, plan.key_offset, plan.spec)
        self._mark("partitioned", bs)
        bk, bi = self._exchange_build(bk_r, bi_r, bc, bcap)
        self._mark("exchanged", bs)
        # every rank's key range, as the partition's range map cut it (they tile the domain)
        rngs = [plan.local_key_range(d, W) for d in range(W)]
        lens = [0 if r is None else r[1] - r[0] + 1 for r in rngs]
        offs = [sum(lens[:d]) for d in range(W)]
        full = torch.empty(sum(lens), dtype=torch.int32, device=dev)  # u32 refs of the whole domain
        mine = full.narrow(0, offs[me], lens[me])
        used = torch.zeros(1, dtype=torch.int64, device=dev)
        local = None
        if bk.numel() and lens[me]:
            # direct-addressed whatever the piece's density: a sparse piece exports refs too
            local = GpuLocalTable(bk, bi, ids_u31=True, key_range=rngs[me], dense=True)
            local.table.dense_export(refs=mine, dup_used=used, stream=bs.cuda_stream)
        elif lens[me]:
            mine.fill_(-1)  # no build rows in this range: every ref kMiss
        packed = 2 * plan.build_rows + 2 < 2**27
        try:
            if W > 1:
                self._allgather_var(full, offs, lens, mine)
            du = self._allgather_counts(used)  # segment words per piece (one host read)
            if sum(du):
                bases = [sum(du[:d]) for d in range(W)]
                dup = torch.empty(sum(du), dtype=torch.int32, device=dev)
                if local is not None and du[me]:
                    local.table.dense_export(dup=dup.narrow(0, bases[me], du[me]), stream=bs.cuda_stream)
                if W > 1:
                    self._allgather_var(dup, bases, du, dup.narrow(0, bases[me], du[me]))
                for d in range(W):
                    if du[d] and bases[d]:
                        HashTable.rebase_dups(full.narrow(0, offs[d], lens[d]), bases[d], packed, bs.cuda_stream)
            else:
                dup = torch.zeros(4, dtype=torch.int32, device=dev)
        finally:
            if local is not None:
                local.close()
        kt = "int64" if probe_dtype == torch.int64 else "int32"
        # the gathered table is keyed in the probe keys' domain: narrowing shifted only the
        # travelling build keys
        return HashTable.wrap_dense(dev.index or 0, kt, plan.build_lo, full, dup, packed, bs.cuda_stream)

    def _allreduce_range(self, lo: torch.Tensor, hi: torch.Tensor) -> tuple[list[int], list[int]]:
        """Element-wise MIN of lo and MAX of hi over the ranks -> host lists."""
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
        return lo.tolist(), hi.tolist()

    # the sharded-build plan's three communication steps (RCCL by default; tests replace
    # them to run several ranks as threads on one device)
    def _exchange_build(self, bk_r, bi_r, bc, bcap):
        """The build side's regions to their owners -> (keys, ids) this rank received."""
        if self.world == 1:
            n = int(host_read_async(bc)()[0])
            check_counts([[n]], bcap)
            return bk_r[:n], bi_r[:n]
        (bk, bi), _ = exchange_regions([bk_r, bi_r], bcap, _count_matrix(bc, self.group), self.group)
        return bk, bi

    def _allgather_var(self, out: torch.Tensor, offs: list[int], lens: list[int], src: torch.Tensor) -> None:
        """out[offs[d] : offs[d] + lens[d]] = rank d's src, on every rank (src may be a view
        of out)."""
        W = len(lens)
        if len(set(lens)) == 1 and offs == [lens[0] * d for d in range(W)] and out.numel() == sum(lens):
            dist.all_gather_into_tensor(out, src.clone(), group=self.group)
            return
        # uneven pieces (the range map's shares differ by a value or so): the plain all-gather
        # of pieces padded to the longest, then each piece to its place
        m = max(lens)
        pad = torch.empty(m, dtype=src.dtype, device=src.device)
        pad[:src.numel()].copy_(src)
        tmp = torch.empty(W * m, dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(tmp, pad, group=self.group)
        if out.numel() == sum(lens) and offs == [sum(lens[:d]) for d in range(W)]:
            # the pieces end to end: one cat kernel (one launch, not one copy per rank)
            torch.cat([tmp.narrow(0, d * m, lens[d]) for d in range(W)], out=out)
            return
        for d in range(W):
            if lens[d]:
                out.narrow(0, offs[d], lens[d]).copy_(tmp.narrow(0, d * m, lens[d]))

    def _allgather_counts(self, t: torch.Tensor) -> list[int]:
        """Every rank's one-element int64 device tensor -> host list (rank order)."""
        if self.world == 1:
            return [int(host_read_async(t)()[0])]
        allt = torch.empty(self.world, dtype=torch.int64, device=t.device)
        dist.all_gather_into_tensor(allt, t, group=self.group)
        return [int(x) for x in host_read_async(allt)()]

    def _probe_own(self, table: HashTable, probe_keys: torch.Tensor, probe_base: int, capacity_hint, cur):
        """This rank's probe rows against a finished table, probe idx = probe_base + row, on
        the current stream. -> result() as GpuLocalTable.probe's."""
        dev = probe_keys.device
        n = probe_keys.numel()
        ws = torch.empty(HashTable.workspace_bytes(n), dtype=torch.uint8, device=dev)
        d_total = torch.empty(1, dtype=torch.int64, device=dev)
        cap = max(capacity_hint or n, 1)

        def launch(c):
            ob = torch.empty(c, dtype=torch.int64, device=dev)
            op = torch.empty(c, dtype=torch.int32, device=dev)
            table.probe_async(probe_keys.data_ptr(), n, ob.data_ptr(), op.data_ptr(), c, d_total.data_ptr(),
                              ws.data_ptr(), cur.cuda_stream, probe_base=probe_base)
            return ob, op

        ob, op = launch(cap)
        read_total = host_read_async(d_total)

        def result(total: int | None = None):
            nonlocal ob, op
            total = int(read_total()[0]) if total is None else total
            if total > cap:
                ob, op = launch(total)
                total = int(d_total.item())
            return ob[:total], op[:total]

        result.d_total = d_total
        return result

    def _broadcast_table(self, build_keys, probe_keys, probe_base, capacity_hint, bs, cur):
        """Fallback of join_sharded: every rank builds the whole gathered build side."""
        dev = build_keys.device
        self._mark("partitioned", bs)
        sizes = gather_sizes(build_keys.numel(), dev, self.group)
        if self.world > 1:
            g = torch.empty(sum(sizes), dtype=build_keys.dtype, device=dev)
            dist.all_gather(list(torch.split(g, sizes)), build_keys, group=self.group)
        else:
            g = build_keys
        self._mark("exchanged", bs)
        table = HashTable(1, "int64" if g.dtype == torch.int64 else "int32", dev.index or 0)
        table.append(0, g)
        table.finish(0)
        table._keep.append(g)
        self._mark("build_end", bs)
        with torch.cuda.stream(cur):
            self._mark("probe_start", cur)
            result = self._probe_own(table, probe_keys, probe_base, capacity_hint, cur)
        return table, result

    # -- broadcast-build plan ------------------------------------------
    @staticmethod
    def choose_plan(build_rows: int, probe_rows: int, world: int) -> str:
        """'broadcast' when every rank receiving the whole build side moves fewer rows than
        the radix all-to-all of both sides (B·G < B + P), else 'radix'."""
        return "broadcast" if build_rows * world < build_rows + probe_rows else "radix"

    def run_broadcast(self, build_keys: torch.Tensor, probe_keys: torch.Tensor, probe_base: int,
                      capacity_hint: int | None = None):
        """Broadcast-build join: every rank all-gathers the build shards (rank order = the
        global canonical row order, so the local table's row numbers are the global build
        ids) and probes only its own probe rows: no probe-side exchange. -> this rank's
        pairs (global build idx int64, global probe idx int32); the ranks' outputs in rank
        order are the global canonical output. Needs equal-typed shards on every rank. When
        the global int64 build keys make a direct-addressed table (broadcast_key_plan), the
        shards travel as int32 offsets and the table is keyed back (hj_build_key_base)."""
        dev = build_keys.device
        n = probe_keys.numel()
        if self.local_join_fn is not gpu_local_join:  # host stand-in (gloo tests): explicit ids
            (gathered,) = all_gather_rows([build_keys], self.group)
            bi = torch.arange(gathered.numel(), dtype=torch.int64, device=dev)
            pi = torch.arange(probe_base, probe_base + n, dtype=torch.int64, device=dev).to(torch.int32)
            return self.local_join_fn(gathered, bi, probe_keys, pi, capacity_hint)
        sizes = gather_sizes(build_keys.numel(), dev, self.group)
        plan = broadcast_key_plan(build_keys, sum(sizes), self.group) if self.compress_keys else None
        src = build_keys if plan is None else (build_keys - plan[0]).to(torch.int32)
        (gathered,) = all_gather_rows([src], self.group, sizes=sizes)
        kt = "int64" if gathered.dtype == torch.int64 else "int32"
        with HashTable(1, kt, dev.index or 0) as t:  # canonical numbering = the global build ids
            t.append(0, gathered)
            if plan is not None:  # int32 offsets, keyed back to the int64 keys
                t.key_range(0, plan[1] - 1)
                t.key_base(plan[0])
            t.finish(0)
            ws = torch.empty(HashTable.workspace_bytes(n), dtype=torch.uint8, device=dev)
            d_total = torch.zeros(1, dtype=torch.int64, device=dev)
            cap = max(capacity_hint or n, 1)
            s = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(2):
                ob = torch.empty(cap, dtype=torch.int64, device=dev)
                op = torch.empty(cap, dtype=torch.int32, device=dev)
                t.probe_async(probe_keys.data_ptr(), n, ob.data_ptr(), op.data_ptr(), cap, d_total.data_ptr(),
                              ws.data_ptr(), s, probe_base=probe_base)  # global probe ids: base + row
                total = int(d_total.item())
                if total <= cap:
                    return ob[:total], op[:total]
                cap = total
        raise RuntimeError("unreachable")

    @staticmethod
    def _probe_chunk(table, rk, ri, works, capacity=None):
        for w in works:
            if w is not None:
                w.wait()  # RCCL: the compute stream waits for the exchange (no host block)
        return table.probe(rk, ri, capacity or rk.numel())


# ---- relational exchanges for multi-GPU query plans (TPC-H C4/C5, tpch.py) -------------

class TorchExchange:
    """A query plan's exchanges over torch.distributed (gloo on the CPU tests, or RCCL):
    `shuffle` (hash repartition with payload), `gather` (rows of every rank in rank order)
    and `sum` (an element-wise sum over the ranks)."""

    def __init__(self, group=None, partition_fn: Callable | None = None):
        self.group, self.partition_fn = group, partition_fn

    def shuffle(self, keys: torch.Tensor, payload: list[torch.Tensor]):
        return shuffle(keys, payload, self.group, self.partition_fn)

    def gather(self, cols: list[torch.Tensor]) -> list[torch.Tensor]:
        return all_gather_rows(cols, self.group)

    def sum(self, t: torch.Tensor) -> torch.Tensor:
        t = t.clone()
        dist.all_reduce(t, group=self.group)
        return t


class NativeExchange:
    """The same exchanges as jobs of an hj_comm behind the C ABI (hj_dist_shuffle /
    hj_dist_gather, RCCL inside the library, or the test library's thread transport): the
    whole query's data movement goes through include/hj.h, as a Rust host would drive it
    (INTEGRATION.md §8). `sum` gathers one row per rank and adds them on the device."""

    def __init__(self, comm: "NativeComm", world: int):
        self.comm, self.world = comm, world

    def shuffle(self, keys: torch.Tensor, payload: list[torch.Tensor]):
        job = self.comm.shuffle(keys, payload)
        k, cols = job.columns()
        return k, cols

    def gather(self, cols: list[torch.Tensor]) -> list[torch.Tensor]:
        _, out = self.comm.gather(cols).columns()
        return out

    def sum(self, t: torch.Tensor) -> torch.Tensor:
        (g,) = self.gather([t.reshape(-1)])
        return g.reshape(self.world, -1).sum(0).reshape(t.shape)


_NATIVE_COMMS: dict = {}


def default_exchange(group=None, partition_fn: Callable | None = None):
    """The plans' exchange for `group`: jobs of a (cached) hj_comm on an RCCL group with a
    power-of-two world and no stand-in partition function; torch.distributed otherwise."""
    if partition_fn is not None or dist.get_backend(group) != "nccl":
        return TorchExchange(group, partition_fn)
    world = dist.get_world_size(group)
    if world & (world - 1):
        return TorchExchange(group, partition_fn)
    dev = torch.device("cuda", torch.cuda.current_device())
    key = (id(group), dev.index)
    if key not in _NATIVE_COMMS:
        _NATIVE_COMMS[key] = NativeComm(dev, group)
    return NativeExchange(_NATIVE_COMMS[key], world)


def all_gather_rows(cols: list[torch.Tensor], group=None, sizes: list[int] | None = None) -> list[torch.Tensor]:
    """Broadcast exchange: every rank receives the concatenation, in rank order, of all
    ranks' rows of `cols` (equal-length columns). For the small, filtered dimension
    sides of a plan and the broadcast-build join (cheaper than a radix
    exchange whenever B·G < B + P). The row counts travel first (one all_gather and a host
    read) unless the caller passes `sizes`; equal counts gather straight into the output
    (all_gather_into_tensor, no padding or concatenation copies)."""
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    dev = cols[0].device
    if sizes is None:
        sizes = gather_sizes(cols[0].numel(), dev, group)
    ns = list(sizes)
    for c in cols:
        assert c.numel() == ns[me], "all_gather_rows: columns of unequal length"
    if all(k == ns[0] for k in ns):
        out = []
        for c in cols:
            o = torch.empty(ns[0] * world, dtype=c.dtype, device=c.device)
            dist.all_gather_into_tensor(o, c.contiguous(), group=group)
            out.append(o)
        return out
    m = max(max(ns), 1)
    out = []
    for c in cols:
        pad = torch.zeros(m, dtype=c.dtype, device=c.device)
        pad[:c.numel()] = c
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out.append(torch.cat([p[:k] for p, k in zip(parts, ns)]))
    return out


def shuffle(keys: torch.Tensor, payload: list[torch.Tensor], group=None, partition_fn: Callable | None = None):
    """Hash-repartition exchange (DataFusion's RepartitionExec Hash, over RCCL): row i goes
    to rank ``mix64(key) & (G-1)``, carrying its payload columns. Two sides shuffled by
    this function on the same key meet on one rank. It is NOT the map a
    DistributedHashJoin plan may choose (dense build domains go by key range there), so
    do not mix shuffle() output with a side partitioned by a join plan.

    hj_radix_partition is run with ids = local row numbers, so its id output is the
    stable destination permutation; payload columns are gathered by it and sent with the
    keys' split sizes (all_to_all_single, all columns in flight together).
    -> (received keys, received payload), ordered by (source rank, source row)."""
    world = dist.get_world_size(group)
    if partition_fn is None or partition_fn is gpu_radix_partition:
        k, perm, counts = gpu_radix_partition(keys, None, 0, world, id_dtype=torch.int64)
    else:
        k, perm, counts = partition_fn(keys, None, 0, world)
    perm = perm.to(torch.int64)
    m = _count_matrix(counts, group)
    outs, works = _exchange_cols([k] + [p[perm] for p in payload], m, group, async_op=True)
    for w in works:
        if w is not None:
            w.wait()
    return outs[0], outs[1:]
