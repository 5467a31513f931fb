"""Thin RAII wrapper of one device hash table (``hj_table``) of the C ABI.

Accepts key columns as pyarrow Int32/Int64 arrays (host, zero-copy pointers incl. the
validity bitmap and offset), numpy int32/int64 arrays (+ optional boolean validity), or
torch int32/int64 tensors (device tensors are passed as device pointers).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Any

import numpy as np
import torch

from . import _lib
from ._lib import HJ_BORROW, HJ_BORROW_KEEP, HJ_IDS_U31, HJ_INPUT_DEVICE, HJ_INT32, HJ_INT64, HJ_OUTPUT_HOST, check

try:  # pyarrow is optional for the device path
    import pyarrow as pa
except ImportError:  # pragma: no cover
    pa = None


@dataclass
class KeyInput:
    ptr: int
    valid_ptr: int | None
    voff: int
    n: int
    flags: int
    key_type: int
    keepalive: Any


def _key_type_of_dtype(dt) -> int:
    if dt in (np.int64, torch.int64) or str(dt) in ("int64",):
        return HJ_INT64
    if dt in (np.int32, torch.int32) or str(dt) in ("int32",):
        return HJ_INT32
    raise TypeError(f"join keys must be int32 or int64, got {dt}")


def as_key_input(keys, valid=None, valid_offset: int = 0) -> KeyInput:
    """Normalise a key column into raw pointers for the C ABI. `valid`: a bool mask (one
    per row), or an LSB validity bitmap (uint8 tensor / array) whose bit `valid_offset` is
    row 0 — a device bitmap goes to the ABI as is (no host round trip)."""
    if pa is not None and isinstance(keys, pa.ChunkedArray):
        keys = keys.combine_chunks()
    if pa is not None and isinstance(keys, pa.Array):
        if pa.types.is_int64(keys.type):
            kt, isz = HJ_INT64, 8
        elif pa.types.is_int32(keys.type):
            kt, isz = HJ_INT32, 4
        else:
            raise TypeError(f"join keys must be Int32 or Int64, got {keys.type}")
        if valid is not None:
            raise ValueError("pyarrow arrays carry their own validity")
        bufs = keys.buffers()
        data = bufs[1]
        ptr = (data.address if data is not None else 0) + keys.offset * isz
        vptr = bufs[0].address if (bufs[0] is not None and keys.null_count > 0) else None
        return KeyInput(ptr, vptr, keys.offset if vptr else 0, len(keys), 0, kt, keys)
    if isinstance(keys, torch.Tensor):
        kt = _key_type_of_dtype(keys.dtype)
        t = keys.contiguous()
        flags = HJ_INPUT_DEVICE if t.is_cuda else 0
        vptr, keep_v, voff = None, None, 0
        if valid is not None:
            vb = torch.as_tensor(valid)
            if vb.dtype == torch.bool:  # mask -> LSB bitmap
                if valid_offset:
                    raise ValueError("valid_offset applies to a bitmap, not to a bool mask")
                bits = np.packbits(vb.cpu().numpy(), bitorder="little")
                vb = torch.from_numpy(bits)
            elif vb.dtype == torch.uint8:
                voff = int(valid_offset)
            else:
                raise TypeError("validity must be a bool mask or a uint8 bitmap")
            if t.is_cuda and not vb.is_cuda:
                vb = vb.to(t.device)
            keep_v = vb.contiguous()
            vptr = keep_v.data_ptr()
        return KeyInput(t.data_ptr(), vptr, voff, t.numel(), flags, kt, (t, keep_v))
    a = np.ascontiguousarray(np.asarray(keys))
    kt = _key_type_of_dtype(a.dtype)
    vptr, keep_v, voff = None, None, 0
    if valid is not None:
        va = np.asarray(valid)
        if va.dtype == np.uint8:  # already a bitmap
            bits, voff = np.ascontiguousarray(va), int(valid_offset)
        else:
            bits = np.packbits(va.astype(bool), bitorder="little")
        keep_v = bits
        vptr = bits.ctypes.data
    return KeyInput(a.ctypes.data if a.size else 0, vptr, voff, a.size, 0, kt, (a, keep_v))


def _producer_stream(keys, device: int) -> int | None:
    """torch's current stream for device tensors (the stream that produced them)."""
    if isinstance(keys, torch.Tensor) and keys.is_cuda:
        return torch.cuda.current_stream(keys.device).cuda_stream or None
    return None


def set_device_budget(nbytes: int) -> int:
    """hj_set_device_budget: per-table device byte budget of later builds (0 = none); a
    one-device build above it raises HjError(HJ_ERR_OOM). -> the previous budget."""
    return _lib.load().hj_set_device_budget(int(nbytes))


def is_budget_error(e: Exception) -> bool:
    """The HjError a build raises when it exceeds the device budget."""
    return isinstance(e, _lib.HjError) and e.status == _lib.HJ_ERR_OOM and "device budget" in str(e)


class HashTable:
    """One shared build table for `parallelism` partitions (hj_build_begin .. finish)."""

    def __init__(self, parallelism: int = 1, key_type: str | int = "int64", device: int = 0,
                 expected_rows: int = 0, devices: list[int] | None = None, plan: int | str = 0):
        """devices: a multi-GPU table over these GPUs (hj_build_begin_multi; repeats
        allowed), `plan` 0/"auto", 1/"broadcast" or 2/"radix"; else one table on `device`."""
        self._L = _lib.load()
        kt = key_type if isinstance(key_type, int) else (HJ_INT64 if key_type == "int64" else HJ_INT32)
        if key_type not in ("int64", "int32", HJ_INT32, HJ_INT64):
            raise TypeError(f"unsupported key type {key_type}")
        self.key_type = kt
        self.parallelism = parallelism
        self.device = devices[0] if devices else device
        self.devices = list(devices) if devices else None
        h = ctypes.c_void_p()
        if devices is not None:
            plan = {"auto": 0, "broadcast": 1, "radix": 2}.get(plan, plan) if isinstance(plan, str) else plan
            arr = (ctypes.c_int * len(devices))(*devices)
            check(self._L.hj_build_begin_multi(len(devices), arr, parallelism, kt, expected_rows, int(plan),
                                               ctypes.byref(h)))
        else:
            check(self._L.hj_build_begin(device, parallelism, kt, expected_rows, ctypes.byref(h)))
        self._h = h
        self._keep = []  # borrowed device inputs stay alive until the table is freed

    # -- build --------------------------------------------------------------
    def append(self, partition: int, keys, valid=None, ids=None, borrow: bool = True, ids_u31: bool = False,
               valid_offset: int = 0) -> None:
        """ids_u31: the explicit ids are < 2^31 and ascend in canonical row order (the
        table then stores them in place of row numbers, HJ_IDS_U31). valid: bool mask or
        LSB bitmap starting at bit valid_offset (as_key_input)."""
        ki = as_key_input(keys, valid, valid_offset)
        if ki.n and ki.key_type != self.key_type:
            raise TypeError("key type of the batch differs from the table's")
        # borrowed device inputs are kept alive (self._keep) until close(), which frees the
        # table first: the build may run on after finish() (HJ_BORROW_KEEP)
        flags = ki.flags | (HJ_BORROW | HJ_BORROW_KEEP if (borrow and ki.flags & HJ_INPUT_DEVICE) else 0)
        if ids is not None and ids_u31:
            flags |= HJ_IDS_U31
        ids_ptr, keep_ids = None, None
        if ids is not None:
            if isinstance(ids, torch.Tensor):
                keep_ids = ids.to(torch.int64).contiguous()
                ids_ptr = keep_ids.data_ptr()
            else:
                keep_ids = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
                ids_ptr = keep_ids.ctypes.data
        check(self._L.hj_build_append(self._h, partition, ki.ptr or None, ki.valid_ptr, ki.voff, ids_ptr, ki.n,
                                      flags, _producer_stream(keys, self.device)))
        if flags & HJ_BORROW:
            self._keep.append((ki.keepalive, keep_ids))

    def key_range(self, lo: int, hi: int) -> None:
        """hj_build_key_range: every valid build key lies in [lo, hi] (before the barrier);
        the build skips its key-range reduction."""
        check(self._L.hj_build_key_range(self._h, int(lo), int(hi)))

    def dense(self) -> None:
        """hj_build_dense: direct-addressed over the key_range whatever the density."""
        check(self._L.hj_build_dense(self._h))

    def key_base(self, base: int) -> None:
        """hj_build_key_base: this int32 table's build keys are offsets from `base`; once
        built, the table is keyed by base + offset and takes int64 probe keys (a
        direct-addressed table only; before the barrier)."""
        check(self._L.hj_build_key_base(self._h, int(base)))
        self._rekey = True

    def finish(self, partition: int) -> None:
        check(self._L.hj_build_finish(self._h, partition))
        if getattr(self, "_rekey", False):
            self.key_type = HJ_INT64

    def finish_all(self) -> None:
        """Call the barrier for every partition concurrently (one thread each), as
        DataFusion's executor does for the reference's partitions."""
        import threading

        errs = []

        def run(p):
            try:
                self.finish(p)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ths = [threading.Thread(target=run, args=(p,)) for p in range(self.parallelism)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errs:
            raise errs[0]

    def build(self, keys, valid=None, ids=None) -> "HashTable":
        """Single-partition convenience: append + finish."""
        self.append(0, keys, valid, ids)
        self.finish(0)
        return self

    def partition_offset(self, partition: int) -> int:
        v = ctypes.c_int64()
        check(self._L.hj_build_partition_offset(self._h, partition, ctypes.byref(v)))
        return v.value

    def stream_wait(self, stream: int = 0) -> None:
        """Order `stream` (a hipStream_t, 0 = the null stream) after the device build
        (hj_table_stream_wait; probes on any stream already wait by themselves)."""
        check(self._L.hj_table_stream_wait(self._h, stream or None))

    def build_ns(self) -> int:
        """Device time of the build (HIP events), no device work."""
        return self._L.hj_table_build_ns(self._h)

    def device_bytes(self) -> int:
        """Peak device bytes the build held (the device budget's measure; a multi-GPU
        table: its largest shard's)."""
        v = ctypes.c_int64()
        check(self._L.hj_table_device_bytes(self._h, ctypes.byref(v)))
        return v.value

    def stats(self) -> dict:
        s = _lib.HjTableStats()
        check(self._L.hj_table_stats_get(self._h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in s._fields_}

    # -- lookups ------------------------------------------------------------
    def lookup(self, key: int) -> list[int]:
        """IndexLookup::get_iter: build rows of `key`, newest first (descending)."""
        cnt = ctypes.c_int64()
        check(self._L.hj_table_lookup(self._h, int(key), None, 0, ctypes.byref(cnt)))
        out = np.empty(max(cnt.value, 1), dtype=np.uint64)
        check(self._L.hj_table_lookup(self._h, int(key), out.ctypes.data, cnt.value, ctypes.byref(cnt)))
        return [int(x) for x in out[: cnt.value]]

    def chain_links(self, nrows: int) -> np.ndarray:
        out = np.empty(max(nrows, 1), dtype=np.int64)
        check(self._L.hj_table_chain_links(self._h, out.ctypes.data, nrows))
        return out[:nrows]

    # -- probe --------------------------------------------------------------
    def probe(self, keys, valid=None, device_output: bool = False, valid_offset: int = 0):
        """Synchronous probe; returns (build_idx uint64, probe_idx uint32) in canonical
        order as numpy arrays, or as torch device tensors (int64, int32) with
        device_output=True (then keys must be a device tensor; a device bitmap `valid`
        with `valid_offset` is read in place)."""
        if device_output:
            return self._probe_device(keys, valid, valid_offset)
        ki = as_key_input(keys, valid, valid_offset)
        if ki.n and ki.key_type != self.key_type:
            raise TypeError("probe key type differs from the build key type")
        pr = _lib.HjPairs()
        flags = ki.flags | HJ_OUTPUT_HOST
        check(self._L.hj_probe(self._h, ki.ptr or None, ki.valid_ptr, ki.voff, ki.n, flags,
                               _producer_stream(keys, self.device), ctypes.byref(pr)))
        try:
            n = pr.count
            b = np.ctypeslib.as_array(pr.build_idx, shape=(n,)).copy() if n else np.empty(0, np.uint64)
            p = np.ctypeslib.as_array(pr.probe_idx, shape=(n,)).copy() if n else np.empty(0, np.uint32)
            return b, p
        finally:
            self._L.hj_pairs_free(ctypes.byref(pr))

    def _probe_device(self, keys: torch.Tensor, valid=None, valid_offset: int = 0):
        if not (isinstance(keys, torch.Tensor) and keys.is_cuda):
            raise TypeError("device_output=True takes a device tensor of keys")
        ki = as_key_input(keys, valid, valid_offset)
        if ki.n and ki.key_type != self.key_type:
            raise TypeError("probe key type differs from the build key type")
        dev = keys.device
        ws = torch.empty(self.workspace_bytes(ki.n), dtype=torch.uint8, device=dev)
        d_total = torch.zeros(1, dtype=torch.int64, device=dev)
        cap = max(ki.n, 1)
        stream = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(2):
            ob = torch.empty(cap, dtype=torch.int64, device=dev)
            op = torch.empty(cap, dtype=torch.int32, device=dev)
            self.probe_async(ki.ptr, ki.n, ob.data_ptr(), op.data_ptr(), cap, d_total.data_ptr(), ws.data_ptr(),
                             stream, ki.valid_ptr, ki.voff)
            total = int(d_total.item())
            if int(ws[8:16].view(torch.int64).item()) != 0:
                raise _lib.HjError(_lib.HJ_ERR_HIP, "probe look-back timed out")
            if total <= cap:
                return ob[:total], op[:total]
            cap = total
        raise RuntimeError("unreachable")

    def probe_async(self, keys_ptr: int, n: int, out_build_ptr: int, out_probe_ptr: int, capacity: int,
                    d_total_ptr: int, workspace_ptr: int, stream: int = 0, valid_ptr: int | None = None,
                    voff: int = 0, probe_ids_ptr: int | None = None, probe_base: int = 0) -> None:
        """hj_probe_async(_ids, _base) on raw device pointers (no sync, no allocation):
        probe_idx = row, probe_ids[row], or probe_base + row (ids and a base together are
        refused: the ids are the probe indices)."""
        if probe_ids_ptr is not None and probe_base:
            raise ValueError("probe_ids_ptr and probe_base are exclusive: add the base to the ids")
        if probe_ids_ptr is None and probe_base:
            check(self._L.hj_probe_async_base(self._h, keys_ptr, valid_ptr, voff, n, probe_base, out_build_ptr,
                                              out_probe_ptr, capacity, d_total_ptr, workspace_ptr, stream or None))
        elif probe_ids_ptr is None:
            check(self._L.hj_probe_async(self._h, keys_ptr, valid_ptr, voff, n, out_build_ptr, out_probe_ptr,
                                         capacity, d_total_ptr, workspace_ptr, stream or None))
        else:
            check(self._L.hj_probe_async_ids(self._h, keys_ptr, valid_ptr, voff, probe_ids_ptr, n, out_build_ptr,
                                             out_probe_ptr, capacity, d_total_ptr, workspace_ptr, stream or None))

    # -- sharded-build broadcast plan (hj_table_dense_piece / hj_table_wrap_dense) -------
    def dense_piece(self) -> dict:
        """A built direct-addressed table's arrays (device pointers): refs, nvalues,
        key_min, dup_rows, dup_used (device pointer to a u64), packed."""
        refs, dup, used = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        nv, kmin, packed = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int()
        check(self._L.hj_table_dense_piece(self._h, ctypes.byref(refs), ctypes.byref(nv), ctypes.byref(kmin),
                                           ctypes.byref(dup), ctypes.byref(used), ctypes.byref(packed)))
        return {"refs": refs.value or 0, "nvalues": nv.value, "key_min": kmin.value, "dup_rows": dup.value or 0,
                "dup_used": used.value or 0, "packed": bool(packed.value)}

    def dense_export(self, refs: torch.Tensor | None = None, v0: int = 0, dup: torch.Tensor | None = None,
                     dup_used: torch.Tensor | None = None, stream: int = 0) -> None:
        """Device copies of the refs [v0, v0 + refs.numel()), the first dup.numel() segment
        words and the segment words in use (one int64) into the given tensors, on `stream`."""
        check(self._L.hj_table_dense_export(self._h, None if refs is None else refs.data_ptr(), v0,
                                            0 if refs is None else refs.numel(),
                                            None if dup is None else dup.data_ptr(), 0 if dup is None else dup.numel(),
                                            None if dup_used is None else dup_used.data_ptr(), stream or None))

    @classmethod
    def wrap_dense(cls, device: int, key_type: str | int, key_min: int, refs: torch.Tensor,
                   dup_rows: torch.Tensor, packed: bool, stream: int = 0) -> "HashTable":
        """A probe-only table over device tensors (int32/uint32 views of the u32 refs and
        segments), kept alive by the table: refs[v] for key key_min + v."""
        self = cls.__new__(cls)
        self._L = _lib.load()
        kt = key_type if isinstance(key_type, int) else (HJ_INT64 if key_type == "int64" else HJ_INT32)
        self.key_type, self.parallelism, self.device, self.devices = kt, 1, device, None
        h = ctypes.c_void_p()
        check(self._L.hj_table_wrap_dense(device, kt, int(key_min), refs.numel(), refs.data_ptr(),
                                          dup_rows.data_ptr(), int(bool(packed)), stream or None, ctypes.byref(h)))
        self._h = h
        self._keep = [refs, dup_rows]
        return self

    @classmethod
    def from_handle(cls, handle: ctypes.c_void_p, device: int, key_type: str | int, keep=(), lib=None) -> "HashTable":
        """Adopt a built table handle another entry point returned (hj_dist_build_sharded);
        `keep`: tensors its build still reads, kept alive until close(); `lib`: the library
        that made it (tests: the thread-transport build), default the product library."""
        self = cls.__new__(cls)
        self._L = lib or _lib.load()
        kt = key_type if isinstance(key_type, int) else (HJ_INT64 if key_type == "int64" else HJ_INT32)
        self.key_type, self.parallelism, self.device, self.devices = kt, 1, device, None
        self._h = handle
        self._keep = list(keep)
        return self

    @staticmethod
    def rebase_dups(refs: torch.Tensor, base: int, packed: bool, stream: int = 0) -> None:
        """hj_dense_rebase_dups on a (view of a) u32 refs tensor."""
        check(_lib.load().hj_dense_rebase_dups(refs.data_ptr(), refs.numel(), int(base), int(bool(packed)),
                                               stream or None))

    @staticmethod
    def workspace_bytes(n: int) -> int:
        return _lib.load().hj_probe_workspace_bytes(n)

    # -- lifetime -----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.hj_table_free(self._h)
            self._h = None
            self._keep.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
