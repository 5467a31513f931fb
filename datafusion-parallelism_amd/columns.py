"""Device-resident Arrow columns and the index primitives of the join types
(SURVEY.md §8f rows f1 and f2), over the C ABI's hj_gather_* / hj_mark_rows /
hj_select_rows kernels.

  reference                                                   here
  ---------------------------------------------------------   ------------------------------
  take_multiple_record_batch (src/shared/shared.rs:83-92)     DeviceColumn.take
  ConcurrentBitSet::set_ones (src/utils/concurrent_bit_set.rs:28-60)
                                                              mark_rows
  get_set_indices_array / get_unset_indices_array,
  get_semi_indices / get_anti_indices
    (src/shared/datafusion_private.rs:85-135)                 select_rows

Index tensors: int64 (build side, the reference's UInt64) or int32 (probe side, UInt32);
-1 is a null index (the outer joins' missing side). Buffers move between host and HBM
only in `from_arrow` / `to_arrow`; the gathers run on the GPU (no CPU fallback).
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import numpy as np
import pyarrow as pa
import torch

from . import _lib
from ._lib import check

_VAR = {pa.string(): 4, pa.binary(): 4, pa.large_string(): 8, pa.large_binary(): 8}


def _is_var(t: pa.DataType) -> bool:
    return t in _VAR


def _fixed_width(t: pa.DataType) -> int:
    if pa.types.is_boolean(t):
        return 1  # held as one byte per value on the device
    try:
        w = t.bit_width
    except ValueError as e:
        raise TypeError(f"column type {t} is not supported on the device") from e
    if w % 8 or w // 8 not in (1, 2, 4, 8, 16):
        raise TypeError(f"column type {t} is not supported on the device")
    return w // 8


def _to_device(buf: np.ndarray, device) -> torch.Tensor:
    # Arrow buffers are read-only; the host tensor is only read by the copy to HBM
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        host = torch.from_numpy(np.ascontiguousarray(buf))
    return host.to(device)


def _bitmap_bytes(n: int) -> int:
    return ((n + 63) // 64) * 8


def _stream(device) -> int | None:
    return torch.cuda.current_stream(device).cuda_stream or None


@dataclass
class DeviceColumn:
    """One Arrow column in HBM: `data` (fixed width) or `offsets` + `values` (Utf8 /
    Binary, 4- or 8-byte offsets), optional LSB validity bitmap starting at bit `voff`."""
    type: pa.DataType
    length: int
    data: torch.Tensor | None = None
    offsets: torch.Tensor | None = None
    values: torch.Tensor | None = None
    valid: torch.Tensor | None = None
    voff: int = 0

    @property
    def device(self):
        t = self.data if self.data is not None else self.offsets
        return t.device

    @classmethod
    def from_arrow(cls, arr: pa.Array | pa.ChunkedArray, device) -> "DeviceColumn":
        if isinstance(arr, pa.ChunkedArray):
            arr = arr.combine_chunks()
        t, n, off = arr.type, len(arr), arr.offset
        bufs = arr.buffers()
        valid = None
        voff = 0
        if arr.null_count > 0 and bufs[0] is not None:
            vb = np.frombuffer(bufs[0], dtype=np.uint8)
            valid, voff = _to_device(vb, device), off
        if _is_var(t):
            ob = _VAR[t]
            odt = np.int32 if ob == 4 else np.int64
            offs = np.frombuffer(bufs[1], dtype=odt)[off:off + n + 1]
            vals = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
            return cls(t, n, offsets=_to_device(offs, device), values=_to_device(vals if vals.size else
                                                                                np.zeros(1, np.uint8), device),
                       valid=valid, voff=voff)
        if pa.types.is_boolean(t):
            data = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False), dtype=np.uint8)
            return cls(t, n, data=_to_device(data if n else np.zeros(1, np.uint8), device), valid=valid, voff=voff)
        w = _fixed_width(t)
        raw = np.frombuffer(bufs[1], dtype=np.uint8)[off * w:(off + n) * w]
        return cls(t, n, data=_to_device(raw if raw.size else np.zeros(w, np.uint8), device), valid=valid,
                   voff=voff)

    def take(self, idx: torch.Tensor) -> "DeviceColumn":
        """Arrow take by device indices (int32 / int64, -1 = null) on the GPU."""
        L = _lib.load()
        if idx.dtype not in (torch.int32, torch.int64):
            raise TypeError("indices must be int32 or int64")
        idx = idx.contiguous()
        n = idx.numel()
        dev = self.device
        ib = 8 if idx.dtype == torch.int64 else 4
        dvalid = torch.empty(max(_bitmap_bytes(n), 8), dtype=torch.uint8, device=dev)
        vptr = self.valid.data_ptr() if self.valid is not None else None
        s = _stream(dev)
        if _is_var(self.type):
            ob = _VAR[self.type]
            out_off = torch.empty(n + 1, dtype=torch.int32 if ob == 4 else torch.int64, device=dev)
            ws = torch.empty(L.hj_gather_var_workspace_bytes(n), dtype=torch.uint8, device=dev)
            d_len = torch.zeros(1, dtype=torch.int64, device=dev)
            cap = max(int(self.values.numel()), 1) if n else 1
            for _ in range(2):
                out_val = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
                check(L.hj_gather_var(self.offsets.data_ptr(), ob, self.values.data_ptr(), vptr, self.voff,
                                      idx.data_ptr() if n else None, ib, n, out_off.data_ptr(), out_val.data_ptr(),
                                      cap, dvalid.data_ptr(), d_len.data_ptr(), ws.data_ptr(), s))
                need = int(d_len.item())
                if need <= cap:
                    break
                cap = need
            if ob == 4 and need >= 2**31:
                raise _lib.HjError(_lib.HJ_ERR_CAPACITY, "gathered Utf8 column exceeds 2^31 bytes: use LargeUtf8")
            return DeviceColumn(self.type, n, offsets=out_off, values=out_val, valid=dvalid, voff=0)
        w = _fixed_width(self.type)
        dst = torch.empty(max(n * w, w), dtype=torch.uint8, device=dev)
        check(L.hj_gather_fixed(self.data.data_ptr(), vptr, self.voff, w, idx.data_ptr() if n else None, ib, n,
                                dst.data_ptr(), dvalid.data_ptr(), s))
        return DeviceColumn(self.type, n, data=dst, valid=dvalid, voff=0)

    def key_tensor(self) -> torch.Tensor:
        """An Int32 / Int64 column's values as a device tensor (no copy)."""
        if pa.types.is_int64(self.type):
            return self.data.view(torch.int64)[: self.length]
        if pa.types.is_int32(self.type):
            return self.data.view(torch.int32)[: self.length]
        raise TypeError(f"{self.type} is not an Int32/Int64 key column")

    def valid_bools(self) -> torch.Tensor | None:
        """The validity bitmap as one bool per row (device), or None without nulls."""
        if self.valid is None:
            return None
        i = torch.arange(self.length, dtype=torch.int64, device=self.device) + self.voff
        return ((self.valid[i >> 3] >> (i & 7).to(torch.uint8)) & 1).bool()

    @classmethod
    def concat(cls, cols: list["DeviceColumn"]) -> "DeviceColumn":
        """Arrow concat of columns of one type, on the device (the build side's
        cooperative concatenation in canonical order,
        src/operator/version10/parallel_join_execution_state.rs:256-298,317-347): fixed
        width values and Utf8/Binary values are copied device to device, offsets re-based,
        validity bitmaps re-packed from bit 0. One host read: the value ranges of the
        variable-width pieces."""
        if not cols:
            raise ValueError("concat of no columns")
        t = cols[0].type
        if any(c.type != t for c in cols):
            raise TypeError("concat of columns of different types")
        if len(cols) == 1 and cols[0].voff == 0:
            return cols[0]
        n = sum(c.length for c in cols)
        dev = cols[0].device
        valid = None
        if any(c.valid is not None for c in cols):
            bits = torch.cat([c.valid_bools() if c.valid is not None
                              else torch.ones(c.length, dtype=torch.bool, device=dev) for c in cols])
            pad = torch.zeros(_bitmap_bytes(n) * 8, dtype=torch.uint8, device=dev)
            pad[:n] = bits.to(torch.uint8)
            w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=dev)
            valid = (pad.view(-1, 8) * w).sum(1, dtype=torch.int32).to(torch.uint8)
            if valid.numel() < 8:
                valid = torch.cat([valid, torch.zeros(8 - valid.numel(), dtype=torch.uint8, device=dev)])
        if _is_var(t):
            bounds = torch.stack([torch.stack([c.offsets[0], c.offsets[c.length]]) for c in cols]).to(torch.int64)
            b = bounds.tolist()  # the one host read
            offs, vals, base = [], [], 0
            for c, (a, e) in zip(cols, b):
                offs.append(c.offsets[: c.length].to(torch.int64) - a + base)
                vals.append(c.values[a:e])
                base += e - a
            odt = cols[0].offsets.dtype
            offs.append(torch.tensor([base], dtype=torch.int64, device=dev))
            values = torch.cat(vals) if base else torch.zeros(1, dtype=torch.uint8, device=dev)
            return cls(t, n, offsets=torch.cat(offs).to(odt), values=values, valid=valid, voff=0)
        w = _fixed_width(t)
        data = torch.cat([c.data[: c.length * w] for c in cols])
        if data.numel() == 0:
            data = torch.zeros(w, dtype=torch.uint8, device=dev)
        return cls(t, n, data=data, valid=valid, voff=0)

    def to_arrow(self) -> pa.Array:
        n, t = self.length, self.type
        vbuf = None
        if self.valid is not None:
            vb = self.valid.cpu().numpy()
            if self.voff:  # re-base the bitmap at bit 0
                bits = np.unpackbits(vb, bitorder="little")[self.voff:self.voff + n]
                vb = np.packbits(bits, bitorder="little")
            vbuf = pa.py_buffer(vb.tobytes())
        if _is_var(t):
            offs = self.offsets.cpu().numpy()
            vals = self.values.cpu().numpy()[: int(offs[-1]) if n else 0]
            return pa.Array.from_buffers(t, n, [vbuf, pa.py_buffer(offs.tobytes()), pa.py_buffer(vals.tobytes())])
        raw = self.data.cpu().numpy()
        if pa.types.is_boolean(t):
            bits = np.packbits(raw[:n].astype(bool), bitorder="little")
            return pa.Array.from_buffers(t, n, [vbuf, pa.py_buffer(bits.tobytes())])
        w = _fixed_width(t)
        return pa.Array.from_buffers(t, n, [vbuf, pa.py_buffer(raw[: n * w].tobytes())])


def _key_column(c: DeviceColumn) -> "_lib.HjKeyColumn":
    """hj_key_column of a device column (fixed width or Utf8 / Binary)."""
    vptr = c.valid.data_ptr() if c.valid is not None else None
    if _is_var(c.type):
        return _lib.HjKeyColumn(c.values.data_ptr(), c.offsets.data_ptr(), vptr, c.voff, 0, _VAR[c.type])
    return _lib.HjKeyColumn(c.data.data_ptr(), None, vptr, c.voff, _fixed_width(c.type), 0)


def _key_columns(cols: list[DeviceColumn]):
    arr = (_lib.HjKeyColumn * len(cols))()
    for i, c in enumerate(cols):
        arr[i] = _key_column(c)
    return arr


def composite_keys(cols: list[DeviceColumn]) -> tuple[torch.Tensor, torch.Tensor]:
    """hj_composite_keys: one int64 key per row from every key column (calculate_hash over
    all key columns, src/shared/shared.rs:11-16) and the LSB validity bitmap (uint8
    device tensor, bit i = no key column null at row i)."""
    L = _lib.load()
    n = cols[0].length
    if any(c.length != n for c in cols):
        raise ValueError("key columns of unequal length")
    dev = cols[0].device
    keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    valid = torch.zeros(max(_bitmap_bytes(n), 8), dtype=torch.uint8, device=dev)
    check(L.hj_composite_keys(len(cols), _key_columns(cols), n, keys.data_ptr(), valid.data_ptr(), _stream(dev)))
    return keys[:n], valid


def filter_equal_pairs(build_cols: list[DeviceColumn], probe_cols: list[DeviceColumn], b: torch.Tensor,
                       p: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """hj_filter_equal_pairs (equal_rows_arr, src/shared/datafusion_private.rs:52-73): the
    candidate pairs whose key tuples are equal in every column, order kept."""
    L = _lib.load()
    n = b.numel()
    dev = b.device
    ob = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    op = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(L.hj_equal_pairs_workspace_bytes(n), dtype=torch.uint8, device=dev)
    b, p = b.contiguous(), p.contiguous()
    check(L.hj_filter_equal_pairs(len(build_cols), _key_columns(build_cols), _key_columns(probe_cols),
                                  b.data_ptr() if n else None, p.data_ptr() if n else None, n, ob.data_ptr(),
                                  op.data_ptr(), cnt.data_ptr(), ws.data_ptr(), _stream(dev)))
    m = int(cnt.item())
    return ob[:m], op[:m]


def mark_rows(idx: torch.Tensor, nflags: int, flags: torch.Tensor | None = None) -> torch.Tensor:
    """flags[idx[i]] = 1 (uint8 device tensor of nflags; -1 / out-of-range ignored)."""
    L = _lib.load()
    dev = idx.device
    if flags is None:
        flags = torch.zeros(max(nflags, 1), dtype=torch.uint8, device=dev)
    idx = idx.contiguous()
    ib = 8 if idx.dtype == torch.int64 else 4
    if idx.numel():
        check(L.hj_mark_rows(idx.data_ptr(), ib, idx.numel(), flags.data_ptr(), nflags, _stream(dev)))
    return flags


def select_rows(flags: torch.Tensor, want: int, n: int | None = None) -> torch.Tensor:
    """Ascending positions i < n with flags[i] == want (int64 device tensor)."""
    L = _lib.load()
    dev = flags.device
    n = flags.numel() if n is None else n
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(L.hj_select_workspace_bytes(n), dtype=torch.uint8, device=dev)
    check(L.hj_select_rows(flags.data_ptr() if n else None, n, want, out.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
                           _stream(dev)))
    return out[: int(cnt.item())]


class DeviceRecordBatch:
    """The concatenated build RecordBatch, resident in HBM (row i <-> build index i): what
    the reference hands every partition's consumer with the lookup
    (src/operator/lookup_consumers.rs:4-9). `num_rows`, `schema` and the device columns
    need no host copy; `column(i)` / `to_batch()` bring columns to the host on demand."""

    def __init__(self, schema: pa.Schema, columns: list[DeviceColumn], num_rows: int):
        self.schema = schema
        self.device_columns = columns
        self.num_rows = num_rows
        self._host: pa.RecordBatch | None = None

    @property
    def num_columns(self) -> int:
        return len(self.device_columns)

    def to_batch(self) -> pa.RecordBatch:
        if self._host is None:
            if not self.device_columns:
                self._host = pa.RecordBatch.from_pylist([], schema=self.schema)
            else:
                self._host = pa.RecordBatch.from_arrays([c.to_arrow() for c in self.device_columns],
                                                        schema=self.schema)
        return self._host

    def column(self, i: int | str) -> pa.Array:
        if isinstance(i, str):
            i = self.schema.get_field_index(i)
        return self.device_columns[i].to_arrow()

    @property
    def columns(self) -> list[pa.Array]:
        return self.to_batch().columns
