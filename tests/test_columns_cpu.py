"""CPU: DeviceColumn.concat (the build side's concatenation on the device, operator.py's
_SharedBuild) checked against pyarrow.concat_arrays. The torch ops run on any device, so
the concatenation logic (offset re-basing, bitmap re-packing from bit 0) is checked here
on CPU tensors; the GPU operator tests run the same code on HBM."""
import numpy as np
import pyarrow as pa
import pytest
import torch

from datafusion_parallelism_amd.columns import DeviceColumn, DeviceRecordBatch


def _pieces(kind, rng):
    if kind == "int64":
        a = pa.array(rng.integers(-1000, 1000, 103), mask=rng.random(103) < 0.2)
    elif kind == "int32_nonull":
        a = pa.array(rng.integers(0, 9, 77).astype(np.int32))
    elif kind == "utf8":
        a = pa.array([None if x < 0.1 else "s" * int(x * 7) for x in rng.random(91)], type=pa.string())
    elif kind == "large_binary":
        a = pa.array([bytes([int(x * 250)]) * int(x * 5) for x in rng.random(64)], type=pa.large_binary())
    elif kind == "bool":
        a = pa.array([bool(x > 0.5) if x > 0.15 else None for x in rng.random(70)])
    else:
        raise ValueError(kind)
    # odd offsets and lengths: bitmaps that start mid-byte, offsets that start past 0
    return [a.slice(0, 13), a.slice(13, 1), a.slice(14, 0), a.slice(21, len(a) - 30), a.slice(len(a) - 9)]


@pytest.mark.parametrize("kind", ["int64", "int32_nonull", "utf8", "large_binary", "bool"])
def test_concat_matches_arrow(kind):
    rng = np.random.default_rng(len(kind))
    parts = _pieces(kind, rng)
    cols = [DeviceColumn.from_arrow(p, "cpu") for p in parts]
    got = DeviceColumn.concat(cols)
    want = pa.concat_arrays(parts)
    assert got.length == len(want)
    assert got.voff == 0
    assert got.to_arrow().equals(want)


def test_single_piece_at_offset_is_rebased():
    a = pa.array([1, None, 3, 4, None, 6, 7, 8, 9], type=pa.int64()).slice(3)
    got = DeviceColumn.concat([DeviceColumn.from_arrow(a, "cpu")])
    assert got.voff == 0 and got.to_arrow().equals(a)


def test_key_tensor_and_valid_bools():
    a = pa.array([5, None, 7, None, 9], type=pa.int32()).slice(1)
    c = DeviceColumn.from_arrow(a, "cpu")
    assert c.key_tensor().tolist()[1] == 7 and c.key_tensor().dtype == torch.int32
    assert c.valid_bools().tolist() == [False, True, False, True]


def test_device_record_batch_host_view():
    rb = pa.RecordBatch.from_pydict({"k": pa.array([1, 2, None]), "v": pa.array(["a", None, "ccc"])})
    d = DeviceRecordBatch(rb.schema, [DeviceColumn.from_arrow(c, "cpu") for c in rb.columns], rb.num_rows)
    assert d.num_rows == 3 and d.num_columns == 2
    assert d.column("v").equals(rb.column(1))
    assert d.to_batch().equals(rb)
