"""CPU: the C-ABI library loads, exports every symbol include/hj.h declares, the ctypes
binding covers them, and without a GPU every compute entry point fails loudly with
HJ_ERR_NO_DEVICE (there is no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hj.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hj_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["hj_build_begin", "hj_build_append", "hj_build_finish", "hj_probe", "hj_probe_async",
                 "hj_table_lookup", "hj_radix_partition", "hj_pairs_free", "hj_table_free"]:
        assert must in names


def test_library_exports_every_declared_symbol(dfp):
    from datafusion_parallelism_amd import _lib

    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (hj_[a-z0-9_]+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(declared_functions()) <= bound, set(declared_functions()) - bound
    for n in declared_functions():
        assert getattr(lib, n) is not None


def test_library_is_gfx950(dfp):
    from datafusion_parallelism_amd import _lib

    lib = _lib.load()
    assert b"gfx950" in lib.hj_version()
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob and b"gfx942" not in blob


def test_single_hip_runtime_link(dfp):
    """The library links the HIP runtime torch ships (one runtime per process)."""
    from datafusion_parallelism_amd import _lib

    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "libamdhip64" in out and "torch/lib" in out


def test_no_device_fails_loudly(dfp):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from datafusion_parallelism_amd import HjError, _lib

    assert dfp.device_count() == 0
    with pytest.raises(HjError) as e:
        dfp.HashTable(1, "int64", 0)
    assert e.value.status == _lib.HJ_ERR_NO_DEVICE
    L = _lib.load()
    x = np.zeros(4, np.int64)
    assert L.hj_gen_uniform_keys(x.ctypes.data, 4, 1, 10, None) == _lib.HJ_ERR_NO_DEVICE
    assert L.hj_radix_partition(1, None, None, 0, None, 0, 0, 2, None, 8, 0, None, 8, None, None, None) == _lib.HJ_ERR_NO_DEVICE
    assert L.hj_partition_rows(1, None, None, 0, None, 0, 0, 2, None, None, 8, 0, None, 8, None, None, None) == _lib.HJ_ERR_NO_DEVICE


def test_null_args_rejected(dfp):
    from datafusion_parallelism_amd import _lib

    L = _lib.load()
    assert L.hj_build_begin(0, 1, 1, 0, None) == _lib.HJ_ERR_INVALID
    assert L.hj_build_finish(None, 0) == _lib.HJ_ERR_INVALID
    assert L.hj_probe(None, None, None, 0, 0, 0, None, None) == _lib.HJ_ERR_INVALID
    assert L.hj_table_build_ns(None) == -1
    assert L.hj_probe_workspace_bytes(0) > 0
    assert L.hj_probe_workspace_bytes(10**8) >= 8 * (10**8 // 4096)
    L.hj_table_free(None)
    p = _lib.HjPairs()
    L.hj_pairs_free(ctypes.byref(p))


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "datafusion-parallelism_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "hj_oracle" not in src and "ora_" not in src, f


def test_probe_mode_switch(dfp):
    """hj_set_probe_mode: 0 auto, 3 fused, 4 sliced; bad (incl. the retired 1 and 2) -> -1.
    No device work."""
    from datafusion_parallelism_amd import _lib

    L = _lib.load()
    for bad in (5, -1, 1, 2):
        assert L.hj_set_probe_mode(bad) == -1
    old = L.hj_set_probe_mode(3)
    assert L.hj_set_probe_mode(4) == 3
    assert L.hj_set_probe_mode(old) == 4


def test_probe_tile_log_switch(dfp):
    """hj_set_probe_tile_log: 0 auto (2^14-row tiles dense, 2^15 hashed), 14, 15; bad -> -1.
    No device work."""
    from datafusion_parallelism_amd import _lib

    L = _lib.load()
    for bad in (13, 16, -1, 1):
        assert L.hj_set_probe_tile_log(bad) == -1
    old = L.hj_set_probe_tile_log(15)
    assert L.hj_set_probe_tile_log(14) == 15
    assert L.hj_set_probe_tile_log(0) == 14
    assert L.hj_set_probe_tile_log(old) == 0


def test_join_type_names():
    """DataFusion JoinType names (probe_lookup_implementation.rs:32-43), host logic only."""
    from datafusion_parallelism_amd.operator import JoinType

    assert JoinType.parse("LEFT OUTER") is JoinType.Left
    assert JoinType.parse("full_outer") is JoinType.Full
    assert JoinType.parse("LeftSemi") is JoinType.LeftSemi
    assert JoinType.parse(JoinType.RightAnti) is JoinType.RightAnti
    assert [j for j in JoinType if j.marks_build] == [JoinType.Left, JoinType.Full, JoinType.LeftSemi,
                                                      JoinType.LeftAnti]
    with pytest.raises(Exception):
        JoinType.parse("cross")


def test_build_mode_switch(dfp):
    """hj_set_build_mode: 0 auto (dense layout when it pays), 1 hashed, 2 auto with the
    histogram partition for dense builds; bad -> -1."""
    from datafusion_parallelism_amd import _lib

    L = _lib.load()
    assert L.hj_set_build_mode(3) == -1
    old = L.hj_set_build_mode(1)
    assert L.hj_set_build_mode(old) == 1
