"""ctypes binding of the C ABI in ``include/hj.h`` (``lib/libdfp_hj.so``).

torch is imported before the library is loaded: the library links the HIP runtime that
torch ships (SONAME ``libamdhip64.so.7``), and loading torch first makes the dynamic
linker reuse torch's copy, so the process holds a single HIP runtime.

The library has no CPU fallback: every compute entry point fails with
``HJ_ERR_NO_DEVICE`` on a machine without a GPU, and this module raises
``ImportError`` if the library has not been built.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# DFP_HJ_LIB: a diagnostic build of the same library (tools/lib_variants.py) in its place
LIB_PATH = os.environ.get("DFP_HJ_LIB") or os.path.join(HERE, "lib", "libdfp_hj.so")

HJ_OK, HJ_ERR_INVALID, HJ_ERR_OOM, HJ_ERR_HIP, HJ_ERR_RCCL, HJ_ERR_CAPACITY, HJ_ERR_NO_DEVICE = range(7)
HJ_INT32, HJ_INT64 = 0, 1
HJ_INPUT_DEVICE, HJ_BORROW, HJ_OUTPUT_HOST, HJ_IDS_U31, HJ_BORROW_KEEP = 1, 2, 4, 8, 16
HJ_MULTI_AUTO, HJ_MULTI_BROADCAST, HJ_MULTI_RADIX = 0, 1, 2

STATUS_NAMES = {
    HJ_OK: "HJ_OK", HJ_ERR_INVALID: "HJ_ERR_INVALID", HJ_ERR_OOM: "HJ_ERR_OOM", HJ_ERR_HIP: "HJ_ERR_HIP",
    HJ_ERR_RCCL: "HJ_ERR_RCCL", HJ_ERR_CAPACITY: "HJ_ERR_CAPACITY", HJ_ERR_NO_DEVICE: "HJ_ERR_NO_DEVICE",
}


class HjError(RuntimeError):
    """A non-OK hj_status (the reference's DataFusionError::Internal for HJ_ERR_INVALID)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


class HjPairs(ctypes.Structure):
    _fields_ = [("build_idx", ctypes.POINTER(ctypes.c_uint64)), ("probe_idx", ctypes.POINTER(ctypes.c_uint32)),
                ("count", ctypes.c_int64), ("device_resident", ctypes.c_int)]


class HjTableStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "build_rows", "inserted_rows", "distinct_keys", "dup_keys", "dup_rows", "max_key_rows", "buckets",
        "table_bytes", "build_ns")]


class HjKeyColumn(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("validity", ctypes.c_void_p),
                ("validity_offset", ctypes.c_int64), ("width", ctypes.c_int), ("offset_bytes", ctypes.c_int)]


class HjPartSpec(ctypes.Structure):
    _fields_ = [("by_range", ctypes.c_int), ("key_lo", ctypes.c_int64), ("key_hi", ctypes.c_int64)]


class HjDistInfo(ctypes.Structure):
    _fields_ = [("build_rows", ctypes.c_int64), ("recv_rows", ctypes.c_int64), ("sharded", ctypes.c_int)]


HJ_COMM_ID_BYTES = 128


# (name, restype, argtypes) of every entry point declared in include/hj.h
P, I64, I32, U32, U64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
PP = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = [
    ("hj_last_error", ctypes.c_char_p, []),
    ("hj_version", ctypes.c_char_p, []),
    ("hj_device_count", I32, []),
    ("hj_build_begin", I32, [I32, I32, I32, I64, PP]),
    ("hj_build_begin_multi", I32, [I32, ctypes.POINTER(ctypes.c_int), I32, I32, I64, I32, PP]),
    ("hj_build_append", I32, [P, I32, P, P, I64, P, I64, U32, P]),
    ("hj_build_finish", I32, [P, I32]),
    ("hj_build_key_range", I32, [P, I64, I64]),
    ("hj_build_key_base", I32, [P, I64]),
    ("hj_build_dense", I32, [P]),
    ("hj_table_dense_piece", I32, [P, PP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64), PP, PP,
                                   ctypes.POINTER(ctypes.c_int)]),
    ("hj_table_dense_export", I32, [P, P, U64, U64, P, U64, P, P]),
    ("hj_table_wrap_dense", I32, [I32, I32, I64, U64, P, P, I32, P, PP]),
    ("hj_dense_rebase_dups", I32, [P, U64, U32, I32, P]),
    ("hj_build_partition_offset", I32, [P, I32, ctypes.POINTER(ctypes.c_int64)]),
    ("hj_table_stats_get", I32, [P, ctypes.POINTER(HjTableStats)]),
    ("hj_table_build_ns", I64, [P]),
    ("hj_table_lookup", I32, [P, I64, P, I64, ctypes.POINTER(ctypes.c_int64)]),
    ("hj_table_chain_links", I32, [P, P, I64]),
    ("hj_table_free", None, [P]),
    ("hj_probe", I32, [P, P, P, I64, I64, U32, P, ctypes.POINTER(HjPairs)]),
    ("hj_pairs_free", None, [ctypes.POINTER(HjPairs)]),
    ("hj_probe_workspace_bytes", I64, [I64]),
    ("hj_set_probe_mode", I32, [I32]),
    ("hj_set_probe_tile_log", I32, [I32]),
    ("hj_set_build_mode", I32, [I32]),
    ("hj_set_device_budget", I64, [I64]),
    ("hj_table_device_bytes", I32, [P, ctypes.POINTER(ctypes.c_int64)]),
    ("hj_probe_async", I32, [P, P, P, I64, I64, P, P, I64, P, P, P]),
    ("hj_probe_async_ids", I32, [P, P, P, I64, P, I64, P, P, I64, P, P, P]),
    ("hj_probe_async_base", I32, [P, P, P, I64, I64, U32, P, P, I64, P, P, P]),
    ("hj_table_stream_wait", I32, [P, P]),
    ("hj_partition_workspace_bytes", I64, [I64, I32]),
    ("hj_radix_partition", I32, [I32, P, P, I64, P, U64, I64, I32, P, I32, I64, P, I32, P, P, P]),
    ("hj_partition_rows", I32, [I32, P, P, I64, P, U64, I64, I32, P, P, I32, I64, P, I32, P, P, P]),
    ("hj_key_minmax_workspace_bytes", I64, []),
    ("hj_key_minmax", I32, [I32, P, P, I64, I64, P, P, P]),
    ("hj_partition_regions_workspace_bytes", I64, [I64, I32]),
    ("hj_partition_regions", I32, [I32, P, P, I64, P, U64, I64, I32, P, P, I32, I64, P, I32, I64, P, P, P]),
    ("hj_mark_rows", I32, [P, I32, I64, P, I64, P]),
    ("hj_select_workspace_bytes", I64, [I64]),
    ("hj_select_rows", I32, [P, I64, I32, P, P, P, P]),
    ("hj_gather_fixed", I32, [P, P, I64, I32, P, I32, I64, P, P, P]),
    ("hj_gather_var_workspace_bytes", I64, [I64]),
    ("hj_gather_var", I32, [P, I32, P, P, I64, P, I32, I64, P, P, I64, P, P, P, P]),
    ("hj_composite_keys", I32, [I32, ctypes.POINTER(HjKeyColumn), I64, P, P, P]),
    ("hj_equal_pairs_workspace_bytes", I64, [I64]),
    ("hj_filter_equal_pairs", I32, [I32, ctypes.POINTER(HjKeyColumn), ctypes.POINTER(HjKeyColumn), P, P, I64, P, P,
                                    P, P, P]),
    ("hj_comm_unique_id", I32, [P]),
    ("hj_comm_create", I32, [I32, I32, P, I32, PP]),
    ("hj_comm_free", None, [P]),
    ("hj_dist_build_sharded", I32, [P, I32, P, P, I64, I64, I64, I32, P, PP, ctypes.POINTER(HjDistInfo)]),
    ("hj_dist_build_sharded_async", I32, [P, I32, P, P, I64, I64, I64, I32, P, PP]),
    ("hj_dist_join_radix", I32, [P, I32, P, P, I64, I64, I64, I32, P, P, I64, I64, I64, P, PP]),
    ("hj_dist_job_wait", I32, [P, ctypes.POINTER(HjDistInfo)]),
    ("hj_dist_job_table", I32, [P, PP, ctypes.POINTER(HjDistInfo)]),
    ("hj_dist_job_pairs", I32, [P, PP, PP, ctypes.POINTER(ctypes.c_int64)]),
    ("hj_dist_job_times", I32, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double)]),
    ("hj_dist_job_free", None, [P]),
    ("hj_dist_shuffle", I32, [P, I32, P, I64, I32, P, P, P, PP]),
    ("hj_dist_gather", I32, [P, I64, I32, P, P, P, PP]),
    ("hj_dist_job_columns", I32, [P, P, PP, P, I32, ctypes.POINTER(ctypes.c_int64)]),
    ("hj_gen_perm_keys", I32, [P, I64, I64, I64, P]),
    ("hj_gen_uniform_keys", I32, [P, I64, U64, I64, P]),
    ("hj_gen_exponential_keys", I32, [P, I32, I32]),
]

# the test library's extra entry points (lib/libdfp_hj_commtest.so: the thread transport)
COMMTEST_PATH = os.path.join(HERE, "lib", "libdfp_hj_commtest.so")
COMMTEST_SIGNATURES = [
    ("hj_test_hub_create", P, [I32, ctypes.c_double]),
    ("hj_test_hub_free", None, [P]),
    ("hj_test_comm_create", I32, [P, I32, I32, PP]),
    ("hj_test_comm_fail_at", None, [P, I32, I32]),
    ("hj_test_range_share", I32, [I64, I64, I32, I32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
]

_lib = None


def _bind(L: ctypes.CDLL, sigs) -> None:
    for name, res, args in sigs:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def load() -> ctypes.CDLL:
    """Load the built library (raises ImportError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python __graft_entry__.py build` "
                          "(or datafusion-parallelism_amd/build.py). There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    _bind(L, SIGNATURES)
    _lib = L
    return L


def load_commtest() -> ctypes.CDLL:
    """The test library (the product's entry points + the in-process thread transport).
    Tests only: a handle made by one library must not be passed to the other."""
    if not os.path.exists(COMMTEST_PATH):
        raise ImportError(f"{COMMTEST_PATH} is missing: run `python __graft_entry__.py build`")
    L = ctypes.CDLL(COMMTEST_PATH)
    _bind(L, SIGNATURES + COMMTEST_SIGNATURES)
    return L


def check(status: int, L: ctypes.CDLL | None = None) -> None:
    """Raise HjError for a non-OK status; the message from library `L` (the one that
    failed: its hj_last_error is thread-local to it), default the product library."""
    if status != HJ_OK:
        msg = (L or load()).hj_last_error()
        raise HjError(status, msg.decode() if msg else "")


def device_count() -> int:
    return load().hj_device_count()
