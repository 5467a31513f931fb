"""Oracle for the hash-join hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker or the reported CPU baseline. The product
path (``datafusion-parallelism_amd``) never imports it.

Contents:
  * ctypes wrapper of ``hj_oracle.c`` (the C restatement of the reference semantics and
    of the Version 10 table, see that file's header for the file:line citations);
  * numpy restatements of the reference's synthetic generators
    (``src/api_utils.rs:6-23``) and of SURVEY.md §8(d)'s seeded generators;
  * ``canonical_pairs`` / ``pairs_digest`` — the canonical parity contract of SURVEY.md
    §8(c): pairs sorted probe ascending, build descending, SHA-256 over
    (u64 build, u32 probe) little-endian records.

Parity pinning: the C restatement is checked against every known-answer test the
reference holds for this path (tests/golden/reference_kats.json, transcribed from the
reference's own tests; see tests/test_oracle.py). The hash boundary itself is unpinned
(no reference test pins ahash values) and does not affect emitted pairs.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libhj_oracle.so")
SRC = os.path.join(HERE, "hj_oracle.c")

_lib = None


def build(force: bool = False) -> str:
    """Compile the C restatement (gcc, -O2, pthreads)."""
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(SRC) > os.path.getmtime(LIB_PATH):
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I64 = ctypes.c_int64
        L.ora_inner_join.restype = I64
        L.ora_inner_join.argtypes = [P, P, I64, P, P, I64, ctypes.c_int, P, P, I64]
        L.ora_chain_links.restype = I64
        L.ora_chain_links.argtypes = [P, P, I64, ctypes.c_int, P]
        L.ora_v10_build.restype = P
        L.ora_v10_build.argtypes = [P, P, I64, ctypes.c_int]
        L.ora_v10_probe.restype = I64
        L.ora_v10_probe.argtypes = [P, P, P, I64, ctypes.c_int, P, P, I64]
        L.ora_v10_probe_emit.restype = I64
        L.ora_v10_probe_emit.argtypes = [P, P, P, I64, ctypes.c_int, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]
        L.ora_free.restype = None
        L.ora_free.argtypes = [P]
        L.ora_make_exponential.restype = None
        L.ora_make_exponential.argtypes = [P, ctypes.c_int32, ctypes.c_int32]
        L.ora_v10_lookup_hashes.restype = I64
        L.ora_v10_lookup_hashes.argtypes = [P, ctypes.c_uint64, I64]
        L.ora_v10_free.restype = None
        L.ora_v10_free.argtypes = [P]
        L.ora_splitmix64.restype = ctypes.c_uint64
        L.ora_splitmix64.argtypes = [ctypes.c_uint64]
        L.ora_gen_uniform.restype = None
        L.ora_gen_uniform.argtypes = [P, I64, ctypes.c_uint64, I64]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _keys64(keys) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(keys).astype(np.int64, copy=False))


def _valid_bits(valid) -> np.ndarray | None:
    """bool mask -> Arrow LSB bitmap (uint8)."""
    if valid is None:
        return None
    v = np.asarray(valid, dtype=bool)
    return np.packbits(v, bitorder="little")


def inner_join(build_keys, probe_keys, build_valid=None, probe_valid=None, hash_mode: int = 0):
    """Reference-semantics inner join (parallelism 1). Returns (build_idx u64, probe_idx
    u32) in canonical order: probe ascending, build descending."""
    L = lib()
    bk, pk = _keys64(build_keys), _keys64(probe_keys)
    bv, pv = _valid_bits(build_valid), _valid_bits(probe_valid)
    n = L.ora_inner_join(_ptr(bk), _ptr(bv), len(bk), _ptr(pk), _ptr(pv), len(pk), hash_mode, None, None, 0)
    if n < 0:
        raise MemoryError("oracle allocation failed")
    ob = np.empty(max(n, 1), dtype=np.uint64)
    op = np.empty(max(n, 1), dtype=np.uint32)
    n2 = L.ora_inner_join(_ptr(bk), _ptr(bv), len(bk), _ptr(pk), _ptr(pv), len(pk), hash_mode, _ptr(ob), _ptr(op), n)
    assert n2 == n
    return ob[:n], op[:n]


def chain_links(build_keys, build_valid=None, hash_mode: int = 0) -> np.ndarray:
    """prev[i] = next older row chained behind row i (-1 if none), parallelism 1."""
    bk = _keys64(build_keys)
    bv = _valid_bits(build_valid)
    out = np.empty(len(bk), dtype=np.int64)
    lib().ora_chain_links(_ptr(bk), _ptr(bv), len(bk), hash_mode, _ptr(out))
    return out


class V10Table:
    """Multithreaded restatement of the Version 10 table (the CPU baseline)."""

    def __init__(self, build_keys, build_valid=None, nthreads: int = 8):
        self._bk = _keys64(build_keys)
        self._bv = _valid_bits(build_valid)
        self._h = lib().ora_v10_build(_ptr(self._bk), _ptr(self._bv), len(self._bk), nthreads)
        if not self._h:
            raise MemoryError("v10 build failed")

    def probe(self, probe_keys, probe_valid=None, nthreads: int = 8, emit: bool = True):
        """One probe pass; emit=True returns the pairs (uint64 build, uint32 probe),
        emit=False the pair count only."""
        pk = _keys64(probe_keys)
        pv = _valid_bits(probe_valid)
        if not emit:
            return lib().ora_v10_probe(self._h, _ptr(pk), _ptr(pv), len(pk), nthreads, None, None, 0)
        pb, pp = ctypes.POINTER(ctypes.c_uint64)(), ctypes.POINTER(ctypes.c_uint32)()
        n = lib().ora_v10_probe_emit(self._h, _ptr(pk), _ptr(pv), len(pk), nthreads, ctypes.byref(pb),
                                     ctypes.byref(pp))
        if n < 0:
            raise MemoryError("v10 probe: allocation failed")
        try:
            ob = np.ctypeslib.as_array(pb, shape=(n,)).copy() if n else np.empty(0, np.uint64)
            op = np.ctypeslib.as_array(pp, shape=(n,)).copy() if n else np.empty(0, np.uint32)
        finally:
            lib().ora_free(ctypes.cast(pb, ctypes.c_void_p))
            lib().ora_free(ctypes.cast(pp, ctypes.c_void_p))
        return ob, op

    def lookup_hashes(self, start: int, count: int) -> int:
        """benches/lookup_speed.rs:240-246: get_iter(&i) for raw i in [start, start+count)
        used as hashes, chains walked; single thread. Returns the rows yielded."""
        return lib().ora_v10_lookup_hashes(self._h, start, count)

    def close(self):
        if self._h:
            lib().ora_v10_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------
# generators
# ---------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """SURVEY.md §8(d) splitmix64, vectorised over uint64 (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_keys(n: int, seed: int, rng: int) -> np.ndarray:
    """k_p[j] = splitmix64(seed + j) mod R."""
    j = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return (splitmix64(np.uint64(seed) + j) % np.uint64(rng)).astype(np.int64)


def perm_keys(n: int, mul: int = 7368787, rng: int | None = None) -> np.ndarray:
    """k_b[i] = (i * mul) mod R (a permutation of [0, R) when gcd(mul, R) = 1)."""
    rng = n if rng is None else rng
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return ((i * np.uint64(mul)) % np.uint64(rng)).astype(np.int64)


def make_int_array_with_shift(lo: int, hi: int, shift: int) -> np.ndarray:
    """src/api_utils.rs:6-9."""
    return np.arange(lo + shift, hi + shift, dtype=np.int32)


def make_exponential_int_array(lo: int, hi: int) -> np.ndarray:
    """src/api_utils.rs:15-23 in f32 with libm powf (ora_make_exponential: f32::powf is
    libm powf; numpy's float32 power differs from it in ~21 % of the C3 inputs)."""
    out = np.empty(max(hi - lo, 0), dtype=np.int32)
    if out.size:
        lib().ora_make_exponential(out.ctypes.data, lo, hi)
    return out


# ---------------------------------------------------------------------------
# canonical parity contract
# ---------------------------------------------------------------------------
def canonical_pairs(build_idx, probe_idx):
    """Sort pairs probe ascending, then build descending."""
    b = np.asarray(build_idx, dtype=np.uint64)
    p = np.asarray(probe_idx, dtype=np.uint64)
    order = np.lexsort((np.iinfo(np.uint64).max - b, p))
    return b[order], np.asarray(probe_idx)[order]


def pairs_digest(build_idx, probe_idx) -> str:
    """SHA-256 over (u64 build, u32 probe) little-endian records, in the given order."""
    rec = np.empty(len(build_idx), dtype=[("b", "<u8"), ("p", "<u4")])
    rec["b"] = np.asarray(build_idx, dtype=np.uint64)
    rec["p"] = np.asarray(probe_idx, dtype=np.uint32)
    return hashlib.sha256(rec.tobytes()).hexdigest()
