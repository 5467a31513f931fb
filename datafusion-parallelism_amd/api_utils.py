"""Synthetic key generators: src/api_utils.rs of the reference, plus the seeded
generators of SURVEY.md §8(d) used by the benchmark configs."""
from __future__ import annotations

import numpy as np


def make_int_array_with_shift(lo: int, hi: int, shift: int) -> np.ndarray:
    """src/api_utils.rs:6-9 (Int32 ids lo+shift .. hi+shift)."""
    return np.arange(lo + shift, hi + shift, dtype=np.int32)


def make_int_array_from_range(lo: int, hi: int) -> np.ndarray:
    """src/api_utils.rs:11-13."""
    return make_int_array_with_shift(lo, hi, 0)


def make_exponential_int_array(lo: int, hi: int) -> np.ndarray:
    """src/api_utils.rs:15-23, f32 math: x = n/diff, y = (16^x - 1)/15,
    value = lo + trunc(y * diff), with libm powf as Rust's f32::powf (hj_gen_exponential_keys;
    numpy's float32 power is a different approximation and moves ~6 % of the C3 keys)."""
    from ._lib import check, load

    out = np.empty(max(hi - lo, 0), dtype=np.int32)
    check(load().hj_gen_exponential_keys(out.ctypes.data, lo, hi))
    return out


def splitmix64(x) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_keys(n: int, seed: int, rng: int) -> np.ndarray:
    """k_p[j] = splitmix64(seed + j) mod R (host twin of hj_gen_uniform_keys)."""
    with np.errstate(over="ignore"):
        return (splitmix64(np.uint64(seed) + np.arange(n, dtype=np.uint64)) % np.uint64(rng)).astype(np.int64)


def perm_keys(n: int, mul: int = 7368787, rng: int | None = None) -> np.ndarray:
    """k_b[i] = (i * mul) mod R (host twin of hj_gen_perm_keys)."""
    rng = n if rng is None else rng
    with np.errstate(over="ignore"):
        return ((np.arange(n, dtype=np.uint64) * np.uint64(mul)) % np.uint64(rng)).astype(np.int64)
