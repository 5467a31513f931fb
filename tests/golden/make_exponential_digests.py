"""Digests of the C3 key generator (src/api_utils.rs:15-23, `make_exponential_int_array`)
at several sizes, committed as tests/golden/exponential_digests.json.

The reference computes x = n / diff, y = (16f32.powf(x) - 1) / 15 and lo + trunc(y * diff)
in f32. Rust's `f32::powf` lowers to the `llvm.pow.f32` intrinsic, which is the platform
libm's `powf` (glibc on the reference's Linux runs). Two restatements are recorded:
  * "libm"  - the C oracle (oracle/hj_oracle.c, glibc powf): the generator this repository
              uses for C3 (6,603,254 distinct keys at 10^7);
  * "numpy" - numpy's float32 `power` (its own SIMD approximation), the restatement
              SURVEY.md §8(d) used (6,602,610 distinct keys at 10^7).
Run from the repo root: python tests/golden/make_exponential_digests.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SIZES = [(0, 10), (-50, 4000), (0, 10**5), (1000, (1 << 20) + 1000), (0, 10**6), (0, 10**7)]


def numpy_f32(lo: int, hi: int) -> np.ndarray:
    diff = hi - lo
    n = np.arange(0, diff, dtype=np.float32)
    x = n / np.float32(diff)
    y = (np.power(np.float32(16.0), x).astype(np.float32) - np.float32(1.0)) / np.float32(15.0)
    return (lo + np.trunc((y.astype(np.float32) * np.float32(diff)).astype(np.float32))).astype(np.int32)


def digest(a: np.ndarray) -> dict:
    a = np.ascontiguousarray(a.astype("<i4"))
    return {"sha256": hashlib.sha256(a.tobytes()).hexdigest(), "distinct": int(np.unique(a).size)}


def main():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    out = []
    for lo, hi in SIZES:
        out.append({"lo": lo, "hi": hi, "libm": digest(oracle.make_exponential_int_array(lo, hi)),
                    "numpy": digest(numpy_f32(lo, hi))})
    with open(os.path.join(ROOT, "tests", "golden", "exponential_digests.json"), "w") as f:
        json.dump({"source": "src/api_utils.rs:15-23", "generator": __doc__.split("\n")[0], "sizes": out}, f, indent=1)
    for r in out:
        print(r)


if __name__ == "__main__":
    main()
