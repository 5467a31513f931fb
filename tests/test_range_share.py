"""CPU: the sharded plan's key-range shares in C (hj_dist.cpp's range_share, through the
test library's host-only hook) equal the Python plan's ExchangePlan.local_key_range and the
partition kernel's range map restated in PartSpec.part_of: each rank's share is exactly the
keys the map sends it, the shares tile [min, max] in rank order, also for ranges near 2^64
(ADVICE r04). No GPU is used."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tl():
    sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
    import build as hipbuild

    sys.path.pop(0)
    hipbuild.build_commtest()
    from datafusion_parallelism_amd import _lib

    return _lib.load_commtest()


def c_share(tl, lo, hi, w, r):
    a, b = ctypes.c_int64(), ctypes.c_int64()
    ok = tl.hj_test_range_share(lo, hi, w, r, ctypes.byref(a), ctypes.byref(b))
    return (a.value, b.value) if ok else None


I64_MIN, I64_MAX = -(2**63), 2**63 - 1
RANGES = [(0, 9_999_999), (-5, 5), (0, 0), (7, 8), (0, 6), (100, 100 + 2**31), (-(2**40), 2**40 + 12345),
          (I64_MIN, I64_MAX), (I64_MIN, I64_MIN + 7), (I64_MAX - 1000, I64_MAX), (I64_MIN, 0), (-1, I64_MAX),
          (I64_MIN + 1, I64_MAX - 1)]


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("rng", RANGES)
def test_range_share_matches_python_plan(tl, world, rng):
    from datafusion_parallelism_amd.distributed import ExchangePlan, PartSpec

    lo, hi = rng
    plan = ExchangePlan(spec=PartSpec(True, lo, hi), build_lo=lo, build_hi=hi)
    shares = [c_share(tl, lo, hi, world, r) for r in range(world)]
    assert shares == [plan.local_key_range(r, world) for r in range(world)]
    # the shares tile [lo, hi] in rank order
    got = [s for s in shares if s is not None]
    assert got[0][0] == lo and got[-1][1] == hi
    for (a0, a1), (b0, b1) in zip(got, got[1:]):
        assert b0 == a1 + 1 and a0 <= a1
    # every share is what the partition kernel's map sends the rank (its ends and neighbours)
    spec = PartSpec(True, lo, hi)
    for r, s in enumerate(shares):
        if s is None:
            continue
        probe = [k for k in (s[0], s[1], s[0] + (s[1] - s[0]) // 2) if lo <= k <= hi]
        dest, keep = spec.part_of(np.array(probe, dtype=object).astype(np.int64) if all(
            I64_MIN <= k <= I64_MAX for k in probe) else probe, world)
        assert all(keep) and all(int(d) == r for d in dest)
        for k, want in ((s[0] - 1, r - 1), (s[1] + 1, r + 1)):
            if lo <= k <= hi:
                d, _ = spec.part_of(np.array([k], dtype=np.int64), world)
                assert int(d[0]) == want


@pytest.mark.parametrize("world", [2, 4, 8])
def test_range_share_random(tl, world):
    from datafusion_parallelism_amd.distributed import ExchangePlan, PartSpec

    rng = np.random.default_rng(world)
    for _ in range(200):
        a, b = sorted(int(x) for x in rng.integers(I64_MIN, I64_MAX, 2, dtype=np.int64))
        if rng.random() < 0.5:
            b = a + int(rng.integers(0, 50))
        plan = ExchangePlan(spec=PartSpec(True, a, b), build_lo=a, build_hi=b)
        assert [c_share(tl, a, b, world, r) for r in range(world)] == [plan.local_key_range(r, world)
                                                                        for r in range(world)]
