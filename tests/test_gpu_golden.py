"""GPU: the committed golden vectors (tests/golden/oracle_vectors.npz — oracle pairs for
seeded inputs with duplicates, nulls, int32/int64, extreme keys, empty sides; the
oracle itself is pinned to the reference's KATs by tests/test_oracle.py) reproduced
bit-exactly by the gfx950 path, from host and from device input."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
V = np.load(os.path.join(HERE, "golden", "oracle_vectors.npz"))
CASES = sorted({k.split("__")[0] for k in V.files})


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("device_input", [False, True])
def test_golden_vectors(dfp, case, device_input):
    bk, pk = V[case + "__bk"], V[case + "__pk"]
    bv, pv = V[case + "__bv"], V[case + "__pv"]
    kt = "int64" if bk.dtype == np.int64 else "int32"
    with dfp.HashTable(1, kt, 0) as t:
        t.append(0, torch.from_numpy(bk.copy()).cuda() if device_input else bk, bv)
        t.finish(0)
        b, p = t.probe(torch.from_numpy(pk.copy()).cuda() if device_input else pk, pv)
    assert np.array_equal(b, V[case + "__ob"]) and np.array_equal(p, V[case + "__op"]), case
