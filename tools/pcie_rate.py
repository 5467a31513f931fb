#!/usr/bin/env python3
"""PCIe-inclusive rate: the C2 join with host-resident input and output,
as a host caller of the C ABI sees it (hj_build_append from host memory, hj_probe with
HJ_OUTPUT_HOST). Never the bench `value`, which starts with inputs resident in HBM."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from datafusion_parallelism_amd.table import HashTable  # noqa: E402

B, P = 10**7, 10**8
bk = (np.arange(B, dtype=np.int64) * 7368787) % B
rng = np.random.default_rng(1)
pk = rng.integers(0, 2 * B, P, dtype=np.int64)
torch.cuda.init()
res = []
for it in range(4):
    t0 = time.perf_counter()
    with HashTable(1, "int64", 0) as t:
        t.append(0, bk)
        t.finish(0)
        t1 = time.perf_counter()
        b, p = t.probe(pk)
    t2 = time.perf_counter()
    res.append((t1 - t0, t2 - t1, len(b)))
build_s, probe_s, m = min(res, key=lambda r: r[0] + r[1])
print(json.dumps({
    "what": "C2 with host input/output (PCIe included): build from host keys, probe host keys -> host pairs",
    "build_ms": round(build_s * 1e3, 2), "probe_ms": round(probe_s * 1e3, 2), "matches": m,
    "mrows_s": round(P / (build_s + probe_s) / 1e6, 1),
    "bytes_over_pcie": 8 * B + 8 * P + 12 * m,
}))
