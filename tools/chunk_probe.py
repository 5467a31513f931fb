"""Diagnostic: does a probe run in K chunks of P/K rows beat one probe of P rows?

With chunks of ~2.5e7 rows the sliced probe's intermediates (entries + refs, ~4-6 B per
in-range row) could stay in the Infinity Cache between its three kernels. Times K
sequential probe_async calls over consecutive key ranges (each into its own output
region) on the null stream with HIP events. C2 shape (B = 1e7, P = 1e8)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

B, P = 10**7, 10**8
MIX = "--mix" in sys.argv
L = dfp.load()
dev = torch.device("cuda", 0)
bk = torch.empty(B, dtype=torch.int64, device=dev)
pk = torch.empty(P, dtype=torch.int64, device=dev)
assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, None) == 0
if MIX:
    bk.mul_(0x9E3779B97F4A7C15 - (1 << 64))
    pk.mul_(0x9E3779B97F4A7C15 - (1 << 64))
ob = torch.empty(P, dtype=torch.int64, device=dev)
op = torch.empty(P, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(64, dtype=torch.int64, device=dev)
t = HashTable(1, "int64", 0)
t.build(bk)
torch.cuda.synchronize()
for K in (1, 2, 3, 4, 6, 8, 16):
    n = P // K
    best = 1e9
    for it in range(6):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for c in range(K):
            lo = c * n
            m = n if c < K - 1 else P - lo
            t.probe_async(pk.data_ptr() + 8 * lo, m, ob.data_ptr() + 8 * lo, op.data_ptr() + 4 * lo, m,
                          dt.data_ptr() + 8 * c, ws.data_ptr(), 0)
        b.record()
        b.synchronize()
        if it:
            best = min(best, a.elapsed_time(b))
    total = int(dt[:K].sum().item())
    print(f"K={K:2d} chunk={n:>10d} probe {best * 1e3:8.1f} us  matches={total}", flush=True)
t.close()
