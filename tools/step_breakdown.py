"""Diagnostic: host-side breakdown of one bench step (build + probe) on C2."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

L = dfp.load()
dev = torch.device("cuda", 0)
B, P = 10**7, 10**8
bk = torch.empty(B, dtype=torch.int64, device=dev)
pk = torch.empty(P, dtype=torch.int64, device=dev)
assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, None) == 0
ob = torch.empty(P, dtype=torch.int64, device=dev)
op = torch.empty(P, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
for it in range(6):
    t0 = time.perf_counter()
    t = HashTable(1, "int64", 0)
    t1 = time.perf_counter()
    t.append(0, bk)
    t2 = time.perf_counter()
    t.finish(0)
    t3 = time.perf_counter()
    t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), P, dt.data_ptr(), ws.data_ptr(), 0)
    t4 = time.perf_counter()
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    m = int(dt.item())
    t.close()
    t6 = time.perf_counter()
    print(f"it {it}: create {1e3*(t1-t0):.3f} append {1e3*(t2-t1):.3f} finish {1e3*(t3-t2):.3f} "
          f"(device build {t.build_ns() if False else 0}) probe-launch {1e3*(t4-t3):.3f} probe-wait {1e3*(t5-t4):.3f} "
          f"close {1e3*(t6-t5):.3f} total {1e3*(t6-t0):.3f} ms matches {m}", flush=True)
