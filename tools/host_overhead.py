"""Diagnostic: host-side time of each call of one bench step (C2), averaged over steps:
table creation, append, finish (build enqueue incl. the key-range read-back), stream wait,
probe enqueue, synchronize, close."""
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
s = torch.cuda.current_stream(dev)
names = ["create", "append", "finish", "stream_wait", "probe_enqueue", "synchronize", "close"]
acc = {n: 0.0 for n in names}
steps = 20
for i in range(steps + 3):
    t = [time.perf_counter()]
    tb = HashTable(1, "int64", 0)
    t.append(time.perf_counter())
    tb.append(0, bk)
    t.append(time.perf_counter())
    tb.finish(0)
    t.append(time.perf_counter())
    tb.stream_wait(s.cuda_stream)
    t.append(time.perf_counter())
    tb.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), P, dt.data_ptr(), ws.data_ptr(), s.cuda_stream)
    t.append(time.perf_counter())
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    tb.close()
    t.append(time.perf_counter())
    if i >= 3:
        for k, n in enumerate(names):
            acc[n] += t[k + 1] - t[k]
tot = sum(acc.values())
for n in names:
    print(f"{n:14s} {acc[n] / steps * 1e6:8.1f} us")
print(f"{'step':14s} {tot / steps * 1e6:8.1f} us")
