"""Diagnostic: probe-kernel time vs build size (table L2 / Infinity-Cache / HBM resident)
and hit rate, P = 10^8 probe rows, HIP events, min of 5."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

L = dfp.load()
dev = torch.device("cuda", 0)
P = 10**8
ob = torch.empty(P, dtype=torch.int64, device=dev)
op = torch.empty(P, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
pk = torch.empty(P, dtype=torch.int64, device=dev)

for B in [10**5, 10**6, 3 * 10**6, 10**7, 3 * 10**7]:
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
    t = HashTable(1, "int64", 0)
    t.build(bk)
    st = t.stats()
    for name, lo, rng in [("hit0", B, 2 * B), ("hit50", 0, 2 * B), ("hit100", 0, B)]:
        assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, rng, None) == 0
        pk += lo
        ts = []
        for _ in range(5):
            ev0.record()
            t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), P, dt.data_ptr(), ws.data_ptr(), 0)
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1))
        ms = min(ts)
        print(f"B={B:>9} table={st['table_bytes'] / 1e6:7.1f}MB {name:6s}: probe {ms:.3f} ms "
              f"({P / ms / 1e6:.1f} Grows/s) matches={int(dt.item())}", flush=True)
    t.close()
