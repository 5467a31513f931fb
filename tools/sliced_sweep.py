"""Diagnostic: probe time of the fused (mode 3) vs the sliced (mode 4) probe on C2-shaped
joins (perm build keys, P = 10^8 uniform probe keys over 2B), HIP events, min of 5;
asserts that both modes emit the same pairs (count + order-sensitive checksum)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

L = dfp.load()
dev = torch.device("cuda", 0)
P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**8
Bs = [int(float(x)) for x in sys.argv[2:]] or [10**6, 3 * 10**6, 10**7, 3 * 10**7]
ob = torch.empty(P, dtype=torch.int64, device=dev)
op = torch.empty(P, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
pk = torch.empty(P, dtype=torch.int64, device=dev)
w = torch.arange(1, P + 1, device=dev, dtype=torch.int64) % 1000003
for B in Bs:
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, None) == 0
    t = HashTable(1, "int64", 0)
    t.build(bk)
    res = {}
    for mode, name in [(3, "fused"), (4, "sliced")]:
        L.hj_set_probe_mode(mode)
        ts = []
        for _ in range(5):
            ev0.record()
            t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), P, dt.data_ptr(), ws.data_ptr(), 0)
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1))
        m = int(dt.item())
        assert int(ws[8:16].view(torch.int64).item()) == 0, "look-back error"
        cs = (int((ob[:m] * w[:m]).sum().item()), int((op[:m].long() * w[:m]).sum().item()))
        res[name] = (m, cs)
        ms = min(ts)
        print(f"B={B:>9} {name:6s}: probe {ms:.3f} ms ({P / ms / 1e6:.1f} Grows/s) matches={m}", flush=True)
    assert res["fused"] == res["sliced"], res
    t.close()
    del bk
L.hj_set_probe_mode(0)
print("modes agree")
