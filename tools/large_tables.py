"""Diagnostic (SURVEY.md §8d sizes beyond one sliced pass): the probe's roofline fraction
for tables past the old 2047-slice limit, against C2/C2h — C2 (10^7-row dense build),
C2h (the same keys times MIX: hashed), H40 (4*10^7-key hashed build: two sliced passes)
and D120 (1.2*10^8-value direct-addressed build); 10^8 probe rows uniform over twice the
build key range each, so half of them match. HIP-event median of 5 probes of one table;
frac = (8P + 16B + 12M) / time / 8 TB/s, the bench's formula."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

MIX = 0x9E3779B97F4A7C15 - (1 << 64)
L = dfp.load()
dev = torch.device("cuda", 0)
P = 10**8
cases = sys.argv[1:] or ["C2", "C2h", "H40", "D120"]
for name in cases:
    B = {"C2": 10**7, "C2h": 10**7, "H40": 4 * 10**7, "D120": 12 * 10**7}[name]
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, None) == 0
    if name in ("C2h", "H40"):
        bk.mul_(MIX)
        pk.mul_(MIX)
    cap = P
    ob = torch.empty(cap, dtype=torch.int64, device=dev)
    op = torch.empty(cap, dtype=torch.int32, device=dev)
    ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
    dt = torch.zeros(1, dtype=torch.int64, device=dev)
    t = HashTable(1, "int64", 0)
    t.build(bk)
    st = t.stats()
    ts = []
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), cap, dt.data_ptr(), ws.data_ptr(), 0)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = sorted(ts[1:])[2]
    M = int(dt.item())
    alg = 8 * P + 16 * B + 12 * M
    layout = "hashed" if st.get("buckets", 0) else "dense"
    print(f"{name}: B={B} {layout} buckets={st.get('buckets', 0)} matches={M} probe {ms * 1e3:.1f} us "
          f"frac {alg / (ms * 1e-3) / 8e12:.4f}", flush=True)
    t.close()
    del bk, pk, ob, op, ws
    torch.cuda.empty_cache()
