"""Sweep: probe-kernel time vs load factor / hit rate (HIP events, one process), plus a
host-side breakdown of one build step. Diagnostic tool (not part of the bench)."""
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
assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
pks = {}
for name, rng in [("hit50", 2 * B), ("hit100", B), ("hit0", 1)]:
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, rng, None) == 0
    if name == "hit0":
        pk += 10**12
    pks[name] = pk
ob = torch.empty(P, dtype=torch.int64, device=dev)
op = torch.empty(P, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def time_probe(t, pk, reps=5):
    ts = []
    for _ in range(reps):
        ev0.record()
        t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), P, dt.data_ptr(), ws.data_ptr(), 0)
        ev1.record()
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    return min(ts), int(dt.item())


for lf in ["0.3", "0.5", "0.7", "0.9"]:
    os.environ["DFP_HJ_LOAD_FACTOR"] = lf
    t = HashTable(1, "int64", 0)
    t.build(bk)
    st = t.stats()
    for name, pk in pks.items():
        ms, m = time_probe(t, pk)
        print(f"LF={lf} table={st['table_bytes'] / 1e6:.0f}MB build={st['build_ns'] / 1e6:.3f}ms {name}: "
              f"probe {ms:.3f} ms ({P / ms / 1e6:.0f} Mrows/s) matches={m}", flush=True)
    t.close()

# host-side breakdown of one build step
os.environ["DFP_HJ_LOAD_FACTOR"] = "0.5"
for it in range(3):
    t0 = time.perf_counter()
    t = HashTable(1, "int64", 0)
    t1 = time.perf_counter()
    t.append(0, bk)
    t2 = time.perf_counter()
    t.finish(0)
    t3 = time.perf_counter()
    dev_ms = t.build_ns() / 1e6
    t.close()
    t4 = time.perf_counter()
    print(f"step {it}: create {1e3 * (t1 - t0):.3f} ms append {1e3 * (t2 - t1):.3f} ms finish {1e3 * (t3 - t2):.3f} ms "
          f"(device {dev_ms:.3f}) close {1e3 * (t4 - t3):.3f} ms", flush=True)
