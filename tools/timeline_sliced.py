"""Diagnostic: per-workgroup timeline of the sliced probe's lookup and emission (the
diagnostic library, tools/build_ablation.py, records start / first phase / end and the
hardware id of every workgroup of the last launch). Prints, per kernel: the span, the
distribution of workgroup durations and of the first phase (the lookup's slice load),
how many workgroups each CU ran, and the tail (time from the 90th-percentile end to the
last end).

usage: python tools/timeline_sliced.py [--config=c2|c3|c2h] [--probes=3]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_ablation as ab  # noqa: E402

ab.use()
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

CFG = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--config=")), "c2")
NPROBE = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--probes=")), "3"))
L = dfp.load()
L.hj_debug_timeline.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda", 0)
bk, pk, _, _ = bench.gen_inputs(bench.CONFIGS[CFG], 0, 1, dev)
P = pk.numel()
CAP = 2 * P
ob = torch.empty(CAP, dtype=torch.int64, device=dev)
op = torch.empty(CAP, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
t = HashTable(1, "int64", 0)
t.build(bk)
for _ in range(NPROBE):
    t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), CAP, dt.data_ptr(), ws.data_ptr(), 0)
torch.cuda.synchronize()
print(f"# {CFG}: matches {int(dt.item())}")
t.close()

for which, name in ((0, "sl_lookup"), (1, "sl_emit")):
    buf = np.zeros(4 * 65536, dtype=np.uint64)
    assert L.hj_debug_timeline(which, buf.ctypes.data, 65536) == 0
    a = buf.reshape(-1, 4).astype(np.int64)
    a = a[a[:, 2] > 0]
    t0 = a[:, 0].min()
    st, ph, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, (a[:, 2] - t0) / 100.0  # us (100 MHz)
    dur, first = en - st, ph - st
    hw = a[:, 3]
    _, per_cu = np.unique(hw, return_counts=True)
    q = lambda x: " ".join(f"{v:7.1f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))  # noqa: E731
    print(f"## {name}: {len(a)} workgroups on {len(per_cu)} CUs, span {en.max():.1f} us "
          f"(last start {st.max():.1f}, p90 end {np.percentile(en, 90):.1f})")
    print(f"   duration  us p0/p10/p50/p90/p100: {q(dur)}  (mean {dur.mean():.1f})")
    print(f"   1st phase us p0/p10/p50/p90/p100: {q(first)}  (mean {first.mean():.1f})")
    print(f"   workgroups per CU: min {per_cu.min()} max {per_cu.max()} mean {per_cu.mean():.2f}")
    # busy CUs over time (10 buckets of the span)
    edges = np.linspace(0, en.max(), 11)
    busy = [int(((st < e1) & (en > e0)).sum()) for e0, e1 in zip(edges[:-1], edges[1:])]
    print(f"   workgroups live per tenth of the span: {busy}")
    # per-CU sequence: sum of durations / span (occupancy of the CU by this kernel)
    occ = []
    for h in np.unique(hw):
        m = hw == h
        occ.append(dur[m].sum() / en.max())
    print(f"   CU busy fraction (sum of its workgroups' durations / span): mean {np.mean(occ):.2f} min {np.min(occ):.2f}")

# per-phase cycle sums of the lookup (DFP_HJ_ABLATE=256 builds them, summed over every wave
# of the NPROBE launches): where a wave's time goes per block / window
if int(os.environ.get("DFP_HJ_ABLATE", "0")) & 256:
    L.hj_debug_lookup_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ph = np.zeros(8, dtype=np.uint64)
    assert L.hj_debug_lookup_phases(ph.ctypes.data, 1) == 0
    blocks, wins = int(ph[5]), int(ph[6])
    tot = float(ph[:5].sum())
    names = ["block setup", "entry loads issued", "wait for loads (+older stores)", "rows (LDS, stores, corr.)",
             "block end (atomics)"]
    print(f"## sl_lookup phases over {NPROBE} launches: {blocks} wave-blocks, {wins} wave-windows")
    for i, nm in enumerate(names):
        per = float(ph[i]) / max(1, blocks if i in (0, 4) else wins)
        print(f"   {nm:34s} {100 * float(ph[i]) / tot:5.1f} %  {per:9.0f} cycles per {'block' if i in (0, 4) else 'window'}")
