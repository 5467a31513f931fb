"""Diagnostic: the sliced lookup with parts of its work removed (diagnostic library,
tools/build_ablation.py; DFP_HJ_ABLATE bits 512 no ref stores, 1024 no entry loads, 2048 no
table reads — wrong pairs by design). One normal probe first fills the refs array, so an
ablated lookup leaves valid refs behind for the emission. Run under rocprofv3 --kernel-trace
--stats: each ablation's lookups are launches 2+5k.. of its block (printed order).

usage: python tools/lookup_ablate.py --config=c2 BITS [BITS ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_ablation as ab  # noqa: E402

ab.use()
import torch  # noqa: E402

import bench  # noqa: E402
import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

CFG = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--config=")), "c2")
BITS = [int(a) for a in sys.argv[1:] if not a.startswith("--")]
dfp.load()
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
for bits in BITS:
    os.environ["DFP_HJ_ABLATE"] = "0"
    t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), CAP, dt.data_ptr(), ws.data_ptr(), 0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    os.environ["DFP_HJ_ABLATE"] = str(bits)
    ev[0].record()
    for _ in range(5):
        t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), CAP, dt.data_ptr(), ws.data_ptr(), 0)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"ablate {bits:5d}: probe {ev[0].elapsed_time(ev[1]) / 5 * 1000:8.1f} us (pairs {int(dt.item())})", flush=True)
t.close()
