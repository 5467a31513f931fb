"""Diagnostic: one build + 5 probes of a C2-shaped join (B from argv, P = 10^8; or a bench.py
config with --config=NAME), for per-kernel profiling with rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd import _lib  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(float(args[0])) if len(args) > 0 else 10**7
P = int(float(args[1])) if len(args) > 1 else 10**8
MIX = "--mix" in sys.argv  # C2h: keys mapped by k -> k * 0x9E3779B97F4A7C15 (hashed table)
CFG = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--config=")), None)  # a bench.py config
if os.environ.get("DFP_HJ_LIB_VARIANT"):  # a diagnostic build (tools/lib_variants.py)
    _lib.LIB_PATH = os.environ["DFP_HJ_LIB_VARIANT"]
L = dfp.load()
dev = torch.device("cuda", 0)
if CFG:
    import bench  # noqa: E402

    bk, pk, _, _ = bench.gen_inputs(bench.CONFIGS[CFG], 0, 1, dev)
    B, P = bk.numel(), pk.numel()
else:
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
    # --prange=F: probe keys uniform over F x B values (default 2: half the probe rows in range)
    PR = float(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--prange=")), "2"))
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, int(PR * B), None) == 0
    if MIX:
        bk.mul_(0x9E3779B97F4A7C15 - (1 << 64))
        pk.mul_(0x9E3779B97F4A7C15 - (1 << 64))
CAP = 2 * P
ob = torch.empty(CAP, dtype=torch.int64, device=dev)
op = torch.empty(CAP, dtype=torch.int32, device=dev)
ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
dt = torch.zeros(1, dtype=torch.int64, device=dev)
t = HashTable(1, "int64", 0)
t.build(bk)
for _ in range(5):
    t.probe_async(pk.data_ptr(), P, ob.data_ptr(), op.data_ptr(), CAP, dt.data_ptr(), ws.data_ptr(), 0)
torch.cuda.synchronize()
print("matches", int(dt.item()))
t.close()
