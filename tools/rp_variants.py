"""Diagnostic: build the library with region-partition tile shapes (threads x rows per
thread) into tools/lib/rp_T_I.so, for tools/part_bench.py (DFP_HJ_LIB_VARIANT)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
import build as hipbuild  # noqa: E402

# name -> defines: tile shape (threads x rows, threads * rows / 64 % 64 == 0), look-back
# windows per flag round trip, ablation bits (hj_kernels.hip kRpAbl: 1 no look-back wait,
# 2 no stores, 4 no ids; wrong output, timing only)
VARIANTS = {
    "t256x16": ("DFP_RP_THREADS=256", "DFP_RP_ITERS=16"),
    "t1024x8": ("DFP_RP_THREADS=1024", "DFP_RP_ITERS=8"),
    "nowait": ("DFP_HJ_ABLATIONS", "DFP_RP_ABL=1"),
    "nostore": ("DFP_HJ_ABLATIONS", "DFP_RP_ABL=2"),
    "noids": ("DFP_HJ_ABLATIONS", "DFP_RP_ABL=4"),
}
if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)

    def one(name):
        out = os.path.join(ROOT, "tools", "lib", f"rp_{name}.so")
        return hipbuild.build(force=True, defines=VARIANTS[name], out=out)
    with ThreadPoolExecutor(4) as ex:
        print(list(ex.map(one, names)))
