"""Diagnostic: build the library with region-partition tile shapes (threads x rows per
thread) into tools/lib/rp_T_I.so, for tools/part_bench.py (DFP_HJ_LIB_VARIANT)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
import build as hipbuild  # noqa: E402

VARIANTS = [(256, 16), (512, 16), (1024, 8), (256, 32)]  # threads x rows; threads * rows / 64 % 64 == 0
if __name__ == "__main__":
    def one(v):
        t, i = v
        out = os.path.join(ROOT, "tools", "lib", f"rp_{t}_{i}.so")
        return hipbuild.build(force=True, defines=(f"DFP_RP_THREADS={t}", f"DFP_RP_ITERS={i}"), out=out)
    with ThreadPoolExecutor(4) as ex:
        print(list(ex.map(one, VARIANTS)))
