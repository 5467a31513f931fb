"""Diagnostic: build the library with compile-time knobs into tools/lib/<name>.so, for the
tools/*_bench.py scripts (DFP_HJ_LIB_VARIANT=tools/lib/<name>.so). Usage:
lib_variants.py NAME=DEF[=V][,DEF[=V]...] ... (e.g. mm512=DFP_MM_BLOCKS=512)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
import build as hipbuild  # noqa: E402

if __name__ == "__main__":
    specs = []
    for a in sys.argv[1:]:
        name, defs = a.split("=", 1)
        specs.append((name, tuple(d for d in defs.split(",") if d)))

    def one(spec):
        name, defs = spec
        return hipbuild.build(force=True, defines=defs, out=os.path.join(ROOT, "tools", "lib", f"{name}.so"))
    with ThreadPoolExecutor(4) as ex:
        print(list(ex.map(one, specs)))
