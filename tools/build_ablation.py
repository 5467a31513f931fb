"""Diagnostic build: the library with the sliced probe's timing ablations compiled in
(-DDFP_HJ_ABLATIONS) into tools/lib/libdfp_hj_abl.so. Ablations produce wrong pairs by
design and are selected at run time by DFP_HJ_ABLATE (bits: emit 1 no stores, 2 no
entries, 8 no duplicate-segment reads; lookup 4 no bucket lookup, 128 plain item order).
The product library (lib/libdfp_hj.so) has none of this code.

Use from a tool script, before anything loads the library:
    import tools.build_ablation as ab; ab.use()
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "lib", "libdfp_hj_abl.so")


def build(force=False):
    sys.path.insert(0, os.path.join(ROOT, "datafusion-parallelism_amd"))
    import build as hipbuild

    sys.path.pop(0)
    return hipbuild.build(force=force, verbose=True, defines=("DFP_HJ_ABLATIONS",), out=OUT)


def use():
    """Point the package's loader at the diagnostic library (must run before load())."""
    sys.path.insert(0, ROOT)
    from datafusion_parallelism_amd import _lib

    if not os.path.exists(OUT):
        raise ImportError(f"{OUT} missing: run python tools/build_ablation.py on the build host")
    _lib.LIB_PATH = OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
