"""Build the in-tree C-ABI library ``lib/libdfp_hj.so`` (gfx950 code objects).

The kernels are compiled by ``hipcc --offload-arch=gfx950``; the host layer by g++.
The library links the HIP runtime and RCCL that PyTorch-ROCm ships (``torch/lib/libamdhip64.so``,
``torch/lib/librccl.so``, SONAME ``librccl.so.1`` as /opt/rocm's)
so that a process which also uses torch for device memory, streams and
``torch.distributed`` holds exactly one HIP/HSA runtime. (``/opt/rocm``'s runtime has
SONAME ``libamdhip64.so.7``; torch's has none, so linking the ROCm one would load a
second runtime next to torch's.)
"""
from __future__ import annotations

import importlib.util
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libdfp_hj.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = "gfx950"

SOURCES_HIP = ["hj_kernels.hip", "hj_columns.hip", "hj_keys.hip"]
SOURCES_CPP = ["hj_api.cpp", "hj_dist.cpp"]
HEADERS = ["hj_device.h", "hj_launch.h", "hj_util.h", "hj_host.h", "hj_comm.h"]
# test library: the product objects + the in-process thread transport for hj_comm
# (tests/test_gpu_dist_threads.py); never part of libdfp_hj.so
COMMTEST_LIB = os.path.join(LIBDIR, "libdfp_hj_commtest.so")
SOURCES_COMMTEST = ["hj_comm_threads.cpp"]


def torch_lib_dir() -> str:
    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("PyTorch-ROCm is required for its HIP runtime")
    d = os.path.join(os.path.dirname(spec.origin), "lib")
    if not os.path.exists(os.path.join(d, "libamdhip64.so")):
        raise RuntimeError(f"no libamdhip64.so under {d}")
    return d


def _stale(lib: str = LIB, extra: tuple[str, ...] = ()) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in SOURCES_HIP + SOURCES_CPP + HEADERS + list(extra)]
    deps += [os.path.join(INCLUDE, "hj.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, verbose: bool = False, defines: tuple[str, ...] = (), out: str = LIB) -> str:
    """Compile the HIP kernels + C-ABI host layer; returns the library path. `defines` and
    `out` serve diagnostic builds only (tools/build_ablation.py); the product library is
    built without defines into lib/libdfp_hj.so."""
    if not force and not _stale(out):
        return out
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    hipcc = shutil.which("hipcc") or os.path.join(rocm, "bin", "hipcc")
    tlib = torch_lib_dir()
    objdir = os.path.join(HERE, "build") if out == LIB else out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    objs, cmds = [], []
    for src in SOURCES_HIP:
        obj = os.path.join(objdir, src + ".o")
        cmds.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", *dflags, "-I", INCLUDE,
                     "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    for src in SOURCES_CPP:
        obj = os.path.join(objdir, src + ".o")
        cmds.append(["g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", INCLUDE,
                     "-I", os.path.join(rocm, "include"), "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    # the translation units compile independently: in parallel
    with ThreadPoolExecutor(max_workers=len(cmds)) as ex:
        list(ex.map(lambda c: _run(c, verbose), cmds))
    tmp = out + ".tmp"
    _run(["g++", "-shared", "-o", tmp, *objs, f"-L{tlib}", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{tlib}",
          "-Wl,--no-undefined", "-lpthread"], verbose)
    os.replace(tmp, out)
    return out


def build_commtest(force: bool = False, verbose: bool = False) -> str:
    """lib/libdfp_hj_commtest.so: the product library's objects (built first) plus the
    thread transport (hj_test_* entry points). Test infrastructure only. `force` relinks
    this library; the product objects are rebuilt only when stale."""
    build(verbose=verbose)
    if not force and not _stale(COMMTEST_LIB, tuple(SOURCES_COMMTEST)):
        return COMMTEST_LIB
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tlib = torch_lib_dir()
    objdir = os.path.join(HERE, "build")
    objs = [os.path.join(objdir, src + ".o") for src in SOURCES_HIP + SOURCES_CPP]
    for src in SOURCES_COMMTEST:
        obj = os.path.join(objdir, src + ".o")
        _run(["g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", INCLUDE,
              "-I", os.path.join(rocm, "include"), "-c", os.path.join(CSRC, src), "-o", obj], verbose)
        objs.append(obj)
    tmp = COMMTEST_LIB + ".tmp"
    _run(["g++", "-shared", "-o", tmp, *objs, f"-L{tlib}", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{tlib}",
          "-Wl,--no-undefined", "-lpthread"], verbose)
    os.replace(tmp, COMMTEST_LIB)
    return COMMTEST_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_commtest(verbose=True))
