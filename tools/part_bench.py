"""Diagnostic: the multi-GPU partition kernels on one GPU — hj_partition_regions (one pass,
look-back) vs hj_partition_rows (histogram + scan + scatter) — for n rows, G destinations,
with and without the runtime filter; HIP-event times (median of 5)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from datafusion_parallelism_amd import _lib  # noqa: E402

if os.environ.get("DFP_HJ_LIB_VARIANT"):  # a diagnostic build (tools/lib_variants.py)
    _lib.LIB_PATH = os.environ["DFP_HJ_LIB_VARIANT"]
L = _lib.load()
dev = torch.device("cuda", 0)
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**8
keys = torch.empty(n, dtype=torch.int64, device=dev)
assert L.hj_gen_uniform_keys(keys.data_ptr(), n, 0xC0FFEE, 2 * 10**7, None) == 0


def timeit(fn, reps=5):
    ts = []
    for _ in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts[1:])[reps // 2]


for G in (1, 8):
    for filt in (False, True):
        sp = ctypes.byref(_lib.HjPartSpec(0, 0, 10**7 - 1)) if filt else None
        off = 2**31 if filt else 0
        ob = 4 if filt else 8
        out_k = torch.empty(G * n * ob // 4, dtype=torch.int32, device=dev)
        out_i = torch.empty(G * n, dtype=torch.int32, device=dev)
        counts = torch.empty(G, dtype=torch.int64, device=dev)
        ws = torch.empty(L.hj_partition_regions_workspace_bytes(n, G), dtype=torch.uint8, device=dev)
        ws2 = torch.empty(L.hj_partition_workspace_bytes(n, G), dtype=torch.uint8, device=dev)

        def reg():
            _lib.check(L.hj_partition_regions(1, keys.data_ptr(), None, 0, None, 0, n, G, sp, out_k.data_ptr(), ob, off,
                                              out_i.data_ptr(), 4, n, counts.data_ptr(), ws.data_ptr(), None))

        def rows():
            _lib.check(L.hj_partition_rows(1, keys.data_ptr(), None, 0, None, 0, n, G, sp, out_k.data_ptr(), ob, off,
                                           out_i.data_ptr(), 4, counts.data_ptr(), ws2.data_ptr(), None))

        tr, tg = timeit(reg), timeit(rows)
        kept = int(counts.sum())
        gb = (8 * n + (ob + 4) * kept) / 1e9
        print(f"G={G} filter={filt}: regions {tr * 1e3:.1f} us ({gb / tr * 1e3:.2f} TB/s), "
              f"rows {tg * 1e3:.1f} us, kept {kept}", flush=True)
        del out_k, out_i
