"""Diagnostic: hj_key_minmax over n int64 keys (the build's key-range reduction kernel),
HIP-event median of 20 calls."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from datafusion_parallelism_amd import _lib  # noqa: E402

if os.environ.get("DFP_HJ_LIB_VARIANT"):
    _lib.LIB_PATH = os.environ["DFP_HJ_LIB_VARIANT"]
L = _lib.load()
dev = torch.device("cuda", 0)
for n in (10**7, 10**8):
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    assert L.hj_gen_uniform_keys(keys.data_ptr(), n, 7, 2 * n, None) == 0
    ws = torch.empty(L.hj_key_minmax_workspace_bytes(), dtype=torch.uint8, device=dev)
    out = torch.empty(2, dtype=torch.int64, device=dev)
    ts = []
    for _ in range(21):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        _lib.check(L.hj_key_minmax(1, keys.data_ptr(), None, 0, n, out.data_ptr(), ws.data_ptr(), None))
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[1:])
    print(f"{os.environ.get('DFP_HJ_LIB_VARIANT', 'product')} n={n}: {ts[10]:.1f} us "
          f"({8 * n / ts[10] / 1e3:.0f} GB/s), min {ts[0]:.1f}", flush=True)
