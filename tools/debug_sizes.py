"""Debug: C2-style join at increasing sizes, printing counts vs the closed form."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import datafusion_parallelism_amd as dfp
L = dfp.load()
dev = torch.device("cuda", 0)
for B, P in [(10**5, 10**6), (10**6, 10**7), (10**7, 10**7), (10**7, 10**8), (2 * 10**6, 10**8)]:
    bk = torch.empty(B, dtype=torch.int64, device=dev)
    pk = torch.empty(P, dtype=torch.int64, device=dev)
    assert L.hj_gen_perm_keys(bk.data_ptr(), B, 7368787, B, None) == 0
    assert L.hj_gen_uniform_keys(pk.data_ptr(), P, 0xC0FFEE, 2 * B, None) == 0
    torch.cuda.synchronize()
    with dfp.HashTable(1, "int64", 0) as t:
        t.build(bk)
        st = t.stats()
        b, p = t.probe(pk, device_output=True)
        hb, hp = t.probe(pk[:100000].cpu().numpy())
    print(B, P, "expected", int((pk < B).sum()), "got", b.numel(), "host-path(1e5)", len(hb),
          "exp1e5", int((pk[:100000] < B).sum()), "distinct", st["distinct_keys"], "build_ms", st["build_ns"] / 1e6,
          flush=True)
