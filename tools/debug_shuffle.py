#!/usr/bin/env python3
"""Diagnostic: the exchange pieces of distributed.shuffle at large row counts on one
rank (radix partition with nparts 1 must be the identity; RCCL all_to_all_single self
copies must be exact). Prints one line per check; no kernel indexes with the results."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from datafusion_parallelism_amd.distributed import gpu_radix_partition  # noqa: E402


def main():
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in (sys.argv[1:] or ["100000000", "200000000", "320000000"])]:
        keys = torch.randint(0, 6 * 10**8, (n,), dtype=torch.int64, device=dev)
        k, perm, counts = gpu_radix_partition(keys, None, 0, 1, id_dtype=torch.int64)
        torch.cuda.synchronize()
        ok_part = (int(counts[0]) == n, bool(torch.equal(k, keys)),
                   bool(torch.equal(perm, torch.arange(n, device=dev))))
        res = []
        # the same self-copy three ways: async + wait (as _exchange_cols), synchronous, and
        # synchronous after a full device sync (input surely complete): a mismatch in all
        # three points at the collective, not at stream ordering or buffer lifetime
        for mode in ("async_wait", "sync", "sync_after_devsync"):
            out = torch.full_like(keys, -1)
            if mode == "sync_after_devsync":
                torch.cuda.synchronize()
            w = dist.all_to_all_single(out, keys, output_split_sizes=[n], input_split_sizes=[n],
                                       async_op=(mode == "async_wait"))
            if w is not None:
                w.wait()
            torch.cuda.synchronize()
            ok_a2a = bool(torch.equal(out, keys))
            mism = int((out != keys).sum()) if not ok_a2a else 0
            first = int(torch.nonzero(out != keys)[0]) if mism else -1
            untouched = int((out == -1).sum()) if mism else 0
            res.append(f"{mode}: exact={ok_a2a} mismatches={mism} first_bad={first} untouched={untouched}")
            del out
        # and in rounds of <= A2A_MAX_BYTES (the fix in distributed._exchange_cols)
        from datafusion_parallelism_amd import distributed as D

        (o2,), _ = D._exchange_cols([keys], [[n]])
        torch.cuda.synchronize()
        res.append(f"rounds_of_{D.A2A_MAX_BYTES >> 20}MiB: exact={bool(torch.equal(o2, keys))}")
        del o2
        print(f"n={n} bytes={8 * n} partition(count,keys,perm)={ok_part} " + " | ".join(res), flush=True)
        del keys, k, perm
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
