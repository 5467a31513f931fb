#!/usr/bin/env python3
"""Diagnostic: the exchange pieces of distributed.shuffle at large row counts on one
rank (radix partition with nparts 1 must be the identity; RCCL all_to_all_single self
copies must be exact). Prints one line per check; no kernel indexes with the results."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from datafusion_parallelism_amd.distributed import gpu_radix_partition  # noqa: E402


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in (sys.argv[1:] or ["100000000", "200000000", "320000000"])]:
        keys = torch.randint(0, 6 * 10**8, (n,), dtype=torch.int64, device=dev)
        k, perm, counts = gpu_radix_partition(keys, None, 0, 1, id_dtype=torch.int64)
        torch.cuda.synchronize()
        ok_part = (int(counts[0]) == n, bool(torch.equal(k, keys)),
                   bool(torch.equal(perm, torch.arange(n, device=dev))))
        out = torch.empty_like(keys)
        w = dist.all_to_all_single(out, keys, output_split_sizes=[n], input_split_sizes=[n], async_op=True)
        w.wait()
        torch.cuda.synchronize()
        ok_a2a = bool(torch.equal(out, keys))
        mism = int((out != keys).sum()) if not ok_a2a else 0
        first = int(torch.nonzero(out != keys)[0]) if mism else -1
        print(f"n={n} bytes={8 * n} partition(count,keys,perm)={ok_part} a2a_exact={ok_a2a} mismatches={mism} "
              f"first_bad={first}", flush=True)
        del keys, k, perm, out
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
