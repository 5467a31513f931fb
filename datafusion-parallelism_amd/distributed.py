"""Multi-GPU hash join: one process per GPU, build side radix-sharded across ranks.

SURVEY.md §8(e): both sides are partitioned by hash bits so that rank g owns the keys
with ``mix64(key) & (G-1) == g`` (the reference's nearest relative is the high-bit shard
function of src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16; here the LOW
hash bits pick the rank because the table index uses the high 32 bits). The one
exchange step is an all-to-all of ``(key, global row id)`` over RCCL (torch.distributed
backend "nccl" on ROCm = RCCL over xGMI); each rank then builds and probes its shard
independently with the single-GPU kernels, emitting global ``(build_row, probe_row)``
pairs. There is no other collective on the data path.

The partition and local-join steps are pluggable only so that the exchange logic can be
exercised by world_size-2 ``gloo`` tests on a machine without a GPU; the default (and
only product) implementations are the HIP kernels.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch
import torch.distributed as dist

from . import _lib
from ._lib import HJ_INT32, HJ_INT64, check
from .table import HashTable


def gpu_radix_partition(keys: torch.Tensor, ids: torch.Tensor | None, id_base: int, nparts: int,
                        stream: int | None = None, id_dtype: torch.dtype = torch.int64):
    """hj_radix_partition on device tensors -> (keys grouped by destination, ids
    (int64 = u64 build ids, int32 = u32 probe ids), counts[nparts] int64 device tensor)."""
    L = _lib.load()
    n = keys.numel()
    kt = HJ_INT64 if keys.dtype == torch.int64 else HJ_INT32
    out_k = torch.empty(n, dtype=keys.dtype, device=keys.device)
    out_i = torch.empty(n, dtype=id_dtype, device=keys.device)
    counts = torch.zeros(nparts, dtype=torch.int64, device=keys.device)
    ws = torch.empty(max(L.hj_partition_workspace_bytes(n, nparts), 8), dtype=torch.uint8, device=keys.device)
    s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
    check(L.hj_radix_partition(kt, keys.data_ptr(), None, 0, None if ids is None else ids.data_ptr(), id_base, n,
                               nparts, out_k.data_ptr(), out_i.data_ptr(), 8 if id_dtype == torch.int64 else 4,
                               counts.data_ptr(), ws.data_ptr(), s))
    return out_k, out_i, counts


def gpu_local_join(build_keys: torch.Tensor, build_ids: torch.Tensor, probe_keys: torch.Tensor,
                   probe_ids: torch.Tensor, capacity_hint: int | None = None):
    """Build this rank's shard with explicit global build ids and probe it with global
    probe ids -> (build_idx int64 [u64 values], probe_idx int32 [u32 values])."""
    dev = probe_keys.device
    kt = "int64" if build_keys.dtype == torch.int64 else "int32"
    # received build ids ascend (stable partition, ranks in order): when they also fit
    # 31 bits the table keeps them in place of row numbers (no id gather per pair)
    nbi = build_ids.numel()
    u31 = nbi == 0 or bool(((build_ids[-1] < 2**31) & (build_ids[0] >= 0) &
                            (nbi < 2 or bool((build_ids[1:] > build_ids[:-1]).all()))).item())
    with HashTable(1, kt, dev.index or 0) as t:
        t.append(0, build_keys, ids=build_ids, ids_u31=u31)
        t.finish(0)
        n = probe_keys.numel()
        pid32 = probe_ids if probe_ids.dtype == torch.int32 else probe_ids.to(torch.int32)
        ws = torch.empty(HashTable.workspace_bytes(n), dtype=torch.uint8, device=dev)
        d_total = torch.zeros(1, dtype=torch.int64, device=dev)
        cap = max(capacity_hint or n, 1)
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(2):
            ob = torch.empty(cap, dtype=torch.int64, device=dev)
            op = torch.empty(cap, dtype=torch.int32, device=dev)
            t.probe_async(probe_keys.data_ptr(), n, ob.data_ptr(), op.data_ptr(), cap, d_total.data_ptr(),
                          ws.data_ptr(), s, probe_ids_ptr=pid32.data_ptr())
            total = int(d_total.item())
            if total <= cap:
                return ob[:total], op[:total]
            cap = total
    raise RuntimeError("unreachable")


@dataclass
class ExchangeStats:
    sent_rows: int = 0
    recv_rows: int = 0


def all_to_all_rows(keys_by_dest: torch.Tensor, ids_by_dest: torch.Tensor, counts: torch.Tensor,
                    group=None) -> tuple[torch.Tensor, torch.Tensor, ExchangeStats]:
    """Exchange destination-grouped rows: counts first (all_to_all of G int64), then
    keys and ids with uneven splits (all_to_all_single)."""
    world = dist.get_world_size(group)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    assert len(send) == world
    rk = torch.empty(sum(recv), dtype=keys_by_dest.dtype, device=keys_by_dest.device)
    ri = torch.empty(sum(recv), dtype=ids_by_dest.dtype, device=ids_by_dest.device)
    dist.all_to_all_single(rk, keys_by_dest, output_split_sizes=recv, input_split_sizes=send, group=group)
    dist.all_to_all_single(ri, ids_by_dest, output_split_sizes=recv, input_split_sizes=send, group=group)
    return rk, ri, ExchangeStats(sum(send), sum(recv))


class DistributedHashJoin:
    """Inner equi-join of a build and a probe column that are each spread over the ranks
    (rank r holds rows [base_r, base_r + n_r) of the global column)."""

    def __init__(self, group=None, partition_fn: Callable | None = None, local_join_fn: Callable | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.partition_fn = partition_fn or gpu_radix_partition
        self.local_join_fn = local_join_fn or gpu_local_join

    def shard(self, keys: torch.Tensor, id_base: int, id_dtype: torch.dtype = torch.int64):
        """Partition by destination rank and exchange: -> (keys, global ids, stats).
        Build rows carry u64 ids (int64), probe rows u32 ids (int32, the reference's
        UInt32 probe index): 16 resp. 12 bytes per int64-key row on the wire."""
        if self.partition_fn is gpu_radix_partition:
            k, i, c = gpu_radix_partition(keys, None, id_base, self.world, id_dtype=id_dtype)
        else:
            k, i, c = self.partition_fn(keys, None, id_base, self.world)
        return all_to_all_rows(k, i, c, self.group)

    def run(self, build_keys: torch.Tensor, build_base: int, probe_keys: torch.Tensor, probe_base: int,
            capacity_hint: int | None = None):
        """-> this rank's share of the global pairs (build_idx, probe_idx)."""
        bk, bi, _ = self.shard(build_keys, build_base)
        pk, pi, _ = self.shard(probe_keys, probe_base, torch.int32)
        return self.local_join_fn(bk, bi, pk, pi, capacity_hint)
