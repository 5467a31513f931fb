"""Host-side mirror of the reference's operator/plugin interface for the hot path.

The reference (Rust, DataFusion 40) plugs build strategies in behind
``BuildImplementation`` and hands the built table to the probe side through the
``IndexLookup`` / ``IndexLookupConsumer`` seam. This module restates that surface in
Python over pyarrow RecordBatches, with a single new strategy, ``JoinReplacement.Gpu``,
whose build and probe run on the gfx950 kernels through the C ABI (``include/hj.h``):

  reference                                                   here
  ---------------------------------------------------------   ---------------------------------
  JoinReplacement (src/parse_sql.rs:12-24)                    JoinReplacement (+ Gpu)
  BuildImplementation::new (src/operator/build_implementation.rs:34-48)
                                                              BuildImplementation(...)
  BuildImplementation::build_side (…:50-112)                  BuildImplementation.build_side
  IndexLookup::get_iter (src/utils/index_lookup.rs:1-6)       GpuIndexLookup.get_iter
  IndexLookupConsumer::call (src/operator/lookup_consumers.rs:4-9)
                                                              consumer.call(lookup, record_batch)
  get_matching_indices + equal_rows_arr (src/shared/shared.rs:29-47,
    src/shared/datafusion_private.rs:40-80)                   GpuIndexLookup.matching_indices
  lookup_inner_join_probe_batch (src/operator/probe_lookup_implementation/inner.rs:79-129)
                                                              lookup_inner_join_probe_batch
  ParallelHashJoin::execute (src/operator/parallel_hash_join.rs:140-167)
                                                              ParallelHashJoin.execute / collect

Only the inner join without a non-equi JoinFilter and with a single Int32/Int64 key
column is in scope; other join types and filters are SURVEY.md §8f rows.
The reference's CPU strategies (Original, New..New10) are not part of this package.
"""
from __future__ import annotations

import enum
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Iterable, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ._lib import HjError, HJ_ERR_INVALID
from .table import HashTable


class JoinReplacement(enum.Enum):
    """src/parse_sql.rs:12-24, plus the MI355X strategy."""
    Original = "Original"
    New = "New"
    New3 = "New3"
    New4 = "New4"
    New5 = "New5"
    New6 = "New6"
    New7 = "New7"
    New8 = "New8"
    New9 = "New9"
    New10 = "New10"
    Gpu = "Gpu"


def evaluate_expressions(expressions: Sequence[str | int], batch: pa.RecordBatch) -> list[pa.Array]:
    """src/shared/shared.rs:18-22 for plain column expressions (name or index)."""
    out = []
    for e in expressions:
        out.append(batch.column(e) if isinstance(e, int) else batch.column(batch.schema.get_field_index(e)))
    return out


def _key_type(arr: pa.Array) -> str:
    if pa.types.is_int64(arr.type):
        return "int64"
    if pa.types.is_int32(arr.type):
        return "int32"
    raise HjError(HJ_ERR_INVALID, f"join key type {arr.type} is not supported (Int32/Int64 only)")


class GpuIndexLookup:
    """The read-only shared table handed to every partition (IndexLookup<u64>)."""

    def __init__(self, table: HashTable):
        self.table = table

    def get_iter(self, key: int):
        """Build rows of `key` in chain order (newest first)
        (src/operator/version10/lookup_implementation_3.rs:22-59). The reference keys
        the lookup by hash; the GPU table is keyed by the exact key (its hash is
        internal), which the equality re-check makes equivalent."""
        return iter(self.table.lookup(key))

    def matching_indices(self, probe_keys: pa.Array) -> tuple[pa.UInt64Array, pa.UInt32Array]:
        """get_matching_indices + equal_rows_arr, fused on the GPU: returns
        ProbeBuildIndices after the equality filter (build UInt64, probe UInt32)."""
        b, p = self.table.probe(probe_keys)
        return pa.array(b, type=pa.uint64()), pa.array(p, type=pa.uint32())


class _SharedBuild:
    """State shared by all partitions of one build (JoinStateInstances)."""

    def __init__(self, parallelism: int, device: int):
        self.parallelism = parallelism
        self.device = device
        self.lock = threading.Lock()
        self.table: HashTable | None = None
        self.key_type: str | None = None
        self.batches: list[list[pa.RecordBatch]] = [[] for _ in range(parallelism)]
        self.taken = [False] * parallelism
        self.ready = threading.Barrier(parallelism)
        self.record_batch: pa.RecordBatch | None = None
        self.schema: pa.Schema | None = None

    def table_for(self, key_type: str) -> HashTable:
        with self.lock:
            if self.table is None:
                self.key_type = key_type
                self.table = HashTable(self.parallelism, key_type, self.device)
            elif key_type != self.key_type:
                raise HjError(HJ_ERR_INVALID, "all build batches must have the same key type")
            return self.table

    def concatenated(self) -> pa.RecordBatch:
        """Build RecordBatch in canonical order (partition 0 batches, then 1, ...):
        row i <-> build index i (cooperatively_concatenate_arrow_arrays,
        src/operator/version10/parallel_join_execution_state.rs:256-298)."""
        with self.lock:
            if self.record_batch is None:
                all_batches = [b for part in self.batches for b in part]
                if all_batches:
                    tbl = pa.Table.from_batches(all_batches).combine_chunks()
                    self.record_batch = tbl.to_batches()[0] if tbl.num_rows else pa.RecordBatch.from_pylist(
                        [], schema=tbl.schema)
                else:
                    self.record_batch = pa.RecordBatch.from_pylist([], schema=self.schema or pa.schema([]))
            return self.record_batch


class BuildImplementation:
    """src/operator/build_implementation.rs:20-112 with the `Gpu` arm only."""

    def __init__(self, build_implementation_version: JoinReplacement, parallelism: int,
                 input_schema: pa.Schema | None = None, device: int = 0):
        if build_implementation_version is not JoinReplacement.Gpu:
            raise NotImplementedError(
                f"{build_implementation_version} is one of the reference's CPU strategies; this package "
                "implements JoinReplacement.Gpu")
        self.parallelism = parallelism
        self._shared = _SharedBuild(parallelism, device)
        self._shared.schema = input_schema

    def build_side(self, partition: int, stream: Iterable[pa.RecordBatch], build_expressions: Sequence[str | int],
                   consumer):
        """Consume one partition's build stream, take part in the cross-partition
        barrier, and hand (lookup, build RecordBatch) to `consumer`. All `parallelism`
        partitions must call this concurrently (the last arriver builds the table)."""
        sh = self._shared
        with sh.lock:
            if partition < 0 or partition >= sh.parallelism:
                raise HjError(HJ_ERR_INVALID, f"bad partition {partition}")
            if sh.taken[partition]:
                raise HjError(HJ_ERR_INVALID, f"State already consumed for partition {partition}")
            sh.taken[partition] = True
        if len(build_expressions) != 1:
            raise HjError(HJ_ERR_INVALID, "only single-column equi-join keys are supported")
        for batch in stream:
            sh.batches[partition].append(batch)
            if sh.schema is None:
                sh.schema = batch.schema
            if batch.num_rows == 0:
                continue
            (keys,) = evaluate_expressions(build_expressions, batch)
            sh.table_for(_key_type(keys)).append(partition, keys)
        # every partition waits for every other before the table exists for all of them
        sh.ready.wait()
        table = sh.table_for(sh.key_type or "int64")
        table.finish(partition)
        return consumer.call(GpuIndexLookup(table), sh.concatenated())


def lookup_inner_join_probe_batch(probe_expressions: Sequence[str | int], build_expressions: Sequence[str | int],
                                  filter, build_side_records: pa.RecordBatch, read_only_join_map: GpuIndexLookup,
                                  probe_batch: pa.RecordBatch, output_schema: pa.Schema | None = None
                                  ) -> pa.RecordBatch:
    """src/operator/probe_lookup_implementation/inner.rs:79-129."""
    if filter is not None:
        raise NotImplementedError("non-equi JoinFilter is a SURVEY.md §8f row, not implemented")
    (probe_keys,) = evaluate_expressions(probe_expressions, probe_batch)
    if probe_batch.num_rows == 0 or build_side_records.num_rows == 0:
        b = pa.array([], type=pa.uint64())
        p = pa.array([], type=pa.uint32())
    else:
        b, p = read_only_join_map.matching_indices(probe_keys)
    cols = [pc.take(c, b) for c in build_side_records.columns] + [pc.take(c, p) for c in probe_batch.columns]
    names = list(build_side_records.schema.names) + list(probe_batch.schema.names)
    if output_schema is not None:
        return pa.RecordBatch.from_arrays(cols, schema=output_schema)
    return pa.RecordBatch.from_arrays(cols, names=names)


class _ProbeConsumer:
    """PerformProbeLookup (src/operator/parallel_hash_join_executor.rs:20-68)."""

    def __init__(self, probe_stream, probe_expressions, build_expressions):
        self.probe_stream = probe_stream
        self.probe_expressions = probe_expressions
        self.build_expressions = build_expressions

    def call(self, lookup: GpuIndexLookup, record_batch: pa.RecordBatch):
        return [lookup_inner_join_probe_batch(self.probe_expressions, self.build_expressions, None, record_batch,
                                              lookup, b) for b in self.probe_stream]


class ParallelHashJoin:
    """src/operator/parallel_hash_join.rs:16-168 for JoinType::Inner: `left` is the build
    side, `right` the probe side, each a list of partitions (lists of RecordBatches).
    Output partitioning follows the probe side (RoundRobinBatch(N), 85-91)."""

    def __init__(self, left: list[list[pa.RecordBatch]], right: list[list[pa.RecordBatch]],
                 on: Sequence[tuple[str, str]], join_type: str = "inner", device: int = 0,
                 replacement: JoinReplacement = JoinReplacement.Gpu):
        if join_type != "inner":
            raise NotImplementedError(f"join type {join_type} is a SURVEY.md §8f row")
        if len(on) != 1:
            raise HjError(HJ_ERR_INVALID, "only single-column equi-join keys are supported")
        n = max(len(left), len(right), 1)
        self.left = list(left) + [[] for _ in range(n - len(left))]
        self.right = list(right) + [[] for _ in range(n - len(right))]
        self.parallelism = n
        self.on = list(on)
        self._build = BuildImplementation(replacement, n, device=device)

    def execute(self, partition: int) -> list[pa.RecordBatch]:
        consumer = _ProbeConsumer(self.right[partition], [self.on[0][1]], [self.on[0][0]])
        return self._build.build_side(partition, self.left[partition], [self.on[0][0]], consumer)

    def collect(self) -> list[pa.RecordBatch]:
        """DataFusion `collect`: execute every partition concurrently."""
        with ThreadPoolExecutor(max_workers=self.parallelism) as ex:
            futs = [ex.submit(self.execute, p) for p in range(self.parallelism)]
            out = []
            for f in futs:
                out.extend(f.result())
        return out
