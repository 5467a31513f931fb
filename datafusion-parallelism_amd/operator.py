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

  ProbeLookupStreamImplementation (src/operator/probe_lookup_implementation/
    probe_lookup_implementation.rs:19-80): Inner, Left, Right, Full, LeftSemi, LeftAnti,
    RightSemi, RightAnti                                      JoinType + _probe_batch /
                                                              _finalize_build_side
  apply_join_filter_to_indices (src/shared/datafusion_private.rs:295-328)
                                                              JoinFilter

Join keys: one Int32/Int64 column goes to the table as is (exact keys); several key
columns, or a key of any other fixed-width or Utf8/Binary type, go through
hj_composite_keys (one 64-bit key per row from all key columns, the reference's
calculate_hash) and the candidate pairs through hj_filter_equal_pairs (equal_rows_arr).
Output columns are materialised on the GPU
(columns.DeviceColumn.take: the build side is uploaded once after the barrier, each probe
batch once). The reference's CPU strategies (Original, New..New10) are not part of this
package.
"""
from __future__ import annotations

import enum
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Iterable, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

from ._lib import HjError, HJ_ERR_INVALID
from .columns import DeviceColumn, DeviceRecordBatch, composite_keys, filter_equal_pairs, mark_rows, select_rows
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
    raise HjError(HJ_ERR_INVALID, f"join key type {arr.type} is not an Int32/Int64 key")


def _is_simple_key(arrays: Sequence[pa.Array]) -> bool:
    """One Int32/Int64 key column: the table takes it as is; anything else is composite."""
    return len(arrays) == 1 and (pa.types.is_int64(arrays[0].type) or pa.types.is_int32(arrays[0].type))


class JoinType(enum.Enum):
    """datafusion_common::JoinType as supported by the reference's probe side
    (probe_lookup_implementation.rs:32-43). Left = build side, right = probe side."""
    Inner = "inner"
    Left = "left"
    Right = "right"
    Full = "full"
    LeftSemi = "leftsemi"
    LeftAnti = "leftanti"
    RightSemi = "rightsemi"
    RightAnti = "rightanti"

    @classmethod
    def parse(cls, v: "JoinType | str") -> "JoinType":
        if isinstance(v, JoinType):
            return v
        key = str(v).lower().replace("_", "").replace(" ", "").replace("outer", "")
        for jt in cls:
            if jt.value == key:
                return jt
        raise HjError(HJ_ERR_INVALID, f"unknown join type {v!r}")

    @property
    def marks_build(self) -> bool:  # build-side visited bitset (ConcurrentBitSet)
        return self in (JoinType.Left, JoinType.Full, JoinType.LeftSemi, JoinType.LeftAnti)


class JoinFilter:
    """A non-equi join condition applied to the equal-key candidate pairs
    (apply_join_filter_to_indices, src/shared/datafusion_private.rs:295-328):
    `expression(left_rows, right_rows)` gets the candidate rows of the `left_columns` /
    `right_columns` it reads (pyarrow RecordBatches, one row per pair) and returns a
    BooleanArray; null counts as false."""

    def __init__(self, expression: Callable[[pa.RecordBatch, pa.RecordBatch], pa.Array],
                 left_columns: Sequence[str] | None = None, right_columns: Sequence[str] | None = None):
        self.expression = expression
        self.left_columns = left_columns
        self.right_columns = right_columns


def _batch(cols: Sequence[DeviceColumn], names: Sequence[str]) -> pa.RecordBatch:
    return pa.RecordBatch.from_arrays([c.to_arrow() for c in cols], names=list(names))


class GpuIndexLookup:
    """The read-only shared table handed to every partition (IndexLookup<u64>), with the
    build RecordBatch's columns resident in HBM for output materialisation."""

    def __init__(self, table: HashTable, shared: "_SharedBuild | None" = None):
        self.table = table
        self._shared = shared

    @property
    def device(self) -> torch.device:
        return torch.device("cuda", self.table.device)

    def get_iter(self, key: int):
        """Build rows of `key` in chain order (newest first)
        (src/operator/version10/lookup_implementation_3.rs:22-59). The reference keys
        the lookup by hash; the GPU table is keyed by the exact key (its hash is
        internal), which the equality re-check makes equivalent."""
        return iter(self.table.lookup(key))

    def matching_indices_device(self, probe_keys: pa.Array | Sequence[pa.Array],
                                build_side_records: pa.RecordBatch | None = None
                                ) -> tuple[torch.Tensor, torch.Tensor]:
        """get_matching_indices + equal_rows_arr on the GPU: ProbeBuildIndices after the
        equality filter as device tensors (build int64, probe int32). One Int32/Int64
        key: the table compares exact keys (fused). Composite keys: candidates of equal
        composite key, then hj_filter_equal_pairs on the key columns."""
        arrays = ([probe_keys] if isinstance(probe_keys, (pa.Array, pa.ChunkedArray, DeviceColumn))
                  else list(probe_keys))
        if self._shared is not None and (self._shared.composite or not _is_simple_key(arrays)):
            return self._composite_matches(arrays, build_side_records)
        if not _is_simple_key(arrays):
            raise HjError(HJ_ERR_INVALID, "probe keys do not match the build keys (one Int32/Int64 column)")
        probe_keys = arrays[0]
        n = probe_keys.length if isinstance(probe_keys, DeviceColumn) else len(probe_keys)
        if n == 0:
            return (torch.empty(0, dtype=torch.int64, device=self.device),
                    torch.empty(0, dtype=torch.int32, device=self.device))
        keys = probe_keys if isinstance(probe_keys, DeviceColumn) else DeviceColumn.from_arrow(probe_keys, self.device)
        # the device validity bitmap goes to the probe as is, from bit voff (no host read)
        return self.table.probe(keys.key_tensor(), keys.valid, device_output=True, valid_offset=keys.voff)

    def _composite_matches(self, arrays: list[pa.Array], build_side_records: pa.RecordBatch | None):
        sh = self._shared
        if len(arrays) != len(sh.key_exprs):
            raise HjError(HJ_ERR_INVALID, f"{len(arrays)} probe key columns for {len(sh.key_exprs)} build key columns")
        pcols = [a if isinstance(a, DeviceColumn) else DeviceColumn.from_arrow(a, self.device) for a in arrays]
        n = pcols[0].length
        if n == 0:
            return (torch.empty(0, dtype=torch.int64, device=self.device),
                    torch.empty(0, dtype=torch.int32, device=self.device))
        keys, valid = composite_keys(pcols)
        b, p = self.table.probe(keys, valid, device_output=True)
        rb = build_side_records if build_side_records is not None else sh.concatenated()
        bcols = self.build_columns(rb)
        kidx = [e if isinstance(e, int) else rb.schema.get_field_index(e) for e in sh.key_exprs]
        return filter_equal_pairs([bcols[i] for i in kidx], pcols, b, p)

    def matching_indices(self, probe_keys: pa.Array) -> tuple[pa.UInt64Array, pa.UInt32Array]:
        """Host form of matching_indices_device (UInt64 build, UInt32 probe)."""
        b, p = self.table.probe(probe_keys)
        return pa.array(b, type=pa.uint64()), pa.array(p, type=pa.uint32())

    def build_columns(self, build_side_records) -> list[DeviceColumn]:
        if isinstance(build_side_records, DeviceRecordBatch):  # resident since the build
            return build_side_records.device_columns
        if self._shared is not None:
            return self._shared.device_columns(build_side_records, self.device)
        return [DeviceColumn.from_arrow(c, self.device) for c in build_side_records.columns]


class _SharedBuild:
    """State shared by all partitions of one build (JoinStateInstances)."""

    def __init__(self, parallelism: int, device: int, devices: Sequence[int] | None = None, plan: str = "auto"):
        self.parallelism = parallelism
        self.device = devices[0] if devices else device
        self.devices = list(devices) if devices else None
        self.plan = plan
        self.lock = threading.Lock()
        self.table: HashTable | None = None
        self.key_type: str | None = None
        # per partition, its batches' columns uploaded once on arrival (DeviceColumn) and
        # their row counts
        self.batches: list[list[tuple[list[DeviceColumn], int]]] = [[] for _ in range(parallelism)]
        self.taken = [False] * parallelism
        self.ready = threading.Barrier(parallelism)
        self.record_batch: DeviceRecordBatch | None = None
        self.schema: pa.Schema | None = None
        self._dev_cols: list[DeviceColumn] | None = None
        self.composite = False          # keys through hj_composite_keys (several / non-integer columns)
        self.key_exprs: list = []       # the build key expressions (the equality filter's columns)

    def table_for(self, key_type: str) -> HashTable:
        with self.lock:
            if self.table is None:
                self.key_type = key_type
                # one table on one GPU, or one table over a node's GPUs (hj_build_begin_multi:
                # broadcast or radix shards behind the same build / probe calls)
                self.table = HashTable(self.parallelism, key_type, self.device, devices=self.devices,
                                       plan=self.plan)
            elif key_type != self.key_type:
                raise HjError(HJ_ERR_INVALID, "all build batches must have the same key type")
            return self.table

    def concatenated(self) -> DeviceRecordBatch:
        """Build RecordBatch in canonical order (partition 0 batches, then 1, ...): row i
        <-> build index i, concatenated on the device from the batches' resident columns
        (cooperatively_concatenate_arrow_arrays,
        src/operator/version10/parallel_join_execution_state.rs:256-298): no host
        combine_chunks and no second upload."""
        with self.lock:
            if self.record_batch is None:
                parts = [b for part in self.batches for b in part]
                schema = self.schema or pa.schema([])
                if parts:
                    ncol = len(parts[0][0])
                    cols = [DeviceColumn.concat([p[0][j] for p in parts]) for j in range(ncol)]
                    self.record_batch = DeviceRecordBatch(schema, cols, sum(p[1] for p in parts))
                    # the per-batch columns are no longer needed (the table keeps the key
                    # tensors it borrows alive itself): drop them, keep the row counts
                    self.batches = [[(None, n) for _, n in part] for part in self.batches]
                else:
                    dev = torch.device("cuda", self.device)
                    empty = [DeviceColumn.from_arrow(pa.array([], type=f.type), dev) for f in schema]
                    self.record_batch = DeviceRecordBatch(schema, empty, 0)
            return self.record_batch

    def device_columns(self, rb: pa.RecordBatch, device) -> list[DeviceColumn]:
        """A host build batch's columns in HBM, uploaded once for all partitions (callers
        that pass their own RecordBatch instead of the resident one)."""
        with self.lock:
            if self._dev_cols is None:
                self._dev_cols = [DeviceColumn.from_arrow(c, device) for c in rb.columns]
            return self._dev_cols


class BuildImplementation:
    """src/operator/build_implementation.rs:20-112 with the `Gpu` arm only."""

    def __init__(self, build_implementation_version: JoinReplacement, parallelism: int,
                 input_schema: pa.Schema | None = None, device: int = 0, devices: Sequence[int] | None = None,
                 plan: str = "auto"):
        """devices: build one table over these GPUs of the node (hj_build_begin_multi;
        DataFusion runs every partition in one process, so the in-process multi-GPU table
        is the drop-in's node-wide form); plan "auto" | "broadcast" | "radix" (the build
        side sharded by key hash, 1/G per GPU: builds larger than one GPU). Batches and
        probe keys live on devices[0]; the table moves rows to the other GPUs itself."""
        if build_implementation_version is not JoinReplacement.Gpu:
            raise NotImplementedError(
                f"{build_implementation_version} is one of the reference's CPU strategies; this package "
                "implements JoinReplacement.Gpu")
        if devices is not None and len(devices) < 1:
            raise HjError(HJ_ERR_INVALID, "devices must name at least one GPU")
        self.parallelism = parallelism
        self._shared = _SharedBuild(parallelism, device, devices, plan)
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
        if len(build_expressions) < 1:
            raise HjError(HJ_ERR_INVALID, "an equi-join needs at least one key column")
        with sh.lock:
            sh.key_exprs = list(build_expressions)
        dev = torch.device("cuda", sh.device)
        for batch in stream:
            with sh.lock:
                if sh.schema is None:
                    sh.schema = batch.schema
            if batch.num_rows == 0:
                continue
            # the batch's columns go to HBM once: the table reads its key column there, and
            # the concatenated build batch is assembled from them on the device
            dcols = [DeviceColumn.from_arrow(c, dev) for c in batch.columns]
            sh.batches[partition].append((dcols, batch.num_rows))
            arrays = evaluate_expressions(build_expressions, batch)
            kcols = [dcols[e if isinstance(e, int) else batch.schema.get_field_index(e)] for e in build_expressions]
            if _is_simple_key(arrays):
                k = kcols[0]
                sh.table_for(_key_type(arrays[0])).append(partition, k.key_tensor(), valid=k.valid,
                                                          valid_offset=k.voff)
            else:  # calculate_hash over every key column -> one int64 key per row
                keys, valid = composite_keys(kcols)
                with sh.lock:
                    sh.composite = True
                sh.table_for("int64").append(partition, keys, valid=valid)
        # every partition waits for every other before the table exists for all of them
        sh.ready.wait()
        table = sh.table_for(sh.key_type or "int64")
        table.finish(partition)
        return consumer.call(GpuIndexLookup(table, sh), sh.concatenated())


def _apply_filter(flt: JoinFilter, build_cols: list[DeviceColumn], build_names: Sequence[str],
                  probe_cols: list[DeviceColumn], probe_names: Sequence[str], b: torch.Tensor, p: torch.Tensor):
    """apply_join_filter_to_indices: evaluate the filter on the candidate rows, keep the
    pairs where it is true (order preserved)."""
    if b.numel() == 0:
        return b, p
    lsel = [i for i, n in enumerate(build_names) if flt.left_columns is None or n in flt.left_columns]
    rsel = [i for i, n in enumerate(probe_names) if flt.right_columns is None or n in flt.right_columns]
    left = _batch([build_cols[i].take(b) for i in lsel], [build_names[i] for i in lsel])
    right = _batch([probe_cols[i].take(p) for i in rsel], [probe_names[i] for i in rsel])
    mask = flt.expression(left, right)
    if isinstance(mask, pa.ChunkedArray):
        mask = mask.combine_chunks()
    keep = np.asarray(mask.fill_null(False).to_numpy(zero_copy_only=False), dtype=np.uint8)
    rows = select_rows(torch.from_numpy(keep).to(b.device), 1, len(keep))
    return b[rows], p[rows]


def probe_batch(join_type: JoinType, probe_expressions: Sequence[str | int], build_expressions: Sequence[str | int],
                filter: JoinFilter | None, build_side_records: pa.RecordBatch, read_only_join_map: GpuIndexLookup,
                probe_batch: pa.RecordBatch, build_visited: torch.Tensor | None = None) -> pa.RecordBatch | None:
    """One probe batch of any join type: the lookup_*_probe_batch functions of
    src/operator/probe_lookup_implementation/{inner,left_outer,right_outer,full,left_semi,
    left_anti,right_semi,right_anti}.rs. Build-side join types only mark `build_visited`
    here (their rows are emitted by finalize_build_side)."""
    jt = JoinType.parse(join_type)
    lookup = read_only_join_map
    dev = lookup.device
    n = probe_batch.num_rows
    # the probe batch goes to HBM once: its key columns feed the lookup, all columns the take
    probe_cols = [DeviceColumn.from_arrow(c, dev) for c in probe_batch.columns]
    key_cols = [probe_cols[e if isinstance(e, int) else probe_batch.schema.get_field_index(e)]
                for e in probe_expressions]
    b, p = lookup.matching_indices_device(key_cols, build_side_records)
    build_cols = lookup.build_columns(build_side_records)
    bnames, pnames = list(build_side_records.schema.names), list(probe_batch.schema.names)
    if filter is not None:
        b, p = _apply_filter(filter, build_cols, bnames, probe_cols, pnames, b, p)
    if jt.marks_build and build_visited is not None:
        mark_rows(b, build_side_records.num_rows, build_visited)
    if jt in (JoinType.LeftSemi, JoinType.LeftAnti):
        return None
    if jt in (JoinType.RightSemi, JoinType.RightAnti):
        flags = mark_rows(p, n)
        rows = select_rows(flags, 1 if jt is JoinType.RightSemi else 0, n).to(torch.int32)
        return _batch([c.take(rows) for c in probe_cols], pnames)
    if jt in (JoinType.Right, JoinType.Full):
        # append_right_indices(preserve_order = false): unmatched probe rows after the pairs
        unmatched = select_rows(mark_rows(p, n), 0, n).to(torch.int32)
        b = torch.cat([b, torch.full((unmatched.numel(),), -1, dtype=torch.int64, device=dev)])
        p = torch.cat([p, unmatched])
    return _batch([c.take(b) for c in build_cols] + [c.take(p) for c in probe_cols], bnames + pnames)


def finalize_build_side(join_type: JoinType, build_side_records: pa.RecordBatch, lookup: GpuIndexLookup,
                        build_visited: torch.Tensor, probe_schema: pa.Schema) -> pa.RecordBatch | None:
    """The once-only build-side emission of the last finishing partition
    (emit_matched_build_records / emit_unmatched_build_records, e.g.
    left_semi.rs:166-178, left_outer.rs:174-193, full.rs:181-200)."""
    jt = JoinType.parse(join_type)
    if not jt.marks_build:
        return None
    nb = build_side_records.num_rows
    rows = select_rows(build_visited, 1 if jt is JoinType.LeftSemi else 0, nb)
    cols = lookup.build_columns(build_side_records)
    out = [c.take(rows).to_arrow() for c in cols]
    names = list(build_side_records.schema.names)
    if jt in (JoinType.Left, JoinType.Full):
        out += [pa.nulls(rows.numel(), type=f.type) for f in probe_schema]
        names += list(probe_schema.names)
    return pa.RecordBatch.from_arrays(out, names=names)


def lookup_inner_join_probe_batch(probe_expressions: Sequence[str | int], build_expressions: Sequence[str | int],
                                  filter, build_side_records: pa.RecordBatch, read_only_join_map: GpuIndexLookup,
                                  probe_batch: pa.RecordBatch, output_schema: pa.Schema | None = None
                                  ) -> pa.RecordBatch:
    """src/operator/probe_lookup_implementation/inner.rs:79-129."""
    rb = globals()["probe_batch"](JoinType.Inner, probe_expressions, build_expressions, filter, build_side_records,
                                  read_only_join_map, probe_batch)
    if output_schema is not None:
        return pa.RecordBatch.from_arrays(rb.columns, schema=output_schema)
    return rb


class _Finalizer:
    """LimitedRc<()> over `parallelism` copies: the last release runs the build-side
    emission (src/utils/limited_rc.rs, InitializeCopiesOnce)."""

    def __init__(self, parallelism: int):
        self.left = parallelism
        self.lock = threading.Lock()
        self.visited: torch.Tensor | None = None

    def visited_for(self, nrows: int, device) -> torch.Tensor:
        with self.lock:
            if self.visited is None:
                self.visited = torch.zeros(max(nrows, 1), dtype=torch.uint8, device=device)
            return self.visited

    def release(self) -> bool:
        with self.lock:
            self.left -= 1
            return self.left == 0


class _ProbeConsumer:
    """PerformProbeLookup (src/operator/parallel_hash_join_executor.rs:20-68)."""

    def __init__(self, probe_stream, probe_expressions, build_expressions, join_type=JoinType.Inner, filter=None,
                 finalizer: _Finalizer | None = None, probe_schema: pa.Schema | None = None):
        self.probe_stream = probe_stream
        self.probe_expressions = probe_expressions
        self.build_expressions = build_expressions
        self.join_type = JoinType.parse(join_type)
        self.filter = filter
        self.finalizer = finalizer
        self.probe_schema = probe_schema

    def call(self, lookup: GpuIndexLookup, record_batch: pa.RecordBatch):
        jt = self.join_type
        visited = None
        if jt.marks_build:
            visited = self.finalizer.visited_for(record_batch.num_rows, lookup.device)
        out = []
        for b in self.probe_stream:
            rb = probe_batch(jt, self.probe_expressions, self.build_expressions, self.filter, record_batch, lookup, b,
                             visited)
            if rb is not None:
                out.append(rb)
        if jt.marks_build and self.finalizer.release():
            rb = finalize_build_side(jt, record_batch, lookup, visited, self.probe_schema)
            if rb is not None:
                out.append(rb)
        return out


class ParallelHashJoin:
    """src/operator/parallel_hash_join.rs:16-168: `left` is the build side, `right` the
    probe side, each a list of partitions (lists of RecordBatches); `join_type` one of
    JoinType (names as DataFusion's); `filter` an optional JoinFilter. Output
    partitioning follows the probe side (RoundRobinBatch(N), 85-91); build-side rows of
    Left / Full / LeftSemi / LeftAnti joins come from the last partition to finish."""

    def __init__(self, left: list[list[pa.RecordBatch]], right: list[list[pa.RecordBatch]],
                 on: Sequence[tuple[str, str]], join_type: JoinType | str = JoinType.Inner, device: int = 0,
                 replacement: JoinReplacement = JoinReplacement.Gpu, filter: JoinFilter | None = None,
                 right_schema: pa.Schema | None = None, devices: Sequence[int] | None = None, plan: str = "auto"):
        """devices / plan: one build table over several GPUs (BuildImplementation)."""
        if len(on) < 1:
            raise HjError(HJ_ERR_INVALID, "an equi-join needs at least one (left, right) key pair")
        self.join_type = JoinType.parse(join_type)
        n = max(len(left), len(right), 1)
        self.left = list(left) + [[] for _ in range(n - len(left))]
        self.right = list(right) + [[] for _ in range(n - len(right))]
        self.parallelism = n
        self.on = list(on)
        self.filter = filter
        self.right_schema = right_schema or next((b.schema for part in self.right for b in part), None)
        self._build = BuildImplementation(replacement, n, device=device, devices=devices, plan=plan)
        self._finalizer = _Finalizer(n)

    def execute(self, partition: int) -> list[pa.RecordBatch]:
        lkeys, rkeys = [l for l, _ in self.on], [r for _, r in self.on]
        consumer = _ProbeConsumer(self.right[partition], rkeys, lkeys, self.join_type, self.filter, self._finalizer,
                                  self.right_schema)
        return self._build.build_side(partition, self.left[partition], lkeys, consumer)

    def collect(self) -> list[pa.RecordBatch]:
        """DataFusion `collect`: execute every partition concurrently."""
        with ThreadPoolExecutor(max_workers=self.parallelism) as ex:
            futs = [ex.submit(self.execute, p) for p in range(self.parallelism)]
            out = []
            for f in futs:
                out.extend(f.result())
        return out
