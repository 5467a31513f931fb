"""GPU: the operator-level mirror (datafusion_parallelism_amd.operator) on the reference's
own integration scenarios (src/lib.rs, JoinReplacement variants vs DataFusion's
HashJoinExec as control): results are compared as sorted sets, the reference's parity
notion (collect_and_sort_results, src/lib.rs:756-772)."""
import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

BATCH = 64


def batches_of(cols: dict, nbatches: int, size: int):
    out = []
    for i in range(nbatches):
        out.append(pa.RecordBatch.from_pydict({k: f(i, size) for k, f in cols.items()}))
    return out


def rng_ids(i, size):
    return pa.array(np.arange(i * size, (i + 1) * size, dtype=np.int32))


def split(batches, parts):
    return [batches[p::parts] for p in range(parts)]


def test_inner_join_no_filter(dfp):
    """src/lib.rs:67-132: base_table (16 x 64 rows, id1..id4) joined with four small
    tables on id -> 1024 rows, every id once; tables 796-820."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    base = batches_of({"id1": rng_ids, "id2": rng_ids, "id3": rng_ids, "id4": rng_ids,
                       "value": lambda i, s: pa.array(["hello"] * s)}, 16, BATCH)
    cur = pa.Table.from_batches(base)
    for k in range(1, 5):
        small = batches_of({"id": rng_ids, "value": lambda i, s: pa.array(["world"] * s)}, 16, BATCH)
        probe = cur.to_batches(max_chunksize=BATCH)
        join = ParallelHashJoin(split(small, 4), split(probe, 4), on=[("id", f"id{k}")])
        res = pa.Table.from_batches(join.collect())
        assert res.num_rows == 1024
        # keep the probe-side columns + the joined id for the next join
        cur = pa.table({n: res.column(i) for i, n in enumerate(res.column_names) if i >= 2})
    ids = np.sort(cur.column("id1").to_numpy())
    assert np.array_equal(ids, np.arange(1024))
    for k in range(2, 5):
        assert np.array_equal(np.sort(cur.column(f"id{k}").to_numpy()), np.arange(1024))


def test_inner_join_with_nulls(dfp):
    """src/lib.rs:149-193."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    left = pa.RecordBatch.from_pydict({"id": pa.array([1, 2, None], pa.int32()), "value": ["left"] * 3})
    right = pa.RecordBatch.from_pydict({"id": pa.array([None, 2, 3], pa.int32()), "value": ["right"] * 3})
    res = pa.Table.from_batches(ParallelHashJoin([[left]], [[right]], on=[("id", "id")]).collect())
    assert res.num_rows == 1
    assert [res.column(i).to_pylist() for i in range(4)] == [[2], ["left"], [2], ["right"]]


def test_inner_join_without_matches(dfp):
    """src/lib.rs:210-246."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    left = pa.RecordBatch.from_pydict({"id": pa.array([1, 2, None], pa.int32()), "value": ["left"] * 3})
    right = pa.RecordBatch.from_pydict({"id": pa.array([None, 4, 5], pa.int32()), "value": ["right"] * 3})
    res = ParallelHashJoin([[left]], [[right]], on=[("id", "id")]).collect()
    assert sum(b.num_rows for b in res) == 0


def test_operator_matches_oracle_parallel(dfp, oracle_mod):
    """8 build partitions (concurrent build_side + barrier) and 8 probe partitions of
    int64 keys with duplicates and nulls: the joined rows equal the oracle's pairs."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    rng = np.random.default_rng(21)
    bk = rng.integers(0, 4000, 20000)
    pk = rng.integers(0, 6000, 30000)
    bnull = rng.random(len(bk)) < 0.05
    build = pa.RecordBatch.from_pydict({"k": pa.array(bk, mask=bnull), "bid": np.arange(len(bk))})
    probe = pa.RecordBatch.from_pydict({"k": pa.array(pk), "pid": np.arange(len(pk))})
    bparts = split(pa.Table.from_batches([build]).to_batches(max_chunksize=1000), 8)
    pparts = split(pa.Table.from_batches([probe]).to_batches(max_chunksize=1000), 8)
    res = pa.Table.from_batches(ParallelHashJoin(bparts, pparts, on=[("k", "k")]).collect())
    got = sorted(zip(res.column("bid").to_pylist(), res.column("pid").to_pylist()))
    ob, op = oracle_mod.inner_join(bk, pk, ~bnull, None)
    want = sorted(zip(ob.tolist(), op.tolist()))
    assert got == want


@pytest.mark.parametrize("plan", ["radix", "broadcast"])
def test_operator_multi_gpu_table_matches_oracle(dfp, oracle_mod, plan):
    """ParallelHashJoin(devices=...) — the drop-in's node-wide form (one process runs every
    partition, build_implementation.rs:34-48, parallel_hash_join.rs:140-167): the shared
    build table of 8 concurrent partitions is one table over 4 GPUs (hj_build_begin_multi;
    [0] * 4 on this one-GPU box), and every probe partition's batches are probed through it.
    Joined rows equal the oracle's pairs; each probe batch's pairs come out in canonical
    order (the multi table merges its shards' pairs)."""
    from datafusion_parallelism_amd.operator import ParallelHashJoin

    rng = np.random.default_rng(23)
    bk = rng.integers(-3000, 4000, 24000)
    pk = rng.integers(-5000, 6000, 30000)
    bnull = rng.random(len(bk)) < 0.05
    pnull = rng.random(len(pk)) < 0.03
    build = pa.RecordBatch.from_pydict({"k": pa.array(bk, mask=bnull), "bid": np.arange(len(bk))})
    probe = pa.RecordBatch.from_pydict({"k": pa.array(pk, mask=pnull), "pid": np.arange(len(pk))})
    # build partitions of consecutive batches: the canonical build index (partition 0's
    # batches, then partition 1's, ...) is then the bid column
    bb = pa.Table.from_batches([build]).to_batches(max_chunksize=1000)
    bparts = [bb[3 * p:3 * (p + 1)] for p in range(8)]
    pparts = split(pa.Table.from_batches([probe]).to_batches(max_chunksize=1000), 8)
    join = ParallelHashJoin(bparts, pparts, on=[("k", "k")], devices=[0] * 4, plan=plan)
    out = join.collect()
    for rb in out:  # per batch: probe rows ascending, build rows of one probe row descending
        pid = np.asarray(rb.column("pid"))
        bid = np.asarray(rb.column("bid"))
        same = pid[1:] == pid[:-1]
        assert np.all(pid[1:] >= pid[:-1]) and np.all(bid[1:][same] < bid[:-1][same])
    res = pa.Table.from_batches(out)
    got = sorted(zip(res.column("bid").to_pylist(), res.column("pid").to_pylist()))
    ob, op = oracle_mod.inner_join(bk, pk, ~bnull, ~pnull)
    want = sorted(zip(ob.tolist(), op.tolist()))
    assert got == want and len(got) > 0


def test_build_implementation_multi_gpu_lookup(dfp):
    """BuildImplementation(devices=...): get_iter on the node-wide table keeps the chain
    order (newest first) and the partition-state rule."""
    from datafusion_parallelism_amd import HjError
    from datafusion_parallelism_amd.operator import BuildImplementation, JoinReplacement

    class Collect:
        def call(self, lookup, record_batch):
            return [list(lookup.get_iter(k)) for k in (1, 2, 7)], record_batch.num_rows

    bi = BuildImplementation(JoinReplacement.Gpu, 1, devices=[0, 0], plan="radix")
    batches = [pa.RecordBatch.from_pydict({"id": pa.array(v, pa.int64())}) for v in ([1, 2, 3], [2, 4, 5], [1, 6, 7])]
    its, n = bi.build_side(0, batches, ["id"], Collect())
    assert its == [[6, 0], [3, 1], [8]] and n == 9  # version10/build_implementation.rs:98-178
    with pytest.raises(HjError, match="State already consumed for partition 0"):
        bi.build_side(0, batches, ["id"], Collect())


def test_build_side_state_consumed(dfp):
    """src/operator/version10/build_implementation.rs:32-33: a partition's state can be
    taken once."""
    from datafusion_parallelism_amd import HjError
    from datafusion_parallelism_amd.operator import BuildImplementation, JoinReplacement

    class Collect:
        def call(self, lookup, record_batch):
            return [lookup.get_iter(k) for k in (1, 2)], record_batch

    bi = BuildImplementation(JoinReplacement.Gpu, 1)
    batch = pa.RecordBatch.from_pydict({"id": pa.array([1, 2, 1], pa.int64())})
    (its, rb) = bi.build_side(0, [batch], ["id"], Collect())
    assert [list(i) for i in its] == [[2, 0], [1]]
    assert rb.num_rows == 3
    with pytest.raises(HjError, match="State already consumed for partition 0"):
        bi.build_side(0, [batch], ["id"], Collect())


def test_cpu_strategies_are_not_reimplemented():
    from datafusion_parallelism_amd.operator import BuildImplementation, JoinReplacement

    with pytest.raises(NotImplementedError):
        BuildImplementation(JoinReplacement.New10, 1)
