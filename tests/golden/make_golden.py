"""Writes the golden fixtures under tests/golden/.

reference_kats.json — the known-answer tests the reference's own test suite holds for
  the hot path, transcribed as data (inputs + expected outputs) with the file:line they
  come from (jamesfer/datafusion-parallelism @ 2026-01-30). They are literal values
  from the reference's assertions; no reference source text is stored.

oracle_vectors.npz — seeded join cases (duplicates, nulls, int32/int64, extreme keys,
  empty sides) with the oracle's canonical pairs, for the GPU parity tests. The oracle
  itself is pinned by reference_kats.json (tests/test_oracle.py).

Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402

KATS = {
    "_source": "jamesfer/datafusion-parallelism @ 2026-01-30; literal values of the reference's assertions",
    "v10_build_lookup_map": {
        "ref": "src/operator/version10/build_implementation.rs:98-178",
        "batches": [[1, 2, 3], [2, 4, 5], [1, 6, 7]],
        "note": "lookup results are reversed by the test before comparison (ascending rows)",
        "expected_ascending": {"1": [0, 6], "2": [1, 3], "3": [2], "4": [4], "5": [5], "6": [7], "7": [8]},
        "absent": [999],
    },
    "fixed_table_insert_returns_previous": {
        "ref": "src/operator/version10/new_map_3/fixed_table.rs:1411-1419",
        "inserts": [[1, 1, None], [1, 2, 1], [4023, 4, None], [1, 5, 2], [4023, 6, 4]],
        "note": "[hash, value, expected previous value]",
    },
    "fixed_table_zero_hash": {
        "ref": "src/operator/version10/new_map_3/fixed_table.rs:1399-1409",
        "inserts": [[0, 100]] + [[i, i] for i in range(1, 64)],
        "expect_get": [[0, 100]],
    },
    "chain_follows_indexes": {
        "ref": "src/utils/concurrent_self_hash_join_map.rs:263-283",
        "note": "indices inserted in reverse; get_all returns them in the listed order",
        "pairs": {"1": [1, 4, 3], "2": [2, 7]},
    },
    "chain_with_zero": {"ref": "src/utils/concurrent_self_hash_join_map.rs:285-301", "key": 1, "indices": [1, 0, 3]},
    "chain_matching_last": {"ref": "src/utils/concurrent_self_hash_join_map.rs:303-319", "key": 1,
                            "indices": [1, 9, 3]},
    "chain_spanning_blocks": {
        "ref": "src/utils/concurrent_self_hash_join_map.rs:321-373",
        "note": "two blocks of 10 (offsets 0 and 10); A inserts 2,4,6 into block 0, B 3,5,7 into block 1, "
                "interleaved A,B,A,B,A,B",
        "inserts": [[0, 2], [1, 3], [0, 4], [1, 5], [0, 6], [1, 7]],
        "block_size": 10,
        "expected": [17, 6, 15, 4, 13, 2],
    },
    "partitioned_chains": {
        "ref": "src/utils/partitioned_concurrent_self_hash_join_map.rs:396-435",
        "blocks": [[1, 2, 1, 2], [3, 2, 1, 3]],
        "expected_after_block_1": {"1": [2, 0], "2": [3, 1]},
        "expected_after_block_2": {"1": [6, 2, 0], "2": [5, 3, 1]},
    },
    "sql_inner_join_no_filter": {
        "ref": "src/lib.rs:67-132 (tables 796-820)",
        "note": "5 tables of 16 batches x 64 rows, ids i*64..(i+1)*64; every id matches once in each join",
        "batches": 16, "batch_size": 64, "expected_rows": 1024,
    },
    "sql_inner_join_with_nulls": {
        "ref": "src/lib.rs:149-193",
        "left": [1, 2, None], "right": [None, 2, 3], "expected_left_right_ids": [[2, 2]],
    },
    "sql_inner_join_without_matches": {
        "ref": "src/lib.rs:210-246", "left": [1, 2, None], "right": [None, 4, 5], "expected_rows": 0,
    },
    "make_exponential_int_array_0_10": {
        "ref": "src/api_utils.rs:51-71", "expected": [0, 0, 0, 0, 1, 2, 2, 3, 5, 7],
    },
}


def oracle_vectors():
    cases = {}
    rng = np.random.default_rng(20261015)
    specs = [
        ("empty_build", 0, 50, 10, 0.0, np.int64),
        ("empty_probe", 50, 0, 10, 0.0, np.int64),
        ("dups_nulls_i64", 3000, 5000, 800, 0.1, np.int64),
        ("dups_nulls_i32", 4097, 4095, 1500, 0.05, np.int32),
        ("unique_i64", 5000, 9000, 0, 0.0, np.int64),
        ("hot_key", 2000, 300, 0, 0.0, np.int64),
    ]
    for name, nb, np_, kr, nf, dt in specs:
        if name == "unique_i64":
            bk = rng.permutation(nb).astype(dt) * 3 - 7000
            pk = rng.integers(-8000, 8000, np_).astype(dt)
        elif name == "hot_key":
            bk = np.where(rng.random(nb) < 0.3, 77, rng.integers(0, 500, nb)).astype(dt)
            pk = rng.integers(0, 600, np_).astype(dt)
            pk[::7] = 77
        else:
            bk = rng.integers(-kr, kr, nb).astype(dt)
            pk = rng.integers(-kr, kr, np_).astype(dt)
        bv = (rng.random(nb) >= nf) if nf else np.ones(nb, bool)
        pv = (rng.random(np_) >= nf) if nf else np.ones(np_, bool)
        ob, op = oracle.inner_join(bk, pk, bv, pv)
        cases[name] = dict(bk=bk, pk=pk, bv=bv, pv=pv, ob=ob, op=op)
    # extreme values incl. the key whose stored form collides with "empty"
    i64 = np.iinfo(np.int64)
    bk = np.array([0, i64.min, i64.max, -1, 0, i64.min, 1, i64.max], np.int64)
    pk = np.array([i64.min, 0, 5, -1, i64.max, i64.min, 1, 2], np.int64)
    ob, op = oracle.inner_join(bk, pk)
    cases["extreme_keys"] = dict(bk=bk, pk=pk, bv=np.ones(len(bk), bool), pv=np.ones(len(pk), bool), ob=ob, op=op)
    flat = {}
    for name, d in cases.items():
        for k, v in d.items():
            flat[f"{name}__{k}"] = v
    return flat


def main():
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **oracle_vectors())
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
