#!/usr/bin/env python3
"""The wrong answer of test_world_of_one_large_calls[28-8-1] (round 6): a
world-of-one RCCL context, 2^lg records, `bits`-bit digits, the exchange
forced with the self segment through ncclAllToAllv in `slices` slices.  Each
repetition sorts a fresh context and, when lsb_verify fails, compares with
numpy's stable sort: how many records differ, where (in 2^26-record = 1 GiB
blocks, the size of one cut RCCL call), and whether the output is still a
permutation of the input (records misplaced) or not (records lost).

    python tools/r06/large_call_probe.py [lg=28] [bits=8] [slices=1] [reps=3]
    (env: LSB_RCCL_CALL_U64, OPTs via LP_GATHER=0/1, LP_P2P=0/1;
     LP_LOOPBACK=1: a loopback context; LP_NOFORCE=1: no forced exchange;
     LP_SEED=1: other random input per repetition)
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-lsb_amd"))
import lsbsort  # noqa: E402

lg, bits, slices, reps = (int(x) for x in (sys.argv[1:] + ["28", "8", "1", "3"][len(sys.argv) - 1:])[:4])
n = 1 << lg
for rep in range(reps):
    if os.environ.get("LP_LOOPBACK"):  # a loopback context: the same sort, no RCCL
        w = lsbsort.World(n, ranks=1, radix_bits=bits)
    else:
        w = lsbsort.World.rank(n, 1, 0, 0, lsbsort.get_unique_id(), radix_bits=bits)
    try:
        w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 0 if os.environ.get("LP_NOFORCE") else 1)
        w.set_option(lsbsort.OPT_EXCHANGE_SELF, 1)
        if slices:
            w.set_option(lsbsort.OPT_EXCHANGE_SLICES, slices)
        if os.environ.get("LP_P2P"):
            w.set_option(lsbsort.OPT_EXCHANGE_P2P, int(os.environ["LP_P2P"]))
        if os.environ.get("LP_GATHER"):
            w.set_option(lsbsort.OPT_EXCHANGE_GATHER, int(os.environ["LP_GATHER"]))
        if os.environ.get("LP_SEED"):  # other input per repetition (generate() is pcg64(rank) every time)
            rng = np.random.default_rng(1000 + rep)
            arr = np.empty(n, dtype=lsbsort.ELEM_DTYPE)
            arr["key"] = rng.integers(0, np.iinfo(np.uint64).max, size=n, dtype=np.uint64, endpoint=True)
            arr["val"] = np.arange(n, dtype=np.uint64)
            w.copy_in(0, arr)
            keys_in = arr["key"].copy()
            del arr
        else:
            w.generate()
        inp = w.copy_out(0)
        w.my_sort()
        w.sync()
        if os.environ.get("LP_SEED"):  # lsb_verify checks against generate()'s input: check on the host
            out = w.copy_out(0)
            k, v = out["key"], out["val"]
            ok = bool((v < n).all()) and bool(np.bincount(v.astype(np.int64), minlength=n).max() == 1)
            ok = ok and bool(np.array_equal(k, keys_in[v.astype(np.int64)]))  # every key with its value
            step = (k[1:] > k[:-1]) | ((k[1:] == k[:-1]) & (v[1:] > v[:-1]))  # stable order
            bad = np.nonzero(~step)[0]
            first = int(bad[0]) if bad.size else -1
            ok = ok and first < 0
            del out, k, v, step
        else:
            ok, first = w.verify()
        row = {"rep": rep, "lg": lg, "bits": bits, "slices": slices, "call_u64": os.environ.get("LSB_RCCL_CALL_U64"),
               "gather": os.environ.get("LP_GATHER"), "p2p": os.environ.get("LP_P2P"), "loopback": bool(os.environ.get("LP_LOOPBACK")),
               "noforce": bool(os.environ.get("LP_NOFORCE")), "seeded": bool(os.environ.get("LP_SEED")),
               "rccl_vmm": os.environ.get("LSB_RCCL_VMM"), "rccl_sync": os.environ.get("LSB_RCCL_SYNC"), "verified": ok, "first_bad": first,
               "exchanges": w.exchange_stats()["exchanges"], "calls": w.exchange_stats()["calls"]}
        print(json.dumps(row), flush=True)
        if not ok and not os.environ.get("LP_QUICK"):
            # (progress lines: the analysis of 2^28 records takes a while)
            out = w.copy_out(0)
            print("analysing", flush=True)
            want = inp[np.argsort(inp["key"], kind="stable")]
            print("reference sorted", flush=True)
            diff = np.nonzero((out["key"] != want["key"]) | (out["val"] != want["val"]))[0]
            blk = np.bincount(diff >> 26, minlength=n >> 26) if diff.size else []
            keys_same = bool(np.array_equal(np.sort(out["key"]), want["key"]))
            vals = np.sort(out["val"])
            vals_perm = bool(np.array_equal(vals, np.sort(inp["val"])))
            sorted_keys = bool(np.all(out["key"][1:] >= out["key"][:-1]))
            print(json.dumps({"rep": rep, "wrong": int(diff.size), "first": int(diff[0]) if diff.size else -1,
                              "last": int(diff[-1]) if diff.size else -1, "per_gib_block": [int(x) for x in blk],
                              "keys_are_the_inputs": keys_same, "vals_are_a_permutation": vals_perm,
                              "keys_sorted": sorted_keys,
                              "head_out": [[int(a), int(b)] for a, b in out[:4].tolist()],
                              "head_want": [[int(a), int(b)] for a, b in want[:4].tolist()]}), flush=True)
    finally:
        w.close()
