#!/usr/bin/env python3
"""Whole-key exchange (radix_bits = 64) on one GPU: P logical ranks of
--n-per-rank records each (lsb_create), HIP-event times per phase.

    python tools/merge_profile.py --ranks 8 --n-per-rank 134217728 [--bits 16]

Phases: local sort (k_subhist + k_onesweep per rank), splitter search +
device-copy all-to-all ("exchange"), merge tree ("place").  With --bits 8/16
the same world runs the per-pass exchange instead, for comparison.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--n-per-rank", type=int, default=1 << 27)
    ap.add_argument("--bits", type=int, default=64)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--slices", type=int, default=0, help="LSB_OPT_EXCHANGE_SLICES (0: default)")
    a = ap.parse_args()
    n = a.ranks * a.n_per_rank
    with lsbsort.World(n, ranks=a.ranks, radix_bits=a.bits) as w:
        w.set_timing(True)
        if a.slices:
            w.set_option(lsbsort.OPT_EXCHANGE_SLICES, a.slices)
        for rep in range(a.reps + 1):
            w.generate(a.dist)
            w.reset_kernel_stats()
            w.sync()
            t0 = time.perf_counter()
            w.my_sort()
            w.sync()
            ms = (time.perf_counter() - t0) * 1e3
            st = w.kernel_stats()
            if rep == 0:
                continue  # warm-up (allocations)
            parts = " ".join(f"{k}={v[1]:.2f}ms/{v[0]}" for k, v in st.items() if v[0])
            print(f"P={a.ranks} n={n} bits={a.bits} sort {ms:.2f} ms wall  {parts}", flush=True)
        ok, bad = w.verify()
        print(f"verify ok={ok} first_bad={bad}", flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
