#!/usr/bin/env python3
"""Repeated single-read sorts (P = 1) with lsb_verify after each: a check that
the look-back never yields wrong offsets, e.g. with several processes sharing
one GPU (run two copies at once).

    python tools/stress_onesweep.py --n 67108864 --iters 20
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--dist", choices=("uniform", "zipf"), default="uniform")  # zipf: split stage
    a = ap.parse_args()
    bad = 0
    with lsbsort.World(a.n, ranks=1) as w:
        for i in range(a.iters):
            w.generate(a.dist)
            try:
                w.my_sort()
                w.sync()
                ok, first = w.verify()
            except lsbsort.LsbError as e:
                print(f"{a.tag} iter {i}: {e}", flush=True)
                ok, first = False, -2
            if not ok:
                bad += 1
                print(f"{a.tag} iter {i}: verify failed at {first}", flush=True)
    print(f"{a.tag} done: {bad} of {a.iters} sorts wrong", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
