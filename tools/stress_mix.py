#!/usr/bin/env python3
"""Randomised stress of every sort form on one GPU: each iteration draws a
size (1 .. 2^27 records, log-uniform, ragged), a rank count (P logical ranks,
device-copy exchange), an exchange digit width (8, 16 or 64), a key
distribution and a stage form, sorts, and checks lsb_verify and
checkSorted.  Runs until --seconds have passed; one line per iteration.

    python tools/stress_mix.py --seconds 240 --seed 1
"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-log2", type=int, default=27)
    a = ap.parse_args()
    rng = random.Random(a.seed)
    t_end = time.time() + a.seconds
    it = bad = 0
    while time.time() < t_end:
        n = int(2 ** rng.uniform(0, a.max_log2)) + rng.randrange(0, 4096)
        P = rng.choice((1, 1, 2, 3, 8))
        bits = rng.choice((8, 16, 64))
        dist = rng.choice(("uniform", "zipf"))
        split = rng.choice((0, 1, 2))
        desc = f"iter {it}: n={n} P={P} bits={bits} dist={dist} split={split}"
        try:
            with lsbsort.World(n, ranks=P, radix_bits=bits) as w:
                w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, split)
                w.generate(dist)
                w.my_sort()
                ok, first = w.verify()
                srt = w.check_sorted()
        except lsbsort.LsbError as e:
            ok, first, srt = False, str(e), False
        if not (ok and srt):
            bad += 1
        print(f"{desc} verify={ok} first_bad={first} sorted={srt}", flush=True)
        it += 1
    print(f"done: {bad} of {it} sorts wrong", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
