#!/usr/bin/env python3
"""Per-kernel times of the exchange path on one GPU (development tool).

P logical ranks share the GPU (lsb_create), so this times the same kernels
and plan as the multi-GPU path (count, place, 16-bit counts) with the
all-to-all done by device copies; P = 1 with --force runs the exchange
path against itself.  `gather`: LSB_OPT_EXCHANGE_GATHER (count-only
placements and gathered passes) on or off.

    python tools/exchange_profile.py  # a fixed set of (n, P, bits) cases
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402

CASES = [  # (n, P, bits, force_exchange, single-read local passes, gathered passes)
    (1 << 30, 1, 8, False, 1, 1),
    (1 << 30, 1, 8, True, 1, 1),
    (1 << 30, 1, 8, True, 1, 0),
    (1 << 30, 1, 8, True, 0, 0),
    (1 << 30, 1, 16, True, 1, 1),
    (1 << 30, 1, 16, True, 1, 0),
    (1 << 30, 1, 16, True, 0, 0),
    (1 << 30, 2, 16, False, 1, 1),
    (1 << 30, 2, 16, False, 1, 0),
    (1 << 30, 4, 16, False, 1, 1),
    (1 << 30, 4, 16, False, 1, 0),
    (1 << 30, 8, 16, False, 1, 1),
]


def run(n, P, bits, force, onesweep, gather, steps=2):
    with lsbsort.World(n, ranks=P, radix_bits=bits) as w:
        w.set_option(lsbsort.OPT_ONESWEEP, onesweep)
        w.set_option(lsbsort.OPT_EXCHANGE_GATHER, gather)
        if force:
            w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()  # warm-up
        w.sync()
        w.reset_kernel_stats()
        w.set_timing(True)
        t = 0.0
        for _ in range(steps):
            w.generate()
            w.sync()
            t0 = time.perf_counter()
            w.my_sort()
            w.sync()
            t += time.perf_counter() - t0
        st = w.kernel_stats()
        ok, _ = w.verify()
    per = {k: round(v[1] / steps, 3) for k, v in st.items() if v[0]}
    return {"n": n, "P": P, "bits": bits, "force_exchange": force, "onesweep": onesweep,
            "gather": gather, "ms_per_sort": round(t / steps * 1e3, 2),
            "melem_s": round(n / (t / steps) / 1e6, 1), "kernel_ms_per_sort": per, "verified": ok}


if __name__ == "__main__":
    for c in CASES:
        print(json.dumps(run(*c)), flush=True)
