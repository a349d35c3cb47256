"""Per-kernel time of one single-rank sort (development tool).

python tools/digit_probe.py [log2 n]  -> ms per sort by kernel, and verify.
Used for the kernel-variant A/B runs recorded in DESIGN.md §5.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-lsb_amd"))
import lsbsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 30
DIST = os.environ.get("LSB_DIST", "uniform")  # uniform | zipf
n = 1 << lg
# LSB_RADIX_BITS=16 and LSB_FORCE_EXCHANGE=1: the per-digit exchange path at
# P = 1 (counts, plan, k_place), as tools/exchange_profile.py, with LSB_DIST keys.
w = lsbsort.World(n, 1, radix_bits=int(os.environ.get("LSB_RADIX_BITS", "8")))
if os.environ.get("LSB_SPLIT"):  # LSB_OPT_ONESWEEP_SPLIT: 0 auto, 1 never, 2 always
    w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, int(os.environ["LSB_SPLIT"]))
if os.environ.get("LSB_FORCE_EXCHANGE") == "1":
    w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
if os.environ.get("LSB_GATHER"):  # LSB_OPT_EXCHANGE_GATHER: 0 places every exchange
    w.set_option(lsbsort.OPT_EXCHANGE_GATHER, int(os.environ["LSB_GATHER"]))
# LSB_PASSES=reduce-scan: count + scan + scatter per pass instead of single-read passes
w.set_option(lsbsort.OPT_ONESWEEP, 0 if os.environ.get("LSB_PASSES") == "reduce-scan" else 1)
# LSB_PASSES=hybrid: k top-byte passes + the segmented local sort (LSB_OPT_HYBRID)
w.set_option(lsbsort.OPT_HYBRID, {"hybrid": 1, "hybrid-segsort": 2}.get(os.environ.get("LSB_PASSES", ""), 0))
w.set_timing(True)
names = ["upsweep", "scan", "scatter", "exchange", "wire", "place", "place_tail", "segsort", "sort"]
for rep in range(2):
    w.generate(DIST)
    w.my_sort()
    w.sync()
    w.generate(DIST)
    w.reset_kernel_stats()
    t0 = time.perf_counter()
    w.my_sort()
    w.sync()
    wall = (time.perf_counter() - t0) * 1e3
    st = w.kernel_stats()
    ok = w.verify()
    parts = " ".join(f"{k}={st[k][1]:.2f}ms/{st[k][0]}" for k in names if st[k][0])
    print(f"n=2^{lg} wall={wall:.2f}ms {n / wall / 1e3:.0f} Melem/s verify={ok} {parts}", flush=True)
