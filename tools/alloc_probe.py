#!/usr/bin/env python3
"""Does where a context's record buffers land change the pass speed?
(development probe; DESIGN.md §4 box-to-box spread)

Several contexts of 2^LG records are created one after another in one
process, each kept alive while the next is made, and each sorts the PCG
input REPS times; the per-pass k_onesweep times (lsb_get_pass_stats) show
whether the first buffers allocated in a fresh process run slower than later
ones.

    python tools/alloc_probe.py [LG] [CONTEXTS] [REPS]

LSB_PLACEMENT_CANDIDATES=2 allocates A and B as they come; the default (8)
picks them among 8 candidates by a timed pass (lsb_get_placement).

(A build whose record buffers came from hipExtMallocWithFlags(...,
hipDeviceMallocContiguous) ran every pass ~48 % slower, 10.3-10.9 ms:
profiles/ab/r03_alloc_contig.log; not kept.)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 30
ctxs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n = 1 << lg
# LSB_PICKS="best,worst,...": the placement pick of each context in turn
# (LSB_PLACEMENT_PICK: does the probe's choice predict the pass times?)
picks = [p for p in os.environ.get("LSB_PICKS", "").split(",") if p]
worlds = []
for c in range(ctxs):
    if picks:
        os.environ["LSB_PLACEMENT_PICK"] = picks[c % len(picks)]
    w = lsbsort.World(n, ranks=1, radix_bits=8)
    worlds.append(w)
    # LSB_PROBE_HYBRID=1: the hybrid local sort (passes A -> B -> R ...: the
    # third record buffer's pairs; R is allocated at its first sort)
    w.set_option(lsbsort.OPT_HYBRID, int(os.environ.get("LSB_PROBE_HYBRID", "0")))
    w.generate()
    w.my_sort()  # warm-up (allocates the look-back rows)
    w.sync()
    for r in range(reps):
        w.generate()
        w.sync()
        w.reset_kernel_stats()
        w.set_timing(True)
        t0 = time.perf_counter()
        w.my_sort()
        w.sync()
        ms = (time.perf_counter() - t0) * 1e3
        passes = [round(p["ms_scatter"], 3) for p in w.pass_stats()]
        w.set_timing(False)
        print(json.dumps({"context": c, "rep": r, "ms": round(ms, 2), "passes": passes}), flush=True)
    ok, _ = w.verify()
    print(json.dumps({"context": c, "verified": ok, "placement": w.placement(),
                      "pick": os.environ.get("LSB_PLACEMENT_PICK", "best"),
                      "env_candidates": os.environ.get("LSB_PLACEMENT_CANDIDATES", "default")}), flush=True)
for w in worlds:
    w.close()
