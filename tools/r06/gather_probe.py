#!/usr/bin/env python3
"""Per-pass scatter ms of the 16-bit per-digit sort at P = 1 with the
exchange forced (loopback: the self segment stays in A), gathered
(LSB_OPT_EXCHANGE_GATHER = 1, the default) against placed (0), and the same
sort without the exchange: what a gathered low-byte pass costs against a
plain one (7.50 vs 6.84 ms in the x16 rows).

    python tools/r06/gather_probe.py [log2 n = 30] [sorts = 3]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-lsb_amd"))
import lsbsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 30
sorts = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << lg
# GP_FORMS="gather": only these forms (A/B of library builds: LSB_LIBRARY)
forms = os.environ.get("GP_FORMS", "gather placed plain gather placed plain").split()
for form in forms:
    with lsbsort.World(n, 1, radix_bits=16) as w:
        if form != "plain":
            w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
            w.set_option(lsbsort.OPT_EXCHANGE_GATHER, 1 if form == "gather" else 0)
        w.set_timing(True)
        w.generate()
        w.my_sort()
        w.sync()
        rows = []
        for _ in range(sorts):
            w.generate()
            w.reset_kernel_stats()
            w.my_sort()
            w.sync()
            rows.append([round(p["ms_scatter"], 3) for p in w.pass_stats()])
        ok = w.verify()[0]
    avg = [round(sum(r[i] for r in rows) / len(rows), 3) for i in range(len(rows[0]))]
    print(json.dumps({"form": form, "verified": ok, "scatter_ms_per_pass": avg, "sum": round(sum(avg), 2)}),
          flush=True)
