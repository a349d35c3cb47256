#!/usr/bin/env python3
"""Device memory and record-buffer addresses over successive contexts of one
process (2^28 records, placement probe on): does a released VMM buffer give
its memory back, and does a later buffer get its addresses?  Run with
LSB_VMM_TRACE=1 and LSB_VMM_VA_MODE=retire|reuse|hint."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-lsb_amd"))
import lsbsort  # noqa: E402

n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 28
for k in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    with lsbsort.World(n, ranks=1, radix_bits=16) as w:
        w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        ok = w.verify()[0]
    free, total = lsbsort.device_memory(0)
    print(f"context {k}: verified={ok} free={free / 2**30:.1f} GiB of {total / 2**30:.1f}", flush=True)
