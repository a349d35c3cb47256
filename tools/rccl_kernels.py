#!/usr/bin/env python3
"""World-of-one RCCL context running the whole-key exchange: run under
rocprofv3 --kernel-trace to see the resources (LDS, VGPRs, grid) of the
RCCL kernels that share the GPU with the merge kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402

n = 1 << 22
w = lsbsort.World.rank(n, 1, 0, 0, lsbsort.get_unique_id(), radix_bits=int(sys.argv[1]) if len(sys.argv) > 1 else 64)
try:
    w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
    for _ in range(2):
        w.generate()
        w.barrier()
        w.my_sort()
        w.barrier()
    print("verify", w.verify(), flush=True)
finally:
    w.close()
