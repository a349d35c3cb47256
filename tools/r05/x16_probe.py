"""The forced 16-bit exchange through a world-of-one RCCL communicator (the
bench's x16 extra) at one size and slice setting: verify result and first
bad index.  (development probe, round 5)

    python3 tools/r05/x16_probe.py LG SLICES P2P SELF
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402

lg, slices, p2p, self_coll = (int(x) for x in sys.argv[1:5])
n = 1 << lg
w = lsbsort.World.rank(n, 1, 0, 0, lsbsort.get_unique_id(), radix_bits=16)
w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
w.set_option(lsbsort.OPT_EXCHANGE_SELF, self_coll)
w.set_option(lsbsort.OPT_EXCHANGE_P2P, p2p)
if slices:
    w.set_option(lsbsort.OPT_EXCHANGE_SLICES, slices)
w.generate()
w.sync()
t0 = time.perf_counter()
w.my_sort()
w.sync()
ms = (time.perf_counter() - t0) * 1e3
ok, bad = w.verify()
print(json.dumps({"lg": lg, "slices": slices, "p2p": p2p, "self": self_coll,
                  "alloc": os.environ.get("LSB_RECORD_ALLOC", "vmm"), "ms": round(ms, 1),
                  "verified": ok, "first_bad": bad}), flush=True)
w.close()
