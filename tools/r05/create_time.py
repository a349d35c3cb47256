#!/usr/bin/env python3
"""Context creation time with and without the placement probe.

Each form in a fresh process: lsb_create for 2^30 records on one GPU, timed
around World(...) (the first sort's R placement is not in it), then the
placement the probe kept.  Forms alternate over ROUNDS rounds.

    python tools/r05/create_time.py [ROUNDS=3] [N=2^30]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(n):
    sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
    import lsbsort
    lsbsort.device_memory(0)  # load the library and start the runtime first
    t0 = time.perf_counter()
    w = lsbsort.World(n, ranks=1)
    dt = time.perf_counter() - t0
    print(json.dumps({"create_s": round(dt, 4), "placement": w.placement()}))
    w.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(int(sys.argv[2]))
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
    forms = [("off", "0"), ("default", None)]
    for k in range(rounds):
        for name, val in (forms if k % 2 == 0 else forms[::-1]):
            env = dict(os.environ)
            env.pop("LSB_PLACEMENT_CANDIDATES", None)
            if val is not None:
                env["LSB_PLACEMENT_CANDIDATES"] = val
            out = subprocess.run([sys.executable, __file__, "--child", str(n)], env=env, capture_output=True,
                                 text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            print(name, k, line[-1] if line else out.stderr[-2000:], flush=True)
            if out.returncode != 0:
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
