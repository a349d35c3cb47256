#!/usr/bin/env python3
"""Context creation time with and without the placement probe.

Each form in a fresh process: lsb_create for 2^30 records on one GPU, timed
around World(...) (the first sort's R placement is not in it), then the
placement the probe kept.  Forms alternate over ROUNDS rounds.
CREATE_TIMES=k: k contexts one after the other in each process (the first
also loads the library's code object).

    python tools/r05/create_time.py [ROUNDS=3] [N=2^30]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(n, times=1):
    sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
    import lsbsort
    lsbsort.device_memory(0)  # load the library and start the runtime first
    out = {}
    for k in range(times):
        # the first context of a process also pays for loading the library's
        # code object (its first kernel launch); later ones do not
        t0 = time.perf_counter()
        w = lsbsort.World(n, ranks=1)
        dt = time.perf_counter() - t0
        key = "create_s" if k == 0 else "create%d_s" % (k + 1)
        out[key] = round(dt, 4)
        out["placement" if k == 0 else "placement%d" % (k + 1)] = w.placement()
        w.close()
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(int(sys.argv[2]), int(os.environ.get("CREATE_TIMES", "1")))
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
