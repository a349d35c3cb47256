#!/usr/bin/env python3
"""Summarise tools/alloc_probe.py logs (LSB_PICKS / LSB_PLACEMENT_CANDIDATES
runs): per context the placement choice (probe ms of the kept
pair, the first pair, the worst pair) against the mean / min / max
k_onesweep pass of its sorts.

    python tools/pick_summary.py gpurun_out/r04_v4/pick.log [...]
"""
import json
import sys


def contexts(path):
    cur = []
    for line in open(path):
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if "passes" in r:
            cur.extend(r["passes"])
        elif "placement" in r:
            yield r, cur
            cur = []


for path in sys.argv[1:]:
    print(f"== {path}")
    for r, passes in contexts(path):
        p = r["placement"]
        m = sum(passes) / len(passes) if passes else 0.0
        print(f"  pick={r.get('pick', '-'):5s} cand={p['candidates']} kept={p['chosen_ms']:.3f} "
              f"first={p['first_pair_ms']:.3f} worst={p['worst_ms']:.3f} | passes mean={m:.3f} "
              f"min={min(passes):.3f} max={max(passes):.3f} verified={r['verified']}")
