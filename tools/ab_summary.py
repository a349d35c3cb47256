#!/usr/bin/env python3
"""Median sort / scatter ms per build from gpurun_out/ab.log (tools/ab.sh)."""
import collections
import re
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"
sort, scat, lib = collections.defaultdict(list), collections.defaultdict(list), None
place = collections.defaultdict(list)
seg = collections.defaultdict(list)
for line in open(path):
    if line.startswith("lib="):
        lib = line.strip()[4:]
    m = re.search(r"wall=([\d.]+)ms.*scatter=([\d.]+)ms", line)
    if m and lib:
        sort[lib].append(float(m.group(1)))
        scat[lib].append(float(m.group(2)))
        p = re.search(r"place=([\d.]+)ms", line)
        if p:
            place[lib].append(float(p.group(1)))
        q = re.search(r"segsort=([\d.]+)ms", line)
        if q:
            seg[lib].append(float(q.group(1)))
for k in sort:
    print(f"{k:32s} sort {statistics.median(sort[k]):7.2f} ms (min {min(sort[k]):.2f})  "
          f"scatter {statistics.median(scat[k]):7.2f} ms  n={len(sort[k])}"
          + (f"  place {statistics.median(place[k]):7.2f} ms" if place[k] else "")
          + (f"  segsort {statistics.median(seg[k]):7.2f} ms" if seg[k] else ""))
