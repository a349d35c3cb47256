#!/usr/bin/env python3
"""Effective GPU clock of every profiled launch (tools/gpu_round.sh `clock`):
GRBM_GUI_ACTIVE counts GPU-active cycles of the graphics clock over a
dispatch, so cycles / duration is the clock the launch ran at; GRBM_COUNT is
the free-running count over the same window.  In dispatch order, so a clock
that sinks as the box warms shows.

    python tools/clock_summary.py gpurun_out/<tag>/clock
"""
import collections
import csv
import os
import sys

root = sys.argv[1]
rows = []
for d, _, files in os.walk(root):
    for f in files:
        if f.endswith("counter_collection.csv"):
            rows += list(csv.DictReader(open(os.path.join(d, f))))
per = collections.OrderedDict()
for r in rows:
    k = int(r["Dispatch_Id"])
    e = per.setdefault(k, {"name": r["Kernel_Name"][:40], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(per):
    e = per[k]
    act = e.get("GRBM_GUI_ACTIVE", 0.0)
    print(f"dispatch {k:5d} {e['name']:40s} {e['ns'] / 1e6:8.3f} ms  GUI_ACTIVE {act:.4g}  "
          f"clock {act / e['ns'] * 1e3 if e['ns'] else 0:.0f} MHz  GRBM_COUNT {e.get('GRBM_COUNT', 0):.4g}")
