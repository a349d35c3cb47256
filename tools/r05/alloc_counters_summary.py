"""Per process of tools/r05/alloc_counters.sh: the mean k_onesweep launch time
and each counter per launch (rocprofv3 counter_collection csv), beside the
pass times the process printed.

    python3 tools/r05/alloc_counters_summary.py gpurun_out/r05_allocpmc
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
for d in sorted(x for x in glob.glob(os.path.join(root, "*_*")) if os.path.isdir(x)):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    per = collections.defaultdict(dict)  # dispatch -> counter -> value
    dur = {}
    for row in csv.DictReader(open(files[0])):
        if "k_onesweep<" not in row["Kernel_Name"]:
            continue
        k = row["Dispatch_Id"]
        # per-instance counters come as several rows of one name: keep their
        # spread (max / mean over instances) beside the sum
        name = row["Counter_Name"]
        per[k].setdefault(name, []).append(float(row["Counter_Value"]))
        dur[k] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    if not per:
        continue
    names = sorted({c for v in per.values() for c in v})
    mean = {c: sum(sum(v.get(c, [0.0])) for v in per.values()) / len(per) for c in names}
    spread = {c: round(sum(max(v[c]) / (sum(v[c]) / len(v[c])) for v in per.values() if c in v and sum(v[c]) > 0)
                       / len(per), 3) for c in names if any(len(v.get(c, [])) > 1 for v in per.values())}
    log = d + ".log"
    passes = [json.loads(l)["passes"] for l in open(log) if l.startswith("{") and '"passes"' in l]
    flat = [p for ps in passes for p in ps if p > 0]
    print(json.dumps({"run": os.path.basename(d), "launches": len(per),
                      "launch_ms_under_profiler": round(sum(dur.values()) / len(dur), 3),
                      "pass_ms_printed": round(sum(flat) / len(flat), 3) if flat else None,
                      "per_launch": {c: round(v) for c, v in mean.items()},
                      "instances_max_over_mean": spread or None}))
