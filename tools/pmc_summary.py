#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/.

Reads gpurun_out/prof/{stats,fetch,write}/ (rocprofv3 CSV; or PROF_DIR) and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_pmc.json           per-kernel avg duration and HBM bytes per launch

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, following
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE (KB) reads exactly half of a
wide (16 B/lane) coalesced stream, WRITE_SIZE (KB) is exact for 16-B stores.
The x2 was calibrated here: k_upsweep/k_scatter each stream 2^30 x 16 B =
17.18e9 B and report FETCH_SIZE = 8.39e6 KB.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


TEMPLATES = False  # --templates: keep template instances apart


def short(name):
    """Kernel base name: template instances (k_onesweep<256, 16, true> and
    <..., false>) are one kernel, averaged over all their launches (unless
    --templates: the hybrid's SEG pass is k_onesweep<..., true>)."""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0].replace("lsb::", "")
    return name if TEMPLATES else name.split("<")[0]


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def durations_of(stats_csv):
    calls, ns = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(stats_csv)):
        k = short(r["Name"])
        calls[k] += int(r["Calls"])
        ns[k] += float(r["TotalDurationNs"])
    return {k: {"calls": calls[k], "avg_ms": ns[k] / calls[k] / 1e6} for k in calls}


def main(tag, prof=os.path.join(ROOT, "gpurun_out", "prof"),
         workload="configs[1]: sort of 2^30 16-byte records per GPU, 8-bit digits, 8 passes, 1 GPU(s)",
         elems=1 << 30):
    stats_csv = os.path.join(prof, "stats", "run_kernel_stats.csv")
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    shutil.copy(stats_csv, os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
    durations = durations_of(stats_csv)
    fetch = per_kernel(os.path.join(prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write) | set(durations)):
        f, w = fetch.get(k), write.get(k)
        hbm = None if f is None or w is None else (2 * f + w) * 1024
        kernels[k] = {**durations.get(k, {}), "fetch_size_kb": f, "write_size_kb": w,
                      "hbm_bytes_per_launch": hbm}
    doc = {"tag": tag, "workload": workload, "elems_per_launch": elems,
           "method": "rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE and --pmc WRITE_SIZE runs; "
                     "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE = half of a 16B/lane stream)",
           "kernels": kernels}
    with open(os.path.join(out_dir, f"{tag}_pmc.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    # pmc_summary.py TAG [PROF_DIR [WORKLOAD]] [--templates]
    args = [a for a in sys.argv[1:] if a != "--templates"]
    TEMPLATES = len(args) < len(sys.argv) - 1
    kw = {}
    if len(args) > 1:
        kw["prof"] = args[1]
    if len(args) > 2:
        kw["workload"] = args[2]
    main(args[0] if args else "r01", **kw)
