#!/usr/bin/env python3
"""Summarise a tools/sq_counters.sh run (two rocprofv3 --pmc passes over
tools/digit_probe.py) into profiles/<tag>_sq.json: per kernel, the average
of every SQ counter per launch, plus the derived shares.

    python tools/sq_summary.py r02_v2 gpurun_out/sq_r02v2

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count quad-cycles
(MI355X_MICROARCH.md); SQ_LDS_BANK_CONFLICT and SQ_LDS_IDX_ACTIVE count LDS
cycles, so their ratio is the conflicted share of LDS-array time.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("lsb::", "")
    return name.split("(")[0]


def main(tag, src):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("a", "b"):
        path = os.path.join(src, p, "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in agg.items():
        if not k.startswith("k_"):
            continue
        c = {n: sum(v) / len(v) for n, v in d.items()}
        e = dict(c)
        if c.get("SQ_WAVE_CYCLES"):
            w = c["SQ_WAVE_CYCLES"]
            e["share_wait_any"] = c.get("SQ_WAIT_ANY", 0) / w
            e["share_active_inst"] = c.get("SQ_ACTIVE_INST_ANY", 0) / w
            e["share_wait_inst_any"] = c.get("SQ_WAIT_INST_ANY", 0) / w
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("SQ_INSTS_LDS"):
            e["lds_cycles_per_inst"] = c.get("SQ_LDS_IDX_ACTIVE", 0) / c["SQ_INSTS_LDS"]
            e["conflict_cycles_per_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
        out[k] = e
    dst = os.path.join(ROOT, "profiles", f"{tag}_sq.json")
    with open(dst, "w") as f:
        json.dump({"source": "tools/sq_counters.sh (digit_probe.py 28: one sort of 2^28 records, "
                             "k_onesweep launches averaged per template instance)",
                   "kernels": out}, f, indent=1, sort_keys=True)
    print(dst)
    for k, e in out.items():
        if "lds_conflict_share" in e:
            print(f"{k:55s} LDS conflict share {e['lds_conflict_share']:.3f}  "
                  f"conflict cycles/LDS inst {e['conflict_cycles_per_inst']:.2f}  "
                  f"wait {e.get('share_wait_any', 0):.2f} active {e.get('share_active_inst', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
