#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel name, launches,
summed duration and the [first start, last end] span relative to the first
kernel of the window; --last K keeps the window from the K-th last launch of
--anchor (e.g. the 8 k_subhist launches of the last sort of 8 logical ranks).

    python tools/trace_summary.py gpurun_out/mt/run_kernel_trace.csv --anchor k_subhist --last 8
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default=None)
    ap.add_argument("--last", type=int, default=1)
    ap.add_argument("--detail", default=None, help="print every launch whose name contains this")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0],
                 r.get("Stream_Id", "")) for r in rows)
    if a.anchor:
        idx = [i for i, k in enumerate(ks) if a.anchor in k[2]]
        ks = ks[idx[-a.last]:]
    t0 = ks[0][0]
    agg = collections.defaultdict(lambda: [0, 0, None, 0])
    for s, e, n, _ in ks:
        g = agg[n]
        g[0] += 1
        g[1] += e - s
        g[2] = s if g[2] is None else min(g[2], s)
        g[3] = max(g[3], e)
    print(f"window {(ks[-1][1] - t0) / 1e6:.2f} ms")
    for n, g in sorted(agg.items(), key=lambda x: x[1][2]):
        print(f"{n[:56]:56s} n={g[0]:5d} sum={g[1] / 1e6:9.3f} ms avg={g[1] / g[0] / 1e3:9.1f} us "
              f"span=[{(g[2] - t0) / 1e6:8.2f}, {(g[3] - t0) / 1e6:8.2f}]")
    if a.detail:
        for s, e, n, st in ks:
            if a.detail in n:
                print(f"  {n[:30]} stream {st} {(s - t0) / 1e6:9.3f} -> {(e - t0) / 1e6:9.3f} "
                      f"({(e - s) / 1e3:.1f} us)")


if __name__ == "__main__":
    main()
