#!/bin/bash
# tools/kbench/merge2 timings, then its FETCH_SIZE / WRITE_SIZE per kernel variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/m2pmc
mkdir -p $O
timeout -k 10 120 $R/tools/kbench/merge2 29 > $O/time.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/tools/kbench/merge2 29 pmc > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $R/tools/kbench/merge2 29 pmc > $O/write.log 2>&1 || exit 1
cat $O/time.log
python3 - <<'PY'
import csv, glob, os, collections
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/m2pmc"
def agg(kind, counter):
    f = glob.glob(f"{O}/{kind}/**/run_counter_collection.csv", recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            d[(r["Kernel_Name"][:90], r["Grid_Size"] if "Grid_Size" in r else "")].append(float(r["Counter_Value"]))
    return d
fe, wr = agg("fetch", "FETCH_SIZE"), agg("write", "WRITE_SIZE")
for k in fe:
    f = sum(fe[k]) / len(fe[k]) * 1024 / 1e9
    w = sum(wr.get(k, [0])) / max(1, len(wr.get(k, [0]))) * 1024 / 1e9
    print(f"{k[0]:90s} {k[1]:>8s} n={len(fe[k]):2d} FETCH={f:7.2f} GB (x2 {2*f:7.2f})  WRITE={w:7.2f} GB")
PY
