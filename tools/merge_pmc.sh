#!/bin/bash
# HBM bytes of the whole-key exchange's merge kernels (rocprofv3 PMC, one
# counter per pass, --kernel-trace only), P = 2 logical ranks on one GPU,
# 2 x 2^29 records, 2 sorts (tools/merge_profile.py --reps 1).  Writes
# gpurun_out/mpmc/{stats,fetch,write} and prints per-kernel bytes vs the
# algorithmic 32 B per record per merge level.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="$R/tools/merge_profile.py --ranks 2 --n-per-rank 536870912 --reps 1"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $P > $O/stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $P > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $P > $O/write.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, os, collections
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/mpmc"
def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("lsb::", "").split("<")[0]
def tot(kind, counter):
    f = glob.glob(f"{O}/{kind}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])] += float(r["Counter_Value"]); cnt[short(r["Kernel_Name"])] += 1
    return agg, cnt
fe, nf = tot("fetch", "FETCH_SIZE")
wr, nw = tot("write", "WRITE_SIZE")
n, sorts, levels = 2 * 536870912, 2, 1
alg = 32.0 * n * sorts * levels
for k in ("k_merge2", "k_merge_path", "k_onesweep"):
    b = (2 * fe.get(k, 0) + wr.get(k, 0)) * 1024
    print(f"{k:14s} launches={nf.get(k,0):4d} hbm={b/1e9:8.2f} GB  fetch={2*fe.get(k,0)*1024/1e9:8.2f} write={wr.get(k,0)*1024/1e9:8.2f}" +
          (f"  algorithmic={alg/1e9:.2f} GB ratio={b/alg:.3f}" if k == "k_merge2" else ""))
PY
