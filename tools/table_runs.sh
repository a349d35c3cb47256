#!/bin/bash
# The DESIGN.md §4 bench table on one box: C2 default, reduce-then-scan,
# Zipf keys, 16-bit digits, 2^32 records, the hybrid local sort at 2^30,
# with Zipf keys and at 2^32, and (round 5) the 16-bit exchange forced through
# a world-of-one RCCL communicator, uniform and Zipf (bench.py lines in
# gpurun_out/${TABLE:-table}.log).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
T=gpurun_out/${TABLE:-table}.log
: > $T
for args in "" "--passes reduce-scan" "--dist zipf" "--radix-bits 16" "--n-per-gpu 4294967296 --steps 3 --warmup 1" \
    "--passes hybrid" "--passes hybrid --dist zipf" "--passes hybrid --n-per-gpu 4294967296 --steps 3 --warmup 1" \
    "--force-exchange --radix-bits 16" "--force-exchange --radix-bits 16 --dist zipf"; do
  echo "args: $args" >> $T
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --no-extras $args >> $T 2>&1 || exit 1
done
export T
python3 - <<'PY'
import json
import os
for line in open(os.environ["T"]):
    if line.startswith("args:"):
        a = line.strip()
    elif line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        k = d.get("kernel_ms_per_step", {})
        print(f"{a:50s} {d['value']:10.1f} Melem/s {d['ms_per_step']:8.2f} ms  {r['kernel']} {r['avg_launch_ms']:.3f} ms "
              f"frac {r['frac']:.3f} verified {d['verified']} passes {d['config'].get('local_passes')} "
              f"segsort {k.get('segsort', 0):.2f} ms")
PY
