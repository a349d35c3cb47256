#!/bin/bash
# Kernel resources of RCCL's kernels next to ours (world-of-one RCCL context).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rk
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/rk -o run -- python3 $R/tools/rccl_kernels.py 64 > $R/gpurun_out/rk/log 2>&1 || { tail -20 $R/gpurun_out/rk/log; exit 1; }
python3 - <<'PY'
import csv, glob, os
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/rk/**/run_kernel_trace.csv", recursive=True)[0]
seen = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:70]
    if k not in seen:
        seen[k] = (r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["Workgroup_Size_X"], r["Grid_Size_X"], r["Scratch_Size"])
for k, v in seen.items():
    print(f"{k:70s} lds={v[0]} vgpr={v[1]} agpr={v[2]} sgpr={v[3]} wg={v[4]} grid={v[5]} scratch={v[6]}")
PY
