#!/bin/bash
# The third record buffer R (hybrid, exchanges): allocated at its first use
# (default), with A and B at creation (LSB_ALLOC_R_EARLY=1), and the pieces of
# A, B (and R) created interleaved (LSB_VMM_ORDER=interleave).  Fresh
# processes of tools/alloc_probe.py; hybrid sorts use R.
set -u
O=gpurun_out/${TAG:-r05_rsweep}
mkdir -p $O
ap() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/alloc_probe.py 30 1 3 > $O/ap_$name.log 2>&1 || exit 1
  echo "$name: $(python3 tools/r05/ap_summary.py $O/ap_$name.log)"
}
for i in 1 2 3; do ap hyb_default$i LSB_PROBE_HYBRID=1; done
for i in 1 2 3; do ap hyb_early$i LSB_PROBE_HYBRID=1 LSB_ALLOC_R_EARLY=1; done
for i in 1 2 3; do ap hyb_early_il$i LSB_PROBE_HYBRID=1 LSB_ALLOC_R_EARLY=1 LSB_VMM_ORDER=interleave; done
for i in 1 2; do ap lsd_il$i LSB_VMM_ORDER=interleave; done
for i in 1 2; do ap lsd_default$i; done
