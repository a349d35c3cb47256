#!/bin/bash
# Counters behind the buffer-placement spread: tools/kbench/allocbw
# (4 fresh 16 GiB buffers: pure read, pure write, LSD-pattern copies between
# every pair) under rocprofv3 --pmc, one counter set per process.  Each
# process allocates its own buffers, so a pass's counters are read against the
# timings that same process printed (its .log), not across passes.
#   TAG=r04_pmc SETS="tcc utcl" bash tools/allocbw_counters.sh
# Output: gpurun_out/$TAG/<set>.log (allocbw's own lines) and <set>/ (csv).
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-allocpmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BIN=$REPO/tools/kbench/allocbw
for s in ${SETS:-list}; do
  case $s in
    list) timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true; continue ;;
    tcc) C="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_STALL_sum" ;;
    tccdram) C="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" ;;
    utcl) C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum" ;;
    ta) C="TA_BUSY_max TA_FLAT_WRITE_WAVEFRONTS_sum" ;;
    *) echo "unknown set $s"; exit 2 ;;
  esac
  # a counter this ROCm does not know ends the pass, not the script
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/$s" -o run -- \
    "$BIN" 4 30 3 > "$OUT/$s.log" 2>&1 || echo "pass $s failed: $?" >> "$OUT/$s.log"
done
