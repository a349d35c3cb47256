#!/bin/bash
# Counters behind the record-buffer allocation: the sort
# of 2^30 records (tools/alloc_probe.py, one context, 2 sorts) in fresh
# processes, hipMalloc'd buffers (LSB_RECORD_ALLOC=malloc, several processes:
# the driver's placement varies) against 1 GiB VMM pieces, one counter set
# per process (UTCL1 translation; L2 -> fabric requests), each process's own
# per-pass times beside its counters.
# Output: gpurun_out/r05_allocpmc/<mode>_<set>/ (csv) and .log; avail.txt.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05_allocpmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
utcl="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum"
tcc="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_STALL_sum"
dram="TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"
inst="TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL"
SETS=${SETS:-"utcl tcc"}
run() {  # name alloc set
  local name=$1 alloc=$2 set=$3 C
  case $set in utcl) C=$utcl ;; tcc) C=$tcc ;; dram) C=$dram ;; inst) C=$inst ;; esac
  LSB_RECORD_ALLOC=$alloc timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --output-format csv \
    -d "$OUT/${name}_$set" -o run -- python3 $REPO/tools/alloc_probe.py 30 1 2 > "$OUT/${name}_$set.log" 2>&1
  local rc=$?
  echo "$name $set rc=$rc $(grep -h '"passes"' "$OUT/${name}_$set.log" | tail -1)"
  return $rc
}
for i in 1 2 3; do
  for s in $SETS; do run malloc$i malloc $s || exit 1; done
done
for i in 1 2; do
  for s in $SETS; do run vmm$i vmm $s || exit 1; done
done
