#!/bin/bash
# Does the pass speed of VMM record buffers change after the GPU test suite
# ran on the box (memory churn, heat)?  Fresh processes of
# tools/alloc_probe.py before and after a part of the suite, GPU temperature
# and memory use beside them.  Output: gpurun_out/r05_churn/.
set -u
O=gpurun_out/${TAG:-r05_churn}
mkdir -p $O
state() { timeout -k 5 30 rocm-smi --showtemp --showmemuse > $O/smi_$1.txt 2>&1; grep -iE "junction|memory.*temp|vram%|use" $O/smi_$1.txt | head -6; }
ap() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/alloc_probe.py 30 1 3 > $O/ap_$name.log 2>&1 || exit 1
  echo "$name: $(python3 tools/r05/ap_summary.py $O/ap_$name.log)"
}
state before
ap pre_vmm1
ap pre_vmm2
timeout -k 10 800 python -u -m pytest ${CHURN_TESTS:-tests/test_gpu_sort.py tests/test_onesweep_gpu.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
state after
ap post_vmm1
ap post_vmm2
ap post_malloc1 LSB_RECORD_ALLOC=malloc
ap post_vmm3
sleep 60
state rested
ap rested_vmm1
