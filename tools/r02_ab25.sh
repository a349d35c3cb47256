#!/bin/bash
# Compiler scheduling strategies for the whole library (lsb_kernels.hip et al.):
# base (default), -amdgpu-sched-strategy=max-ilp, =max-memory-clause,
# -amdgpu-schedule-relaxed-occupancy.  Uniform 2^30 sorts, interleaved.
set -euo pipefail
O=gpurun_out/ab25
mkdir -p $O
rm -f $O/*.log
LSB_LIBRARY=abtest/base/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4; do
  if [ $((i % 2)) = 1 ]; then for v in base ilp memclause relaxed; do run $v uniform; done
  else for v in relaxed memclause ilp base; do run $v uniform; done; fi
done
python tools/ab_summary.py $O/uniform.log
grep -c "verify=(True" $O/uniform.log || true
