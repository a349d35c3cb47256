#!/bin/bash
# Look-back status stores without sc1 (which drops the line from the writer's
# L2, so same-XCD pollers read at the cross-XCD rate): plain (s0) and sc0 (s1)
# stores, sc1 loads unchanged; then the phase profile of s0.
set -euo pipefail
O=gpurun_out/ab10
mkdir -p $O
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/w1/liblsb.so abtest/s0/liblsb.so abtest/s1/liblsb.so
python tools/ab_summary.py $O/uniform.log
grep -c "verify=(True" $O/uniform.log
LSB_LIBRARY=abtest/ps0/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > $O/ps0.log 2>&1
cat $O/ps0.log
