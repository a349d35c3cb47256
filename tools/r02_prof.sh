#!/bin/bash
# k_onesweep phase profile (LSB_OS_PROFILE build in abtest/prof): thread 0's
# time per phase, look-back rows summed per tile; uniform and Zipf keys.
set -euo pipefail
O=gpurun_out/prof2
mkdir -p $O
LSB_LIBRARY=abtest/prof/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > $O/uniform.log 2>&1
LSB_DIST=zipf LSB_LIBRARY=abtest/prof/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > $O/zipf.log 2>&1
cat $O/uniform.log $O/zipf.log
