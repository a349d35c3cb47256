#!/bin/bash
# u32 look-back granules: GPU suite, A/B against the previous commit (uniform,
# Zipf), and k_onesweep's phase profile (LSB_OS_PROFILE build) for both inputs.
set -euo pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2/gputests.log 2>&1 \
  || { tail -40 gpurun_out/ab2/gputests.log; exit 1; }
tail -2 gpurun_out/ab2/gputests.log
AB_LOG=gpurun_out/ab2/uniform.log ROUNDS=4 bash tools/ab.sh abtest/prev/liblsb.so abtest/u32/liblsb.so
LSB_DIST=zipf AB_LOG=gpurun_out/ab2/zipf.log ROUNDS=3 bash tools/ab.sh abtest/prev/liblsb.so abtest/u32/liblsb.so
python tools/ab_summary.py gpurun_out/ab2/uniform.log
python tools/ab_summary.py gpurun_out/ab2/zipf.log
LSB_LIBRARY=abtest/prof/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > gpurun_out/ab2/prof_uniform.log 2>&1
LSB_DIST=zipf LSB_LIBRARY=abtest/prof/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > gpurun_out/ab2/prof_zipf.log 2>&1
grep -h os_profile gpurun_out/ab2/prof_*.log
