#!/bin/bash
# A/B: HEAD (abtest/base) vs the working tree (abtest/new), 2^30 records, uniform then Zipf keys.
set -euo pipefail
mkdir -p gpurun_out/ab1
AB_LOG=gpurun_out/ab1/uniform.log ROUNDS=4 bash tools/ab.sh abtest/base/liblsb.so abtest/new/liblsb.so
LSB_DIST=zipf AB_LOG=gpurun_out/ab1/zipf.log ROUNDS=3 bash tools/ab.sh abtest/base/liblsb.so abtest/new/liblsb.so
python tools/ab_summary.py gpurun_out/ab1/uniform.log
python tools/ab_summary.py gpurun_out/ab1/zipf.log
