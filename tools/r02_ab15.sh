#!/bin/bash
# Own-XCD look-back chains: every workgroup takes tiles only from the
# sub-array of its XCD (s_getreg XCC_ID; no helping across XCDs), with plain
# status stores that stay in that XCD's L2 (xo) or write-through sc1 stores
# (xo16), against the shipped build (auto).  Uniform keys.
set -euo pipefail
O=gpurun_out/ab15
mkdir -p $O
rm -f $O/*.log
AB_LOG=$O/uniform.log ROUNDS=3 bash tools/ab.sh abtest/auto/liblsb.so abtest/xo16/liblsb.so abtest/xo/liblsb.so || true
python tools/ab_summary.py $O/uniform.log
grep -c "verify=(True" $O/uniform.log || true
