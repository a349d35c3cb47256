#!/bin/bash
# rocprofv3 --stats of the forced 16-bit exchange at P = 1 (tools/digit_probe.py,
# 2^30 records): Zipf keys with gathered passes (g1) and without (g0), and
# uniform keys (u1): which kernels the exchange path adds or slows.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r04_zprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for form in ${FORMS:-g1 g0 u1}; do
  case $form in
    g1) E="LSB_DIST=zipf" ;;
    g0) E="LSB_DIST=zipf LSB_GATHER=0" ;;
    u1) E="LSB_DIST=uniform" ;;
  esac
  env $E LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/$form -o run -- python3 $R/tools/digit_probe.py 30 > $O/$form.log 2>&1
done
echo done
