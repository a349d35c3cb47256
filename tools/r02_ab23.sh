#!/bin/bash
# Look-back service workgroups (abtest/svc = working tree) against the same
# build without them (abtest/nosvc): single-read suites first, then the GPU
# suite, then uniform keys, Zipf keys and the forced 16-bit exchange.
set -euo pipefail
O=gpurun_out/ab23
mkdir -p $O
rm -f $O/*.log
timeout -k 10 300 python -u -m pytest tests/test_onesweep_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gputests_os.log 2>&1 \
  || { tail -40 $O/gputests_os.log; exit 1; }
tail -2 $O/gputests_os.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
LSB_LIBRARY=abtest/nosvc/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 > /dev/null 2>&1
run() { echo "lib=$1" >> $O/$2.log; LSB_LIBRARY=abtest/$1/liblsb.so timeout -k 10 120 python tools/digit_probe.py 30 >> $O/$2.log 2>&1; }
for i in 1 2 3 4 5 6 7 8; do
  if [ $((i % 2)) = 1 ]; then run nosvc uniform; run svc uniform; else run svc uniform; run nosvc uniform; fi
done
python tools/ab_summary.py $O/uniform.log
for i in 1 2 3; do LSB_DIST=zipf run nosvc zipf; LSB_DIST=zipf run svc zipf; done
python tools/ab_summary.py $O/zipf.log
export LSB_RADIX_BITS=16 LSB_FORCE_EXCHANGE=1
for i in 1 2; do run nosvc x16; run svc x16; done
python tools/ab_summary.py $O/x16.log
