#!/bin/bash
# Round 6: the chunked per-digit exchange (LSB_OPT_EXCHANGE_CHUNKS) on the GPU:
# its tests, then the x16 extra's form (P = 1, the 16-bit exchange forced
# through a world-of-one RCCL communicator) with and without chunks, in fresh
# processes, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/${TAG:-r06_g2}; mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_chunked_exchange_gpu.py > $O/tests.log 2>&1 || { tail -80 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  for C in 0 8; do
    echo "== x16 chunks=$C #$i $(date +%T)"
    LSB_EXCHANGE_CHUNKS=$C timeout -k 10 300 python -u bench.py --force-exchange --radix-bits 16 --no-extras \
      --no-cpu-baseline --no-traffic --steps 5 --warmup 2 > $O/x16_c${C}_$i.log 2>&1 || { tail -30 $O/x16_c${C}_$i.log; exit 1; }
    tail -1 $O/x16_c${C}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','verified')}, d.get('kernel_ms_per_step'))"
  done
done
