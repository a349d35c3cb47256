#!/bin/bash
# bench.py's N > 1 RCCL path rehearsed on one GPU: P ranks under
# torch.distributed.run, one NCCL_HOSTID each (--transport rccl-sockets), so
# RCCL links them by its socket transport.  A shape/correctness check of the
# exact command the driver runs at N = 2..8, not a measurement.  Then the
# multi-rank RCCL golden-digest tests.
set -o pipefail
O=gpurun_out/rcclbench
mkdir -p $O
tr() { timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
        --master-port $2 bench.py --gpus $1 --transport rccl-sockets --n-per-gpu 67108864 --steps 2 --warmup 1 "${@:3}"; }
tr 2 29511 --no-cpu-baseline > $O/n2.log 2>&1 && tail -1 $O/n2.log | cut -c1-400 && \
tr 4 29512 --no-cpu-baseline --dist zipf > $O/n4_zipf.log 2>&1 && tail -1 $O/n4_zipf.log | cut -c1-400 && \
tr 2 29513 --no-cpu-baseline --no-whole-key --exchange peer > $O/n2_peer.log 2>&1 && tail -1 $O/n2_peer.log | cut -c1-400 && \
timeout -k 10 600 python -u -m pytest tests/test_rccl_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -12 $O/tests.log
exit $rc
