#!/bin/bash
# Real multi-rank RCCL on one GPU: P processes, one NCCL_HOSTID each, socket
# transport over loopback (tools/rccl_two_ranks.py).  Golden digests at
# (n, P) = (1e6, 2), (1000003, 4), (1048576, 8); verify-only at 2^26.
set -o pipefail
O=gpurun_out/rcclmulti
mkdir -p $O
run() { echo "== $*" | tee -a $O/log; timeout -k 10 240 python -u tools/rccl_two_ranks.py "$@" >> $O/log 2>&1; }
run 8 1000000 2 alltoallv && \
run 16 1000000 2 alltoallv && \
run 16 1000000 2 p2p 1 && \
run 64 1000000 2 alltoallv && \
run 16 1000003 4 alltoallv 7 && \
run 64 1000003 4 p2p && \
run 8 1000003 4 alltoallv && \
run 16 1048576 8 alltoallv && \
run 64 1048576 8 alltoallv && \
run 16 67108864 2 alltoallv
rc=$?
grep -E '^\{|^==' $O/log
exit $rc
