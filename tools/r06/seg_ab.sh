#!/bin/bash
# Round 6, VERDICT r05 item 5: the hybrid's fused segment pass.  SQ counters
# of the hybrid sort at 2^28 (tools/sq_counters.sh), then an interleaved A/B
# of the SEG walk's window (LSB_SEG_WIN = 0: the round-5 walk, one LDS read at
# a time; 2: the shipped default; 3) on the hybrid sort of 2^30 records, then
# the hybrid GPU tests on the default build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
B=$R/distributed-lsb_amd/build
SQ_TAG=_r06_hyb_w0 LSB_LIBRARY=$B/ab_seg0/liblsb.so LSB_PASSES=hybrid bash tools/sq_counters.sh && echo "sq done" || { echo "sq failed"; exit 1; }
cd $R
TAG=${TAG:-r06_seg} ROUNDS=${ROUNDS:-5} FORMS=hybrid TESTS="tests/test_hybrid_gpu.py tests/test_hybrid_model.py" \
  bash tools/ab.sh w0=$B/ab_seg0/liblsb.so w2=$B/liblsb.so w3=$B/ab_seg3/liblsb.so
