#!/bin/bash
# Round 6, SEG pass, second A/B: the batched write-out for the SEG instance
# (LSB_SEG_BATCH records read with their delta entries first; 0: one by one)
# with the windowed walk (LSB_SEG_WIN = 2) against round 5's form (w0b0), on
# the hybrid sort of 2^30 records, then SQ counters of the shipped form and
# the hybrid GPU tests on it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
B=$R/distributed-lsb_amd/build
TAG=${TAG:-r06_seg2} ROUNDS=${ROUNDS:-5} FORMS=hybrid TESTS="tests/test_hybrid_gpu.py tests/test_region_gpu.py" \
  bash tools/ab.sh w0b0=$B/ab_seg0/liblsb.so w2b0=$B/ab_b0/liblsb.so w2b8=$B/ab_b8/liblsb.so w2b4=$B/liblsb.so || exit 1
SQ_TAG=_r06_hyb_b4 LSB_PASSES=hybrid bash tools/sq_counters.sh && echo "sq done"
