#!/bin/bash
# Round 6, SEG pass, third A/B: the shipped form of seg_ab2 (w2b4, built from
# git HEAD at the time into build/ab_segprev) against the same with the
# window's first neighbour taken from the neighbour test (new default) and
# against stage neighbours read from LDS instead of DPP (LSB_SEG_LDSNB = 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
B=$R/distributed-lsb_amd/build
TAG=${TAG:-r06_seg3} ROUNDS=${ROUNDS:-5} FORMS=hybrid TESTS="tests/test_hybrid_gpu.py" \
  bash tools/ab.sh prev=$B/ab_segprev/liblsb.so ldsnb=$B/ab_ldsnb/liblsb.so new=$B/liblsb.so
