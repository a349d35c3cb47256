#!/bin/bash
# Interleaved A/B of whole-key loopback sorts (tools/merge_profile.py) for
# several builds of liblsb.so:  bash tools/merge_ab.sh "<profile args>" lib1 lib2 ...
set -o pipefail
R=$GRAFT_REPO_ROOT
ARGS=$1; shift
mkdir -p $R/gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    echo "lib=$lib" >> $R/gpurun_out/merge_ab.log
    LSB_LIBRARY=$lib timeout -k 10 120 python3 $R/tools/merge_profile.py $ARGS >> $R/gpurun_out/merge_ab.log 2>&1 || exit 1
  done
done
cat $R/gpurun_out/merge_ab.log
