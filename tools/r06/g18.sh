#!/bin/bash
# After the whole GPU suite a sort runs ~8 % slower while a copy between
# hipMalloc'd buffers does not (profiles/r06/churn/g17): the record buffers'
# backing after much allocation churn?  Fresh, then after the suite: the
# default (1 GiB VMM pieces, 4 candidates), hipMalloc'd buffers
# (LSB_RECORD_ALLOC=malloc), 2 MiB pieces, and 8 candidates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r06_g18; mkdir -p $O
one() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-traffic --steps 5 --warmup 2 \
    > $O/bench_$tag.log 2>&1 || return 1
  echo "$tag: $(tail -1 $O/bench_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["placement"]["candidates"], d["placement"]["chosen_ms"], d["placement"]["worst_ms"], d["placement"]["record_alloc"])')"
}
forms() {
  one $1_default LSB_X=0 || return 1
  one $1_malloc LSB_RECORD_ALLOC=malloc || return 1
  one $1_vmm2m LSB_VMM_CHUNK_MIB=2 || return 1
  one $1_k8 LSB_PLACEMENT_CANDIDATES=8 || return 1
}
forms fresh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { tail -20 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
forms suite || exit 1
