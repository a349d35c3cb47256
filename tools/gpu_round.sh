#!/bin/bash
# One GPU check of the tree (run from the repo root on the GPU box):
#   TAG=r03_v1 RUN="tests smoke bench n2 n4zipf torchrun profile profhyb sq" bash tools/gpu_round.sh
# Steps (each under its own time limit; the first failure ends the call):
#   tests     the whole -m gpu suite
#   smoke     __graft_entry__.smoke()
#   bench     bench.py at N = 1 (live PMC traffic + CPU baseline)
#   n2        bench.py --gpus 2 with no launcher over RCCL's socket transport
#             (two rank processes on the one GPU: the N > 1 code path, not a speed)
#   n2big     the same at 2^28 records per rank (the placement probe runs in each rank)
#   n4zipf    the same at N = 4 with Zipf keys
#   n8        bench.py --gpus 8 over RCCL sockets at 2^22 records per rank (the driver's N = 8 flow)
#   table     tools/table_runs.sh: the DESIGN.md §4 table on this box
#   torchrun  bench.py --gpus 2 under torch.distributed.run (the driver's form)
#   profile   tools/profile.sh: rocprofv3 stats + FETCH_SIZE / WRITE_SIZE passes
#   profhyb   the same for bench.py --passes hybrid (gpurun_out/prof_hybrid;
#             summarise with tools/pmc_summary.py TAG_hybrid gpurun_out/prof_hybrid ... --templates)
#   sq        tools/sq_counters.sh: SQ counters of the sort at 2^28
#   stress    tools/stress_mix.py for STRESS_S seconds (default 150): random sorts, 0 wrong
#   dropin    tests/test_dropin_gpu.py alone (the reference program with its mySort on the library)
#   (experiments: allocbw placement allocpmc abx pick rot clock kcand refine; see each case)
# Output under gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-check}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
RUN=${RUN:-"tests smoke bench"}
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }
for s in $RUN; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/gputests.log 2>&1 || fail tests $O/gputests.log
      tail -2 $O/gputests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || fail smoke $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || fail bench $O/bench.log
      tail -1 $O/bench.log | cut -c1-400 ;;
    n2)
      timeout -k 10 400 python -u bench.py --gpus 2 --transport rccl-sockets --n-per-gpu 67108864 \
        --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_n2.log 2>&1 || fail n2 $O/bench_n2.log
      tail -1 $O/bench_n2.log | cut -c1-400 ;;
    n2big)  # N = 2 at 2^28 records per rank: 4 GiB buffers, so each rank runs the placement probe
      timeout -k 10 400 python -u bench.py --gpus 2 --transport rccl-sockets --n-per-gpu 268435456 \
        --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_n2big.log 2>&1 || fail n2big $O/bench_n2big.log
      tail -1 $O/bench_n2big.log | cut -c1-400 ;;
    n4zipf)
      timeout -k 10 400 python -u bench.py --gpus 4 --transport rccl-sockets --dist zipf \
        --n-per-gpu 16777216 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_n4_zipf.log 2>&1 \
        || fail n4zipf $O/bench_n4_zipf.log
      tail -1 $O/bench_n4_zipf.log | cut -c1-400 ;;
    n8)  # the driver's largest N over RCCL sockets: eight rank processes on the one GPU, both extras
      timeout -k 10 600 python -u bench.py --gpus 8 --transport rccl-sockets --n-per-gpu 4194304 \
        --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_n8.log 2>&1 || fail n8 $O/bench_n8.log
      tail -1 $O/bench_n8.log | cut -c1-400 ;;
    table)  # the DESIGN.md §4 table (tools/table_runs.sh)
      TABLE=$TAG/table timeout -k 10 1100 bash tools/table_runs.sh > $O/table_summary.log 2>&1 || fail table $O/table_summary.log
      cat $O/table_summary.log ;;
    torchrun)
      timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --transport rccl-sockets \
        --n-per-gpu 67108864 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_torchrun_n2.log 2>&1 \
        || fail torchrun $O/bench_torchrun_n2.log
      grep '^{' $O/bench_torchrun_n2.log | tail -1 | cut -c1-400 ;;
    profile)
      bash tools/profile.sh > $O/profile.log 2>&1 || fail profile $O/profile.log
      cp $(find gpurun_out/prof/stats -name "*kernel_stats.csv" -print -quit) $O/kernel_stats.csv || true ;;
    profhyb)
      PROF=prof_hybrid BENCH_ARGS="--passes hybrid" bash tools/profile.sh > $O/profile_hybrid.log 2>&1 \
        || fail profhyb $O/profile_hybrid.log ;;
    sq)
      SQ_TAG=_$TAG bash tools/sq_counters.sh > $O/sq.log 2>&1 || fail sq $O/sq.log ;;
    stress)
      timeout -k 10 400 python -u tools/stress_mix.py --seconds ${STRESS_S:-150} --seed ${STRESS_SEED:-7} --max-log2 ${STRESS_LOG2:-27} --rccl-share ${STRESS_RCCL:-0} --trace --stop-on-error \
        > $O/stress_mix.log 2>&1 || fail stress $O/stress_mix.log
      tail -1 $O/stress_mix.log
      grep -q "done: 0 of" $O/stress_mix.log || fail stress $O/stress_mix.log ;;
    dropin)
      timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py -m gpu -x -v --timeout 240 \
        --timeout-method thread > $O/dropin.log 2>&1 || fail dropin $O/dropin.log
      tail -2 $O/dropin.log ;;
    allocbw)  # buffer-placement probe: 3 fresh processes, then one pooled allocation
      [ -x tools/kbench/allocbw ] || fail allocbw /dev/null
      for k in 1 2 3; do
        timeout -k 10 120 tools/kbench/allocbw 4 30 5 > $O/allocbw_$k.log 2>&1 || fail allocbw $O/allocbw_$k.log
      done
      timeout -k 10 120 tools/kbench/allocbw 4 30 5 1 > $O/allocbw_pool.log 2>&1 || fail allocbw $O/allocbw_pool.log
      grep -h "buffer .: read\|runs" $O/allocbw_*.log | head -60 ;;
    placement)  # A/B: plain A/B allocation vs the calibrated choice, alternating fresh processes
      for k in 1 2 3; do
        for cand in 2 4; do
          LSB_PLACEMENT_CANDIDATES=$cand timeout -k 10 200 python -u tools/alloc_probe.py 30 2 2 \
            >> $O/placement_c$cand.log 2>&1 || fail placement $O/placement_c$cand.log
        done
      done
      grep -h verified $O/placement_c*.log ;;
    allocpmc)  # counters of the placement probe (tools/allocbw_counters.sh)
      TAG=$TAG/allocpmc SETS="${PMC_SETS:-list tcc utcl}" bash tools/allocbw_counters.sh > $O/allocpmc.log 2>&1 \
        || fail allocpmc $O/allocpmc.log
      grep -h "buffer .: read" $O/allocpmc/*.log | head -20 ;;
    abx)  # gathered passes on / off for the forced 16-bit exchange, uniform and Zipf (tools/ab.sh)
      TAG=$TAG/abx ROUNDS=${ABX_ROUNDS:-4} FORMS="x16 x16-g0 x16zipf x16zipf-g0" bash tools/ab.sh \
        cur=distributed-lsb_amd/build/liblsb.so > $O/abx.log 2>&1 || fail abx $O/abx.log
      tail -20 $O/abx.log ;;
    pick)  # does the placement probe predict k_onesweep? best / worst pair alternately, 2 processes
      for k in 1 2; do
        LSB_PICKS=best,worst,best,worst timeout -k 10 300 python -u tools/alloc_probe.py 30 4 2 \
          >> $O/pick.log 2>&1 || fail pick $O/pick.log
      done
      grep -h verified $O/pick.log ;;
    rot)  # A/B: rotated write sweep (-DLSB_OS_ROTATE=1, abtest/rot) against the tree's build
      TAG=$TAG/rot ROUNDS=${ROT_ROUNDS:-4} FORMS="uniform zipf" bash tools/ab.sh \
        base=distributed-lsb_amd/build/liblsb.so rot=abtest/rot/liblsb.so > $O/rot.log 2>&1 || fail rot $O/rot.log
      tail -12 $O/rot.log ;;
    clock)  # effective GPU clock per k_onesweep launch: GRBM_GUI_ACTIVE cycles / launch ns (warming box)
      (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
        --kernel-include-regex 'k_onesweep<' --output-format csv -d $O/clock -o run -- \
        python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-traffic --no-extras) > $O/clock.log 2>&1 \
        || fail clock $O/clock.log
      python3 tools/clock_summary.py $O/clock | tail -20 ;;
    kcand)  # the bench's case: the FIRST context of fresh processes, 4 vs 8 placement candidates
      for k in 1 2 3 4; do
        for cand in 4 8; do
          LSB_PLACEMENT_CANDIDATES=$cand timeout -k 10 200 python -u tools/alloc_probe.py 30 1 3 \
            >> $O/kcand_c$cand.log 2>&1 || fail kcand $O/kcand_c$cand.log
        done
      done
      python3 tools/pick_summary.py $O/kcand_c4.log $O/kcand_c8.log ;;
    refine)  # a placement variant: the FIRST context of fresh processes, abtest/old vs the tree's build
      for k in 1 2 3 4 5; do
        for lib in old new; do
          L=abtest/old/liblsb.so; [ $lib = new ] && L=distributed-lsb_amd/build/liblsb.so
          [ -n "${REFINE_NEW_ENV:-}" ] && L=distributed-lsb_amd/build/liblsb.so
          E=""; [ $lib = new ] && E="${REFINE_NEW_ENV:-}"
          env $E LSB_LIBRARY=$L timeout -k 10 200 python -u tools/alloc_probe.py 30 1 3 \
            >> $O/refine_$lib.log 2>&1 || fail refine $O/refine_$lib.log
        done
      done
      python3 tools/pick_summary.py $O/refine_old.log $O/refine_new.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done $(date +%T)"
