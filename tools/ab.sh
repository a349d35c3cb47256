#!/bin/bash
# Interleaved A/B timing of several builds of liblsb.so on one GPU box (the
# one A/B driver; every profiles/ab log names the command that made it):
#
#   TAG=r03_ab1 ROUNDS=6 FORMS="uniform zipf" bash tools/ab.sh \
#       base=abtest/base/liblsb.so new=abtest/new/liblsb.so
#
# Builds: name=path pairs (tools/build_at.sh REV DIR for a git revision,
# tools/build_variant.sh DIR -DFLAG for a compile-time variant).
# FORMS (tools/digit_probe.py at 2^LG records, default LG=30):
#   uniform      the LSD sort of the PCG input
#   zipf         Zipf (s = 1.1) keys                      (LSB_DIST=zipf)
#   x16          the per-digit exchange at P = 1, 16-bit  (LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16)
#   x16zipf      the same with Zipf keys; -g0 suffix: LSB_GATHER=0 (placement at every exchange)
#   hybrid       the hybrid local sort                    (LSB_PASSES=hybrid)
#   reduce-scan  count + scan + scatter passes            (LSB_PASSES=reduce-scan)
# Each round runs every build once per form, alternating the build order so
# that clock and thermal drift hit every build alike; one untimed warm-up run
# first.  TESTS="tests/test_onesweep_gpu.py ..." then runs those GPU tests
# against the last build.  Logs: gpurun_out/$TAG/<form>.log, each starting
# with a "# ab.sh" header line; summaries by tools/ab_summary.py.
set -euo pipefail
TAG=${TAG:-ab}
LG=${LG:-30}
R=${ROUNDS:-4}
FORMS=${FORMS:-uniform}
O=gpurun_out/$TAG
mkdir -p "$O"
names=()
paths=()
for b in "$@"; do
  names+=("${b%%=*}")
  paths+=("${b#*=}")
done
rev=$(git rev-parse --short HEAD 2>/dev/null || echo "no-git")
form_env() {
  case $1 in
    uniform) echo "" ;;
    zipf) echo "LSB_DIST=zipf" ;;
    x16) echo "LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16" ;;
    x16-g0) echo "LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16 LSB_GATHER=0" ;;
    x16zipf) echo "LSB_DIST=zipf LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16" ;;
    x16zipf-g0) echo "LSB_DIST=zipf LSB_FORCE_EXCHANGE=1 LSB_RADIX_BITS=16 LSB_GATHER=0" ;;
    hybrid) echo "LSB_PASSES=hybrid" ;;
    reduce-scan) echo "LSB_PASSES=reduce-scan" ;;
    *) echo "unknown form $1" >&2; exit 2 ;;
  esac
}
run() {  # build index, form
  local i=$1 f=$2
  echo "lib=${names[$i]}" >> "$O/$f.log"
  env $(form_env "$f") LSB_LIBRARY="${paths[$i]}" timeout -k 10 180 python tools/digit_probe.py "$LG" \
    >> "$O/$f.log" 2>&1
}
for f in $FORMS; do
  rm -f "$O/$f.log"
  digests=""
  for i in "${!paths[@]}"; do
    digests+=" ${names[$i]}=$(sha256sum "${paths[$i]}" | cut -c1-12)"
  done
  echo "# ab.sh TAG=$TAG LG=$LG ROUNDS=$R form=$f env=[$(form_env "$f")] git=$rev builds:$digests" > "$O/$f.log"
done
env LSB_LIBRARY="${paths[0]}" timeout -k 10 180 python tools/digit_probe.py "$LG" > /dev/null 2>&1
for r in $(seq 1 "$R"); do
  order=("${!paths[@]}")
  if [ $((r % 2)) = 0 ]; then order=($(printf '%s\n' "${order[@]}" | tac)); fi
  for f in $FORMS; do
    for i in "${order[@]}"; do run "$i" "$f"; done
  done
done
for f in $FORMS; do
  echo "== $f"
  python tools/ab_summary.py "$O/$f.log"
  echo "verified: $(grep -c 'verify=(True' "$O/$f.log" || true) runs"
done
if [ -n "${TESTS:-}" ]; then
  last=$((${#paths[@]} - 1))
  LSB_LIBRARY="${paths[$last]}" timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 \
    --timeout-method thread > "$O/tests.log" 2>&1 || true
  echo "tests (${names[$last]}): $(tail -1 "$O/tests.log")"
fi
