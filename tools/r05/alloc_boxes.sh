#!/bin/bash
# VMM pieces vs hipMalloc on whichever box this call got: fresh processes of
# tools/alloc_probe.py (one context, 3 sorts each), then the bench's own
# process.  Output: gpurun_out/r05_boxes/<box>_<n>/.
set -u
box=$(hostname | tr -c 'a-zA-Z0-9_\n-' _)
O=gpurun_out/r05_boxes/${box}_$(date +%H%M%S)
mkdir -p $O
echo "box $box"
ap() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 tools/alloc_probe.py 30 1 3 > $O/ap_$name.log 2>&1 || exit 1
  echo "$name: $(python3 tools/r05/ap_summary.py $O/ap_$name.log)"
}
for i in 1 2 3 4; do ap vmm$i LSB_PLACEMENT_CANDIDATES=0; done
for i in 1 2; do ap malloc$i LSB_RECORD_ALLOC=malloc; done
timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline --no-traffic > $O/bench.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('bench', d['value'], d['roofline']['avg_launch_ms'], [p['ms'] for p in d['per_pass']])"
