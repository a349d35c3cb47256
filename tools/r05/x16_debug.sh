#!/bin/bash
# Which setting breaks the x16 extra (world-of-one RCCL, 16-bit exchange)?
set -u
out=gpurun_out/${TAG:-r05_x16dbg}
mkdir -p $out
p() { timeout -k 10 120 python3 tools/r05/x16_probe.py "$@" >> $out/probe.log 2>&1; local rc=$?; tail -1 $out/probe.log; [ $rc -le 1 ] || exit $rc; }
p 27 0 0 1
p 28 0 0 1
p 30 0 0 1
p 30 1 1 1
LSB_RECORD_ALLOC=malloc p 29 0 0 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q -k "world_of_one or record_buffers" --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
tail -1 $out/tests.log
