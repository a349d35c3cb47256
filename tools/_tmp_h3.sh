set -o pipefail
mkdir -p gpurun_out/r03_h3; rm -f gpurun_out/r03_h3/*
timeout -k 10 600 python -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_h3/tests.log 2>&1; echo "tests rc=$?"; tail -30 gpurun_out/r03_h3/tests.log
for i in 1 2; do
LSB_PASSES=hybrid timeout -k 10 120 python -u tools/digit_probe.py 30 >> gpurun_out/r03_h3/probe.log 2>&1 || exit 1
done
cat gpurun_out/r03_h3/probe.log
timeout -k 10 120 ./tools/kbench/copybw 30 > gpurun_out/r03_h3/copybw.log 2>&1 || exit 1
cat gpurun_out/r03_h3/copybw.log
