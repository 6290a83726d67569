#!/bin/bash
# Round check on the 1-GPU box with the in-tree build (no rebuild): smoke, -m gpu suite, N=1 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 4; }
echo smoke-ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit 5; }
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 6; }
cat gpurun_out/bench_n1.json
exit 0
