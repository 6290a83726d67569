#!/bin/bash
# Full round check on the 1-GPU box: build, smoke, -m gpu suite, N=1 bench, rocprof + PMC.
set -o pipefail
TAG=${1:-r1}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 4; }
timeout -k 10 1200 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit 5; }
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 6
cat gpurun_out/bench_n1.json
bash tools/profile_n1.sh prof_n1_$TAG || exit 7
exit 0
