#!/bin/bash
# full -m gpu suite (one process, per-test timeout), then an optional extra step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_$TAG.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests_$TAG.log | awk '{print $(NF-1)}' | sort | uniq -c
exit $rc
