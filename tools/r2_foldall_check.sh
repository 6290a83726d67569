#!/bin/bash
# read-kernel tests, then A/B (build_ab = previous commit vs in-tree) of the read schedule on
# the one GPU: 4 and 8 ranks at 16 MiB - 1 GiB, and 2 ranks at 4 KiB - 1 MiB (per-call overhead)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "${PYTEST_K:-read or full_size or 8_ranks or late_peer}" > gpurun_out/gpu_tests_$1.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$1.log; [ $rc -eq 0 ] || exit $rc
export GPU_MAX_HW_QUEUES=2
NRS="4 8" ALGOS=read SIZES=16,64,256,1024 timeout -k 10 400 bash tools/ab_perf_test.sh > gpurun_out/ab_$1.txt 2>&1 || exit 21
NRS="2" ALGOS=read SIZES=4k,64k,1 timeout -k 10 200 bash tools/ab_perf_test.sh > gpurun_out/ab_small_$1.txt 2>&1 || exit 22
timeout -k 10 60 tools/probe_host_calls > gpurun_out/probe_host_calls.txt 2>&1 || exit 23
echo done
