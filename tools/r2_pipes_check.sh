#!/bin/bash
# full -m gpu suite, then A/B (build_ab = previous commit vs in-tree) of small and mid read calls
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
bash tools/r2_gpu_suite.sh $1 || exit 10
export GPU_MAX_HW_QUEUES=2
NRS="2 4 8" ALGOS=read SIZES=4k,64k,1,16 timeout -k 10 400 bash tools/ab_perf_test.sh > gpurun_out/ab_$1.txt 2>&1 || exit 21
echo done
