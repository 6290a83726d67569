#!/bin/bash
# Round-end rehearsal on the one GPU: full -m gpu suite, smoke, bench N=1 as the driver runs it,
# then the N>1 flows with ranks sharing the GPU (2 HW queues per process).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/bench
TAG=${1:-rc}
bash tools/r2_gpu_suite.sh $TAG || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench/n1_$TAG.json 2> gpurun_out/bench/n1_$TAG.err || exit 12
cut -c1-300 gpurun_out/bench/n1_$TAG.json
NRS="${NRS:-2 4 8}" BENCH_ARGS="${BENCH_ARGS}" bash tools/r2_proxy_bench.sh $TAG || exit 13
echo round-check-done
