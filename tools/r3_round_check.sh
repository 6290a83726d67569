#!/bin/bash
# Round-end rehearsal on the one GPU, as the driver runs it: the full -m gpu suite (one process),
# smoke, bench N=1; then the N>1 bench flows with ranks sharing the GPU (NRS, 2 HW queues each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/bench
TAG=${1:-r3}
bash tools/r2_gpu_suite.sh $TAG || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 11
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench/n1_$TAG.json 2> gpurun_out/bench/n1_$TAG.err || exit 12
cut -c1-300 gpurun_out/bench/n1_$TAG.json
[ -n "$NRS" ] && { NRS="$NRS" bash tools/r3_bench_check.sh $TAG || exit 13; }
echo round-check-done
