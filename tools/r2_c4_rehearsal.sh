#!/bin/bash
# Targeted GPU tests, then bench.py's N=8 flow on the one GPU (8 rank processes, 2 HW queues
# each) with a long extras guard, so the C5 / C4 points of BASELINE.json run to the end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/bench
TAG=${1:-c4}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-late_peer or watchdog}" > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 10; }
tail -3 gpurun_out/gpu_tests_$TAG.log
n=${N:-8}
MNCCL_BENCH_EXTRAS_S=${EXTRAS_S:-700} GPU_MAX_HW_QUEUES=2 timeout -k 10 ${BENCH_TIMEOUT:-850} python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29788 bench.py --gpus $n --same-device \
  ${BENCH_ARGS} > gpurun_out/bench/n${n}_$TAG.json 2> gpurun_out/bench/n${n}_$TAG.err
rc=$?; echo "n=$n rc=$rc"; cut -c1-300 gpurun_out/bench/n${n}_$TAG.json
exit $rc
