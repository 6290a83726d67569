#!/bin/bash
# The C4 grid at its full 4 GiB per rank (BASELINE.json configs[3]) rehearsed with 2 rank
# processes on one GPU (the driver runs it at n = 8): the 4 GiB path end to end, verified.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-c4}
MNCCL_BENCH_C4=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --same-device --no-alt > gpurun_out/bench_n2_$TAG.json 2> gpurun_out/bench_n2_$TAG.err
rc=$?; echo "n2 rc=$rc lines=$(wc -l < gpurun_out/bench_n2_$TAG.json)"; exit $rc
