#!/bin/bash
# The N=8 bench flow (auto-tune, link probe, alt schedule, sizes, host buffers, sweep and the
# C4 4 GiB grid) rehearsed with 8 rank processes on the ONE GPU of a gpurun box.  Not xGMI
# numbers; it checks that the path the driver's 8-GPU run takes completes and verifies.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-px8}
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 8 --same-device > gpurun_out/bench_n8_$TAG.json 2> gpurun_out/bench_n8_$TAG.err
rc=$?; echo "n8 rc=$rc lines=$(wc -l < gpurun_out/bench_n8_$TAG.json)"; cut -c1-600 gpurun_out/bench_n8_$TAG.json; exit $rc
