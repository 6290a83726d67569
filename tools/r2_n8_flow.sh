#!/bin/bash
# The full N=8 bench flow (probes, both schedules, RCCL skipped, sizes, host buffers, 18 sweep
# points, the C4 4 GiB grid) with 8 rank processes on the one GPU of a gpurun box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r2_bench
TAG=${1:-r2}
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29788 bench.py --gpus 8 --same-device > gpurun_out/r2_bench/n8_flow_$TAG.json 2> gpurun_out/r2_bench/n8_flow_$TAG.err
rc=$?; echo "n8 rc=$rc"; cut -c1-800 gpurun_out/r2_bench/n8_flow_$TAG.json; exit $rc
