#!/bin/bash
# N>1 bench flow rehearsed on the 1-GPU box (every rank on GPU 0): n=2 with the C4 grid forced
# at 256 MiB, n=4 as the driver would run it (its sweep included).  Not xGMI numbers.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-px}
MNCCL_BENCH_C4=1 MNCCL_BENCH_C4_MIB=256 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_$TAG.json 2> gpurun_out/bench_n2_$TAG.err
rc=$?; echo "n2 rc=$rc lines=$(wc -l < gpurun_out/bench_n2_$TAG.json)"; cut -c1-400 gpurun_out/bench_n2_$TAG.json; [ $rc -ne 0 ] && exit 6
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --same-device > gpurun_out/bench_n4_$TAG.json 2> gpurun_out/bench_n4_$TAG.err
rc=$?; echo "n4 rc=$rc lines=$(wc -l < gpurun_out/bench_n4_$TAG.json)"; cut -c1-400 gpurun_out/bench_n4_$TAG.json; exit $rc
