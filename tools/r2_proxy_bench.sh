#!/bin/bash
# bench.py's N>1 flow rehearsed on the one GPU (rank processes sharing it, 2 HW queues each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/bench
TAG=${1:-r2}
for n in ${NRS:-2 4}; do
  GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --same-device ${BENCH_ARGS} > gpurun_out/bench/n${n}_$TAG.json \
    2> gpurun_out/bench/n${n}_$TAG.err
  rc=$?; echo "n=$n rc=$rc"; cut -c1-400 gpurun_out/bench/n${n}_$TAG.json
  [ $rc -ne 0 ] && exit $((20 + n))
done
echo proxy-bench-done
