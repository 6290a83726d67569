#!/bin/bash
# 8 torch bench processes on one GPU: per-process hardware queues vs the persistent kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r2_q
for q in 2 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $((29600 + q)) bench.py --gpus 8 --same-device --no-sweep --no-alt --no-cpu-baseline --count 16777216 \
    --steps 5 --warmup 2 > gpurun_out/r2_q/bench_n8_q$q.json 2> gpurun_out/r2_q/bench_n8_q$q.err
  rc=$?; echo "q=$q rc=$rc"; cut -c1-420 gpurun_out/r2_q/bench_n8_q$q.json
  [ $rc -ne 0 ] && exit $rc
done
exit 0
