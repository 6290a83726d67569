#!/bin/bash
# bench.py's N>1 flow on the one GPU (ranks sharing it, 2 HW queues each): the full flow at
# NRS ranks, then (last: it aborts rank 0 on purpose) the same with an abort injected at the
# link probes -- the armed line must come out with every schedule's point, roofline and
# cpu_baseline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/bench
TAG=${1:-r3}
for n in ${NRS:-2}; do
  GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --same-device ${BENCH_ARGS} \
    > gpurun_out/bench/n${n}_$TAG.json 2> gpurun_out/bench/n${n}_$TAG.err
  rc=$?; echo "n=$n rc=$rc"; cut -c1-600 gpurun_out/bench/n${n}_$TAG.json
  [ $rc -ne 0 ] && exit $((20 + n))
done
if [ -n "$INJECT" ]; then
  MNCCL_BENCH_INJECT=$INJECT GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29790 bench.py --gpus 2 --same-device --no-sweep \
    > gpurun_out/bench/inject_${INJECT}_$TAG.json 2> gpurun_out/bench/inject_${INJECT}_$TAG.err
  echo "inject $INJECT rc=$?"; cut -c1-600 gpurun_out/bench/inject_${INJECT}_$TAG.json
fi
echo bench-check-done
