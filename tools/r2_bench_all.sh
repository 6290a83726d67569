#!/bin/bash
# bench.py as the driver runs it (N=1), the N>1 flows rehearsed on the one GPU (2, 4, 8 rank
# processes), then the N=1 rocprofv3 evidence (trace + separate PMC passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r2_bench
TAG=${1:-r2}
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench/n1_$TAG.json 2> gpurun_out/r2_bench/n1_$TAG.err || exit 11
cut -c1-600 gpurun_out/r2_bench/n1_$TAG.json
for n in 2 4 8; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --same-device ${BENCH_ARGS} > gpurun_out/r2_bench/n${n}_$TAG.json \
    2> gpurun_out/r2_bench/n${n}_$TAG.err
  rc=$?; echo "n=$n rc=$rc"; cut -c1-500 gpurun_out/r2_bench/n${n}_$TAG.json
  [ $rc -ne 0 ] && exit $((20 + n))
done
bash tools/profile_n1.sh prof_n1_$TAG || exit 31
echo bench-all-done
