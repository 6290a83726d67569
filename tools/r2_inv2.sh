#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r2_inv2
cd $R
timeout -k 10 300 bash tools/r2_direct_sweep.sh > gpurun_out/r2_inv2/direct_sweep.txt 2>&1 || exit 11
cat gpurun_out/r2_inv2/direct_sweep.txt
timeout -k 10 420 python -u tools/r2_coloc8.py > gpurun_out/r2_inv2/coloc8.txt 2> gpurun_out/r2_inv2/coloc8.err || { cat gpurun_out/r2_inv2/coloc8.txt; exit 12; }
cat gpurun_out/r2_inv2/coloc8.txt
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29582 \
  bench.py --gpus 8 --same-device --no-sweep --no-alt --no-cpu-baseline --count 16777216 --steps 5 --warmup 2 \
  > gpurun_out/r2_inv2/bench_n8.json 2> gpurun_out/r2_inv2/bench_n8.err
rc=$?; echo "bench n8 rc=$rc"; cut -c1-700 gpurun_out/r2_inv2/bench_n8.json
echo inv2-done
