set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -k "c2_full or misaligned" > gpurun_out/gpu_tests_c2.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_c2.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_c2.log | head -30; exit 5; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_same.json 2> gpurun_out/bench_n2_same.err
rc=$?; echo "bench n2 rc=$rc"; cat gpurun_out/bench_n2_same.json
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 9
(export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=29912; timeout -k 5 120 apps/bin/perf_test 1 2 --mode staged > gpurun_out/perf_staged_r1.log 2>&1 & timeout -k 5 120 apps/bin/perf_test 0 2 --mode staged > gpurun_out/perf_staged_r0.log 2>&1; wait); echo "staged rc=$?"
cat gpurun_out/perf_staged_r0.log
exit 0
