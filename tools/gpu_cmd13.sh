set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -k "8_ranks" > gpurun_out/gpu_tests8.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests8.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests8.log | head -30; exit 5; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --same-device > gpurun_out/bench_n8_same.json 2> gpurun_out/bench_n8_same.err
rc=$?; echo "bench n8 rc=$rc"; cat gpurun_out/bench_n8_same.json
exit 0
