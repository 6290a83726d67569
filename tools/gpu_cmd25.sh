set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests_25.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_25.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_25.log | head -30; exit 5; }
timeout -k 10 300 python bench.py > gpurun_out/bench_n1_25.json 2> gpurun_out/bench_n1_25.err; rc=$?
echo "bench n1 rc=$rc"; cat gpurun_out/bench_n1_25.json; [ $rc -ne 0 ] && exit 6
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_same_25.json 2> gpurun_out/bench_n2_same_25.err
rc=$?; echo "bench n2 rc=$rc"; cat gpurun_out/bench_n2_same_25.json; [ $rc -ne 0 ] && exit 7
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --same-device --no-sweep > gpurun_out/bench_n4_same_25.json 2> gpurun_out/bench_n4_same_25.err
rc=$?; echo "bench n4 rc=$rc"; cat gpurun_out/bench_n4_same_25.json
exit $rc
