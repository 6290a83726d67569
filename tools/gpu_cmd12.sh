set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit 5; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --same-device > gpurun_out/bench_n4_same.json 2> gpurun_out/bench_n4_same.err
rc=$?; echo "bench n4 rc=$rc"; cat gpurun_out/bench_n4_same.json
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 9
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/bench_n1_bf16.json 2>gpurun_out/bench_n1_bf16.err; echo "bf16 rc=$?"; cat gpurun_out/bench_n1_bf16.json
exit 0
