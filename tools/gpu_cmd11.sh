set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 4; }
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 5; }
for NRK in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NRK --master-addr 127.0.0.1 --master-port 2953$NRK bench.py --gpus $NRK --same-device > gpurun_out/bench_n${NRK}_same.json 2> gpurun_out/bench_n${NRK}_same.err
rc=$?; echo "bench n$NRK rc=$rc"; cat gpurun_out/bench_n${NRK}_same.json
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 9
done
exit 0
