set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 4; }
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 5; }
timeout -k 10 900 bash tools/ring_sweep.sh > gpurun_out/ring_sweep2.log 2>&1; echo "sweep rc=$?"
cat gpurun_out/ring_sweep2.log
timeout -k 10 120 ./tools/lr_sweep > gpurun_out/lr_sweep4.log 2>&1; cat gpurun_out/lr_sweep4.log
