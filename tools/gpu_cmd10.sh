set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q -k "allreduce" > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 5; }
NR=2 timeout -k 10 900 bash tools/ring_sweep.sh > gpurun_out/ring_sweep3.log 2>&1; echo "sweep2 rc=$?"
NR=4 SIZE=256 timeout -k 10 900 bash tools/ring_sweep.sh > gpurun_out/ring_sweep4.log 2>&1; echo "sweep4 rc=$?"
cat gpurun_out/ring_sweep3.log gpurun_out/ring_sweep4.log
