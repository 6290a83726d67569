set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu --durations=10 > gpurun_out/gpu_tests_34.log 2>&1; rc=$?
tail -14 gpurun_out/gpu_tests_34.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_34.log | head -30; exit 5; }
exit 0
