set -o pipefail
timeout -k 10 120 ./tools/probe_unaligned > gpurun_out/probe_unaligned.log 2>&1; echo "probe rc=$?"; tail -6 gpurun_out/probe_unaligned.log
grep -q "TOTAL_BAD 0" gpurun_out/probe_unaligned.log || exit 7
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit 5; }
CH=16 timeout -k 10 400 bash tools/nr_scan.sh > gpurun_out/nr_scan16b.log 2>&1; cat gpurun_out/nr_scan16b.log
exit 0
