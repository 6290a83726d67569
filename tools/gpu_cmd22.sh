set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -k "host_buffers" > gpurun_out/gpu_tests_host.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_host.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_host.log | head -30; exit 5; }
for m in device host staged; do
  for sh in 0 1; do
    [ $m != host ] && [ $sh = 1 ] && continue
    (export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=2991$sh MINI_NCCL_STAGE_HOST=$sh; timeout -k 5 120 apps/bin/perf_test 1 2 --mode $m > gpurun_out/perf_${m}${sh}_r1.log 2>&1 & timeout -k 5 120 apps/bin/perf_test 0 2 --mode $m > gpurun_out/perf_${m}${sh}_r0.log 2>&1; r=$?; wait; exit $r); rc=$?
    echo "== $m stage_host=$sh rc=$rc"; cat gpurun_out/perf_${m}${sh}_r0.log
    [ $rc -ne 0 ] && exit 7
  done
done
exit 0
