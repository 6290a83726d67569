set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
MINI_NCCL_SYS_FENCE=0 timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests_24_nofence.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_24_nofence.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_24_nofence.log | head -30; exit 5; }
port=29800
for n in 2 4; do
 for f in 1 0 1 0; do
  port=$((port+1))
  log=gpurun_out/fence_n${n}_f${f}_$port.log
  ( export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=$port MINI_NCCL_SYS_FENCE=$f
    for r in $(seq 1 $((n-1))); do timeout -k 5 120 apps/bin/perf_test $r $n --sizes 1,4,16,64,128 > /dev/null 2>&1 & done
    timeout -k 5 120 apps/bin/perf_test 0 $n --sizes 1,4,16,64,128 > $log 2>&1; r=$?; wait; exit $r ); rc=$?
  echo "== n=$n sys_fence=$f rc=$rc"; grep -E "^ +[0-9]" $log
  [ $rc -ne 0 ] && exit 7
 done
done
exit 0
