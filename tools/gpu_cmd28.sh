set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu --durations=8 > gpurun_out/gpu_tests_28.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_28.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_28.log | head -30; exit 5; }
port=29950
for n in 2 4; do
 for cfg in "direct 1" "direct 0" "ring 1"; do
   set -- $cfg; port=$((port+1))
   log=gpurun_out/ovl_n${n}_$1_$2_$port.log
   ( export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=$port MINI_NCCL_ALGO=$1 MINI_NCCL_DIRECT_OVERLAP=$2
     for r in $(seq 1 $((n-1))); do timeout -k 5 120 apps/bin/perf_test $r $n --sizes 1,16,128,512 > /dev/null 2>&1 & done
     timeout -k 5 120 apps/bin/perf_test 0 $n --sizes 1,16,128,512 > $log 2>&1; r=$?; wait; exit $r ); rc=$?
   echo "== n=$n $1 overlap=$2 rc=$rc :" $(grep -E "^ +[0-9]" $log | awk '{printf "%s:%s ", $1/1048576, $3}')
   [ $rc -ne 0 ] && exit 7
 done
done
exit 0
