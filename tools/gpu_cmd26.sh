set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
port=29900
for n in 2 4; do
 for algo in ring direct; do
  for cfg in "64 256 131072" "128 128 131072" "256 64 131072" "128 64 131072" "128 64 524288" "256 64 262144" "256 128 131072" "128 256 131072"; do
   set -- $cfg; port=$((port+1))
   log=gpurun_out/geo_n${n}_${algo}_$1_$2_$3.log
   ( export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=$port MINI_NCCL_CHANNELS=$1 MINI_NCCL_THREADS=$2 MINI_NCCL_SLICE_SIZE=$3 MINI_NCCL_ALGO=$algo
     for r in $(seq 1 $((n-1))); do timeout -k 5 120 apps/bin/perf_test $r $n --sizes 1,16,128,512 > /dev/null 2>&1 & done
     timeout -k 5 120 apps/bin/perf_test 0 $n --sizes 1,16,128,512 > $log 2>&1; r=$?; wait; exit $r ); rc=$?
   echo "== n=$n $algo ch=$1 thr=$2 slice=$3 rc=$rc :" $(grep -E "^ +[0-9]" $log | awk '{printf "%s:%s ", $1/1048576, $3}')
   [ $rc -ne 0 ] && exit 7
  done
 done
done
exit 0
