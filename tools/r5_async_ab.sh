#!/bin/bash
# blocking vs stream-ordered calls, perf_test rank 0, 2 and 8 ranks on one GPU
R=${GRAFT_REPO_ROOT:-$(pwd)}
export GPU_MAX_HW_QUEUES=2 MINI_NCCL_PERF_DEVICE=0
for round in 1 2; do
for nr in 2 8; do
for blk in 1 0; do
  for algo in read ring; do
    port=$((21000 + RANDOM % 20000)); pids=()
    for ((r = 1; r < nr; r++)); do
      MINI_NCCL_BLOCKING=$blk MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr --sizes 4k,64k,1,16 --iters 200 > /tmp/ab_$r.log 2>&1 &
      pids+=($!)
    done
    MINI_NCCL_BLOCKING=$blk MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr --sizes 4k,64k,1,16 --iters 200 > /tmp/ab_0.log 2>&1
    rc=$?
    for p in "${pids[@]}"; do wait $p; done
    echo "== n=$nr blocking=$blk algo=$algo round=$round rc=$rc"
    grep -E "^ +[0-9]+ " /tmp/ab_0.log
    [ $rc -ne 0 ] && exit 9
  done
done
done
done
exit 0
