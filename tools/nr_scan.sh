#!/bin/bash
# How the same-GPU proxy degrades with the number of rank processes sharing GPU 0.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for NR in 2 3 4 5 6 7 8; do
  for algo in ring direct; do
    port=$((20000 + RANDOM % 20000))
    for ((r = 1; r < NR; r++)); do
      MINI_NCCL_ALGO=$algo MINI_NCCL_CHANNELS=${CH:-16} MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test $r $NR --sizes 64 --iters 5 --warmup 2 > /tmp/nr_$r.log 2>&1 &
    done
    MINI_NCCL_ALGO=$algo MINI_NCCL_CHANNELS=${CH:-16} MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test 0 $NR --sizes 64 --iters 5 --warmup 2 > /tmp/nr_0.log 2>&1
    rc=$?
    wait
    echo "NR=$NR algo=$algo ch=${CH:-16} | $(tail -1 /tmp/nr_0.log) rc=$rc"
    [ $rc -eq 124 ] && exit 9
  done
done
exit 0
