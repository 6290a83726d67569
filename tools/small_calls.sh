#!/bin/bash
# Small-call time with 2 / 4 / 8 rank processes sharing one GPU (perf_test rank 0, ITERS blocking
# calls per size, ROUNDS rounds interleaved).  CFGS: schedules -- ring | read | oneshot | window
# (read on registered windows, perf_test --window: no host rendezvous) | window_neg (the same
# windows with MINI_NCCL_WINDOW_RENDEZVOUS=1: negotiated like other calls).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export GPU_MAX_HW_QUEUES=${QUEUES:-2} MINI_NCCL_PERF_DEVICE=0
for round in ${ROUNDS:-1}; do
for nr in ${NRS:-2 4 8}; do
  for cfg in ${CFGS:-ring read oneshot window}; do
    algo=$cfg; extra=""; wr=-1
    if [ "$cfg" = window ]; then algo=read; extra=--window; fi
    if [ "$cfg" = window_neg ]; then algo=read; extra=--window; wr=1; fi
    port=$((21000 + RANDOM % 20000))
    pids=()
    for ((r = 1; r < nr; r++)); do
      MINI_NCCL_ALGO=$algo MINI_NCCL_WINDOW_RENDEZVOUS=$wr MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr \
        --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_$r.log 2>&1 &
      pids+=($!)
    done
    MINI_NCCL_ALGO=$algo MINI_NCCL_WINDOW_RENDEZVOUS=$wr MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr \
      --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_0.log 2>&1
    rc=$?
    for p in "${pids[@]}"; do wait $p; done
    echo "== n=$nr algo=$cfg round=$round rc=$rc"
    grep -E "^ +[0-9]+ " /tmp/sc_0.log
    [ $rc -ne 0 ] && exit 9
  done
done
done
exit 0
