#!/bin/bash
# Small-call time at 2 / 4 / 8 rank processes sharing one GPU: ring, read (push form), the read
# schedule's load form, one-shot (perf_test rank 0, ITERS blocking calls per size, ROUNDS rounds
# interleaved), CFGS = "algo:read_push ..." (algo "window": read on registered windows, perf_test
# --window: no host rendezvous).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export GPU_MAX_HW_QUEUES=${QUEUES:-2} MINI_NCCL_PERF_DEVICE=0
for round in ${ROUNDS:-1}; do
for nr in ${NRS:-2 4 8}; do
  for cfg in ${CFGS:-ring:1 read:1 read:0 oneshot:1}; do
    algo=${cfg%%:*}; push=${cfg#*:}; extra=""
    if [ "$algo" = window ]; then algo=read; extra=--window; fi
    port=$((21000 + RANDOM % 20000))
    pids=()
    for ((r = 1; r < nr; r++)); do
      MINI_NCCL_ALGO=$algo MINI_NCCL_READ_PUSH=$push MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr \
        --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_$r.log 2>&1 &
      pids+=($!)
    done
    MINI_NCCL_ALGO=$algo MINI_NCCL_READ_PUSH=$push MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr \
      --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_0.log 2>&1
    rc=$?
    for p in "${pids[@]}"; do wait $p; done
    echo "== n=$nr algo=$algo$extra read_push=$push round=$round rc=$rc"
    grep -E "^ +[0-9]+ " /tmp/sc_0.log
    [ $rc -ne 0 ] && exit 9
  done
done
done
exit 0
