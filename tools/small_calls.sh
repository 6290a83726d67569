#!/bin/bash
# Per-call time with 2 / 4 / 8 rank processes sharing one GPU (perf_test rank 0, ITERS calls per
# size, ROUNDS rounds interleaved).  CFGS: entries "label[:algo[:KNOB=V...]]" -- label alone is a
# schedule: ring | read | oneshot | read_grid | auto | window (read on registered windows, perf_test
# --window: no host rendezvous) | window_neg (the same windows, MINI_NCCL_WINDOW_RENDEZVOUS=1);
# with an algo, the label names the point and KNOB=V are extra environment (e.g.
# "grid256k:auto:MINI_NCCL_GRID_MIN=262144:MINI_NCCL_BLOCKING=0").  SIZES: perf_test --sizes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
export GPU_MAX_HW_QUEUES=${QUEUES:-2} MINI_NCCL_PERF_DEVICE=0
for round in ${ROUNDS:-1}; do
for nr in ${NRS:-2 4 8}; do
  for cfg in ${CFGS:-ring read oneshot window}; do
    IFS=: read -r label algo knobs <<< "$cfg"
    algo=${algo:-$label}; extra=""; envs=(MINI_NCCL_WINDOW_RENDEZVOUS=-1)
    if [ "$algo" = window ]; then algo=read; extra=--window; fi
    if [ "$algo" = window_neg ]; then algo=read; extra=--window; envs=(MINI_NCCL_WINDOW_RENDEZVOUS=1); fi
    [ -n "$knobs" ] && envs+=(${knobs//:/ })
    port=$((21000 + RANDOM % 20000))
    pids=()
    for ((r = 1; r < nr; r++)); do
      env MINI_NCCL_ALGO=$algo "${envs[@]}" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr \
        --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_$r.log 2>&1 &
      pids+=($!)
    done
    env MINI_NCCL_ALGO=$algo "${envs[@]}" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr \
      --sizes ${SIZES:-4k,64k,1} --iters ${ITERS:-200} $extra > /tmp/sc_0.log 2>&1
    rc=$?
    for p in "${pids[@]}"; do wait $p; done
    echo "== n=$nr algo=$label round=$round rc=$rc"
    grep -E "^ +[0-9]+ " /tmp/sc_0.log
    [ $rc -ne 0 ] && exit 9
  done
done
done
exit 0
