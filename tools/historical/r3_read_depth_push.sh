#!/bin/bash
# HISTORICAL: the recipe of a round-2/3 profile; it sets knobs or schedules removed in 4.0 (direct,
# PIPE_DEPTH, TUNE), so it does not run against the 4.x library.
# Read schedule (push form) vs iterations per pipeline (MINI_NCCL_PIPE_DEPTH; the default is
# schedule.h kReadDepth = 16, chosen in round 2 for the load form's fill and drain): perf_test
# rank 0, every rank on GPU 0 (2 HW queues each), 16 MiB / 64 MiB / 1 GiB, interleaved rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
SIZES=${SIZES:-16,64,1024}
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2 timeout -k 5 90 $R/apps/bin/perf_test $r $nr --sizes $SIZES > /tmp/rd_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2 timeout -k 5 90 $R/apps/bin/perf_test 0 $nr --sizes $SIZES > /tmp/rd_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "== $tag rc=$rc"
  grep -E "^ +[0-9]+ " /tmp/rd_0.log
  [ $rc -ne 0 ] && exit 9
  return 0
}
for round in 1 2; do
  for nr in ${NRS:-2 4 8}; do
    for d in ${DEPTHS:-4 8 16 32}; do
      run $nr "round=$round n=$nr depth=$d" MINI_NCCL_ALGO=read MINI_NCCL_PIPE_DEPTH=$d
    done
  done
done
