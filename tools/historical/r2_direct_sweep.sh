#!/bin/bash
# HISTORICAL: the recipe of a round-2/3 profile; it sets knobs or schedules removed in 4.0 (direct,
# PIPE_DEPTH, TUNE), so it does not run against the 4.x library.
# Direct vs ring on the 4-rank one-GPU proxy (1 GiB fp32 per rank): which knob closes direct's
# gap (PMC traffic is 1.007x for both, so the gap is hand-off, not bytes).  perf_test rank 0's
# row per point; MINI_NCCL_TUNE=0.
NR=${NR:-4}
SIZE=${SIZE:-1024}
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  local tag="$1"; shift
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < NR; r++)); do
    env "$@" MINI_NCCL_TUNE=0 MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test $r $NR --sizes $SIZE --iters 10 --warmup 3 > /tmp/ps_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_TUNE=0 MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test 0 $NR --sizes $SIZE --iters 10 --warmup 3 > /tmp/ps_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "$tag | $(tail -1 /tmp/ps_0.log) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit 9; fi
  return 0
}
run "ring defaults" MINI_NCCL_ALGO=ring
run "direct defaults" MINI_NCCL_ALGO=direct
for v in "MINI_NCCL_SLOTS=4" "MINI_NCCL_SLOTS=8" "MINI_NCCL_DIRECT_OVERLAP=0" "MINI_NCCL_SLICE_SIZE=65536" \
         "MINI_NCCL_SLICE_SIZE=262144" "MINI_NCCL_CHANNELS=128" "MINI_NCCL_CHANNELS=512" \
         "MINI_NCCL_SLOTS=4 MINI_NCCL_SLICE_SIZE=65536" "MINI_NCCL_THREADS=128 MINI_NCCL_CHANNELS=256"; do
  run "direct $v" MINI_NCCL_ALGO=direct $v
done
run "ring MINI_NCCL_SLOTS=4" MINI_NCCL_ALGO=ring MINI_NCCL_SLOTS=4
