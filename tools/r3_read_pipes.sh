#!/bin/bash
# Read schedule vs pipelines per rank on the one-GPU proxy (every rank on GPU 0, 2 HW queues
# each): is the 2-rank read kernel short of waves in flight (2 per CU at the default 256
# pipelines per rank)?  perf_test rank 0, 1 GiB + 64 MiB fp32, interleaved rounds.  Co-resident
# waves are bounded by 2 per SIMD (the kernels' launch bound): ranks x pipelines <= 2048.
R=${GRAFT_REPO_ROOT:-$(pwd)}
SIZES=${SIZES:-64,1024}
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2 timeout -k 5 90 $R/apps/bin/perf_test $r $nr --sizes $SIZES > /tmp/rp_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2 timeout -k 5 90 $R/apps/bin/perf_test 0 $nr --sizes $SIZES > /tmp/rp_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "== $tag rc=$rc"
  grep -E "^ +[0-9]+ " /tmp/rp_0.log
  [ $rc -ne 0 ] && exit 9
  return 0
}
for round in 1 2; do
  for pt in ${POINTS:-2:256 2:512 2:768 4:256 4:384 4:512}; do
    nr=${pt%%:*}; ch=${pt#*:}
    run $nr "round=$round n=$nr pipelines=$ch" MINI_NCCL_ALGO=read MINI_NCCL_CHANNELS=$ch
  done
done
