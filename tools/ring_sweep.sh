#!/bin/bash
# Protocol-efficiency sweep on ONE GPU: 2 (or $NR) perf_test ranks sharing GPU 0 (the reference's
# own test topology, perf_test.cpp:46).  Measures the persistent kernels' hand-off machinery, not
# xGMI.  Each line: config -> perf_test row for the given size.
NR=${NR:-2}
SIZE=${SIZE:-256}
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  local tag="$1"; shift
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < NR; r++)); do
    env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test $r $NR --sizes $SIZE > /tmp/ps_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test 0 $NR --sizes $SIZE > /tmp/ps_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "$tag | $(tail -1 /tmp/ps_0.log) rc=$rc"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 9
  return 0
}
for algo in ${ALGOS:-ring read}; do
  for ch in 16 32 64 128; do
    for thr in 64 256 512; do
      for sl in 131072 262144 524288; do
        run "n=$NR algo=$algo ch=$ch thr=$thr slice=$sl" MINI_NCCL_ALGO=$algo MINI_NCCL_CHANNELS=$ch MINI_NCCL_THREADS=$thr MINI_NCCL_SLICE_SIZE=$sl
      done
    done
  done
  run "n=$NR algo=$algo defaults fence=0" MINI_NCCL_ALGO=$algo MINI_NCCL_SYS_FENCE=0
  run "n=$NR algo=$algo defaults slots=4" MINI_NCCL_ALGO=$algo MINI_NCCL_SLOTS=4
done
