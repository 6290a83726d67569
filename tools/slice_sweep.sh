#!/bin/bash
# Slice-size sweep on ONE GPU (all ranks on GPU 0): perf_test rows at SIZE MiB for NR ranks,
# ring and read, MINI_NCCL_SLICE_SIZE in SLICES.  Protocol efficiency only, not xGMI.
SIZE=${SIZE:-1024}
SLICES=${SLICES:-"16384 32768 65536 131072"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test $r $nr --sizes $SIZE > /tmp/ps_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test 0 $nr --sizes $SIZE > /tmp/ps_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "$tag | $(tail -1 /tmp/ps_0.log) rc=$rc"
  [ $rc -ne 0 ] && exit 9
  return 0
}
for nr in ${NRS:-2 4 8}; do
  for algo in ${ALGOS:-ring read}; do
    for sl in $SLICES; do
      run $nr "n=$nr algo=$algo slice=$sl" MINI_NCCL_ALGO=$algo MINI_NCCL_SLICE_SIZE=$sl ${EXTRA_ENV}
    done
  done
done
