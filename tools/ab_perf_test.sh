#!/bin/bash
# A/B of two libmini_nccl.so builds on ONE GPU box (every rank on GPU 0): perf_test rows for
# NR ranks, interleaved rounds, A = $AB_DIR/libmini_nccl.so (LD_LIBRARY_PATH wins over the
# apps' RUNPATH), B = the in-tree build.  Protocol latency / throughput only, not xGMI.
R=${GRAFT_REPO_ROOT:-$(pwd)}
AB_DIR=${AB_DIR:-$R/build_ab}
SIZES=${SIZES:-1,16,64,128}
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test $r $nr --sizes $SIZES > /tmp/ab_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test 0 $nr --sizes $SIZES > /tmp/ab_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "== $tag rc=$rc"
  grep -E "^ +[0-9]+ " /tmp/ab_0.log
  [ $rc -ne 0 ] && exit 9
  return 0
}
for round in 1 2 3; do
  for nr in ${NRS:-2 4}; do
    for algo in ${ALGOS:-ring read}; do
      run $nr "A round=$round n=$nr algo=$algo" LD_LIBRARY_PATH=$AB_DIR MINI_NCCL_ALGO=$algo
      run $nr "B round=$round n=$nr algo=$algo" MINI_NCCL_ALGO=$algo
    done
  done
done
