#!/bin/bash
# Ring small calls, interleaved A/B of two libmini_nccl.so builds on ONE GPU (every rank on GPU 0,
# 2 HW queues per process): A = $AB_DIR/libmini_nccl.so (LD_LIBRARY_PATH wins over the apps'
# RUNPATH), B = the in-tree build.  perf_test rank 0, $ITERS blocking calls per size.
# was the 8-rank ring's 254 -> 502 us (profiles/r3_small_calls_by_ranks.txt) the
# code or the box?
R=${GRAFT_REPO_ROOT:-$(pwd)}
AB_DIR=${AB_DIR:-$R/build_ab}
SIZES=${SIZES:-4k,64k,1}
ITERS=${ITERS:-200}
export GPU_MAX_HW_QUEUES=${QUEUES:-2} MINI_NCCL_PERF_DEVICE=0
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr --sizes $SIZES --iters $ITERS > /tmp/rs_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr --sizes $SIZES --iters $ITERS > /tmp/rs_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "== $tag rc=$rc"
  grep -E "^ +[0-9]+ " /tmp/rs_0.log
  [ $rc -ne 0 ] && { tail -5 /tmp/rs_0.log; exit 9; }
  return 0
}
for round in ${ROUNDS:-1 2 3}; do
  for nr in ${NRS:-8}; do
    run $nr "A round=$round n=$nr ($AB_DIR)" LD_LIBRARY_PATH=$AB_DIR MINI_NCCL_ALGO=ring
    run $nr "B round=$round n=$nr (HEAD)" MINI_NCCL_ALGO=ring
  done
done
