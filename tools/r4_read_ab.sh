#!/bin/bash
# Interleaved A/B/... of the read schedule between library builds on ONE GPU (every rank on GPU 0,
# $QUEUES HW queues each, default 2): LIBS = "tag:dir ..." where dir holds a libmini_nccl.so
# (LD_LIBRARY_PATH wins over the apps' RUNPATH) or is "in-tree"; perf_test rank 0 (bytes, us,
# algbw, busbw, schedule), MINI_NCCL_ALGO=$ALGO (default read).
R=${GRAFT_REPO_ROOT:-$(pwd)}
LIBS=${LIBS:-"in-tree:in-tree stream:$R/tools/variants/stream"}
SIZES=${SIZES:-64,1024}
export GPU_MAX_HW_QUEUES=${QUEUES:-2} MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_ALGO=${ALGO:-read}
run() {
  local nr="$1" tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test $r $nr --sizes $SIZES > /tmp/ra_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" MINI_NCCL_PORT=$port timeout -k 5 120 $R/apps/bin/perf_test 0 $nr --sizes $SIZES > /tmp/ra_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "== $tag rc=$rc"
  grep -E "^ +[0-9]+ " /tmp/ra_0.log
  [ $rc -ne 0 ] && { tail -5 /tmp/ra_0.log; exit 9; }
  return 0
}
for round in ${ROUNDS:-1 2 3}; do
  for nr in ${NRS:-2 4 8}; do
    for spec in $LIBS; do
      tag=${spec%%:*}; dir=${spec#*:}
      if [ "$dir" = in-tree ]; then run $nr "$tag round=$round n=$nr" X=1
      else run $nr "$tag round=$round n=$nr" LD_LIBRARY_PATH=$dir; fi
    done
  done
done
