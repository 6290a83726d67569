#!/bin/bash
# perf_test on the NR-rank one-GPU proxy (SIZE MiB per rank) for each library variant of
# tools/build_variants.sh ("default" = the shipped library) and each schedule in ALGOS.
NR=${NR:-4}; SIZE=${SIZE:-1024}; ALGOS=${ALGOS:-direct}
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  local tag="$1" lib="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < NR; r++)); do
    env "$@" GPU_MAX_HW_QUEUES=2 LD_LIBRARY_PATH=$lib MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test $r $NR --sizes $SIZE --iters 10 --warmup 3 > /tmp/vs_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" LD_LIBRARY_PATH=$lib MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 60 $R/apps/bin/perf_test 0 $NR --sizes $SIZE --iters 10 --warmup 3 > /tmp/vs_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "$tag | $(tail -1 /tmp/vs_0.log) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit 9; fi
}
for rep in $(seq 1 ${REPS:-2}); do
  for algo in $ALGOS; do
    for v in default ${VARIANTS}; do
      lib=$R/mini-nccl_amd/lib; [ $v != default ] && lib=$R/tools/variants/$v
      run "rep$rep n=$NR $algo $v" $lib MINI_NCCL_ALGO=$algo
    done
  done
done
