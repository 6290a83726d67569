#!/bin/bash
# Read schedule (MINI_NCCL_ALGO=read): its GPU tests, then ring / read on the one-GPU
# proxy (2, 4, 8 rank processes, 1 GiB fp32 per rank; perf_test rank 0's row per point).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
TAG=${1:-read}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${K:-read}" \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/gpu_tests_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
SIZE=${SIZE:-1024}
run() {
  local nr="$1"; local tag="$2"; shift 2
  local port=$((20000 + RANDOM % 20000))
  local pids=()
  for ((r = 1; r < nr; r++)); do
    env "$@" GPU_MAX_HW_QUEUES=2 MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test $r $nr --sizes $SIZE --iters 10 --warmup 3 > /tmp/ps_$r.log 2>&1 &
    pids+=($!)
  done
  env "$@" GPU_MAX_HW_QUEUES=2 MINI_NCCL_PORT=$port MINI_NCCL_PERF_DEVICE=0 timeout -k 5 90 $R/apps/bin/perf_test 0 $nr --sizes $SIZE --iters 10 --warmup 3 > /tmp/ps_0.log 2>&1
  local rc=$?
  for p in "${pids[@]}"; do wait $p; done
  echo "n=$nr $tag | $(tail -1 /tmp/ps_0.log) rc=$rc" | tee -a gpurun_out/read_perf_$TAG.txt
  if [ $rc -ne 0 ]; then cat /tmp/ps_0.log | tail -5; exit 9; fi
  return 0
}
IFS=';' read -ra VARS <<< "${VARIANTS:-}"
[ ${#VARIANTS} -eq 0 ] && VARS=("")
for n in ${NRS:-2 4 8}; do
  for a in ${ALGOS:-ring read}; do
    for v in "${VARS[@]}"; do
      run $n "$a $v" MINI_NCCL_ALGO=$a $v
    done
  done
done
echo read-check-done
