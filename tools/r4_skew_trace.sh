#!/bin/bash
# VERDICT r3 #2, second half: on the one-GPU proxy each rank is its own process with its own
# queue, so the ranks' kernels of one call do not start together, and a rank's kernel waits for
# its last peer's START.  Every rank of apps/bin/perf_test (1 GiB fp32, 10 calls) under its own
# rocprofv3 --kernel-trace: per call, the ranks' start / end timestamps (one clock per node) give
# the launch skew and the window in which every rank's kernel ran.  Summary:
# tools/r4_skew_summary.py gpurun_out/<tag>.
set -o pipefail
TAG=${1:-r4_skew}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2
for cfg in ${CFGS:-2:read 4:read 8:read 2:ring 4:ring}; do
  n=${cfg%%:*}; algo=${cfg#*:}
  port=$((22000 + RANDOM % 20000))
  pids=()
  for r in $(seq 0 $((n-1))); do
    MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 5 90 rocprofv3 --kernel-trace -d $OUT/${algo}_n${n}/r$r -o run \
      --output-format csv -- $R/apps/bin/perf_test $r $n --sizes 1024 --iters 10 --warmup 2 > $OUT/${algo}_n${n}.r$r.log 2>&1 &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "${algo}_n${n} rc=$rc"
  [ $rc -ne 0 ] && exit 10
done
echo skew-done
