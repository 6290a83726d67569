#!/bin/bash
# HISTORICAL: the recipe of a round-2/3 profile; it sets knobs or schedules removed in 4.0 (direct,
# PIPE_DEPTH, TUNE), so it does not run against the 4.x library.
# Round-2 evidence on the one-GPU box (ranks share GPU 0):
#  part A: 8 perf_test rank processes on one GPU (the reference's own topology,
#          perf_test.cpp:46) under several settings; per-variant wall time, exit codes and the
#          watchdog's "stuck on ... word" diagnostic, to find why the default stalls;
#  part B: rocprofv3 on rank 0 of a 4-rank perf_test (1 GiB fp32): kernel trace for ring and
#          direct, then FETCH_SIZE / WRITE_SIZE passes (separate runs) for both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r2_inv}
PART=${2:-AB}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0

coloc() {  # coloc <tag> <limit s> <env...>: 8 ranks, 1 and 16 MiB, 1 warm-up + 3 timed
  local tag=$1 lim=$2; shift 2
  local port=$((29400 + RANDOM % 500))
  local t0=$(date +%s%N)
  for r in $(seq 0 7); do
    env "$@" MINI_NCCL_PORT=$port timeout -k 5 $lim $R/apps/bin/perf_test $r 8 --sizes 1,16 --iters 3 --warmup 1 \
      > $OUT/$tag.r$r.log 2>&1 &
  done
  local rcs=""
  for j in $(jobs -p); do wait $j; rcs="$rcs $?"; done
  local t1=$(date +%s%N)
  echo "$tag: rcs [$rcs ] wall $(( (t1 - t0) / 1000000 )) ms" | tee -a $OUT/summary.txt
  grep -h "stuck on\|timed out\|TIMEOUT\|Init Failed" $OUT/$tag.r*.log | sort | uniq -c | head -8 | tee -a $OUT/summary.txt
  grep -h "^ *[0-9]" $OUT/$tag.r0.log | tee -a $OUT/summary.txt
  # a rank killed at the limit (124/137) means a hang: stop here, nothing more on the GPU
  for rc in $rcs; do if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then echo "$tag: killed/crashed"; return 1; fi; done
  return 0
}

prof() {  # prof <n> <pass> <port> <algo> <rocprof args...>
  local n=$1 pass=$2 port=$3 algo=$4; shift 4
  for r in $(seq 1 $((n-1))); do
    MINI_NCCL_ALGO=$algo MINI_NCCL_TUNE=0 MINI_NCCL_PORT=$port timeout -k 10 200 $R/apps/bin/perf_test $r $n --sizes 1024 > $OUT/$pass.r$r.log 2>&1 &
  done
  MINI_NCCL_ALGO=$algo MINI_NCCL_TUNE=0 MINI_NCCL_PORT=$port timeout -k 10 240 rocprofv3 "$@" -d $OUT/$pass -o run --output-format csv -- $R/apps/bin/perf_test 0 $n --sizes 1024 > $OUT/$pass.log 2>&1
  local rc=$?
  wait
  echo "prof $pass rc=$rc" | tee -a $OUT/summary.txt
  return $rc
}

if [[ $PART == *B* ]]; then
  prof 4 trace_ring_n4 29311 ring --kernel-trace --stats || exit 31
  prof 4 trace_direct_n4 29312 direct --kernel-trace --stats || exit 32
  prof 4 fetch_direct_n4 29313 direct --pmc FETCH_SIZE --kernel-trace || exit 33
  prof 4 write_direct_n4 29314 direct --pmc WRITE_SIZE --kernel-trace || exit 34
  prof 4 fetch_ring_n4 29315 ring --pmc FETCH_SIZE --kernel-trace || exit 35
  prof 4 write_ring_n4 29316 ring --pmc WRITE_SIZE --kernel-trace || exit 36
fi
if [[ $PART == *A* ]]; then
  # watchdog 10 s (the default); every variant bounded at 75 s
  coloc q1_ring_c256 75 GPU_MAX_HW_QUEUES=1 MINI_NCCL_ALGO=ring MINI_NCCL_TUNE=0 || exit 21
  coloc default_ring_c256 75 MINI_NCCL_ALGO=ring MINI_NCCL_TUNE=0 || exit 22
  coloc default_ring_c32 75 MINI_NCCL_ALGO=ring MINI_NCCL_TUNE=0 MINI_NCCL_CHANNELS=32 || exit 23
  coloc q1_direct_c256 75 GPU_MAX_HW_QUEUES=1 MINI_NCCL_ALGO=direct MINI_NCCL_TUNE=0 || exit 24
fi
echo investigate-done
