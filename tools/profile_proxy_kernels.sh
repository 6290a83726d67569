#!/bin/bash
# rocprofv3 on rank 0 of an N-rank perf_test on the one GPU (1 GiB fp32 per rank): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in separate passes, per (n, kernel form) in POINTS ("2:read_push
# 4:ring 8:read_grid"; read_push = the persistent read kernel; the pass directories carry the form,
# as tools/proxy_pmc_n.py reads them).
# Summary: python tools/proxy_pmc_n.py <tag> <round> <n> <form>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof_proxy}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2
prof() {  # prof <n> <pass> <port> <form: ring | read | read_push | read_grid> <rocprof args...>
  local n=$1 pass=$2 port=$3 algo=$4; shift 4
  [ $algo = read_push ] && algo=read
  for r in $(seq 1 $((n-1))); do
    MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 10 200 $R/apps/bin/perf_test $r $n --sizes 1024 > $OUT/$pass.r$r.log 2>&1 &
  done
  MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 10 240 rocprofv3 "$@" -d $OUT/$pass -o run --output-format csv -- $R/apps/bin/perf_test 0 $n --sizes 1024 > $OUT/$pass.log 2>&1
  local rc=$?
  wait
  echo "prof $pass rc=$rc"
  return $rc
}
port=29500
for pt in ${POINTS:-2:read 4:read}; do
  n=${pt%%:*}; a=${pt#*:}
  prof $n trace_${a}_n$n $((port++)) $a --kernel-trace --stats || exit 31
  prof $n fetch_${a}_n$n $((port++)) $a --pmc FETCH_SIZE --kernel-trace || exit 32
  prof $n write_${a}_n$n $((port++)) $a --pmc WRITE_SIZE --kernel-trace || exit 33
done
echo profile-read-done
