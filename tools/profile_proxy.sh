#!/bin/bash
# rocprofv3 evidence for the all-reduce kernels on ONE GPU (ranks sharing it; the 8-GPU run is
# the driver's): rank 0 of apps/bin/perf_test under the profiler, the other ranks plain.
#   1) --kernel-trace --stats, 2 ranks (ring, the default) and 4 ranks (auto-tuned at init)
#   2) --pmc FETCH_SIZE, 3) --pmc WRITE_SIZE (separate passes), 2 ranks.  The counts come out
#      at ONE rank's bytes (1.007 x): the other rank process's concurrent kernel is not in them.
# Summaries: tools/proxy_stats.py <tag> <round>, tools/proxy_pmc.py <tag> <round>.
set -o pipefail
TAG=${1:-prof_proxy}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0
run() {  # run <n> <pass> <port> <rocprof args...>
  local n=$1 pass=$2 port=$3; shift 3
  for r in $(seq 1 $((n-1))); do
    MINI_NCCL_PORT=$port timeout -k 10 200 $R/apps/bin/perf_test $r $n --sizes 1024 > $OUT/$pass.r$r.log 2>&1 &
  done
  MINI_NCCL_PORT=$port timeout -k 10 240 rocprofv3 "$@" -d $OUT/$pass -o run --output-format csv -- $R/apps/bin/perf_test 0 $n --sizes 1024 > $OUT/$pass.log 2>&1
  local rc=$?
  wait
  return $rc
}
run 2 trace_n2 29301 --kernel-trace --stats || exit 11
run 4 trace_n4 29302 --kernel-trace --stats || exit 12
run 2 fetch_n2 29303 --pmc FETCH_SIZE --kernel-trace || exit 13
run 2 write_n2 29304 --pmc WRITE_SIZE --kernel-trace || exit 14
echo profile-done
