#!/bin/bash
# Where a small blocking all-reduce's time goes: rank 0 of a 2-rank perf_test at 4 KiB under
# rocprofv3 (kernel + HIP API trace, no counters), the other rank plain.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-small_trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2
MINI_NCCL_PORT=29611 timeout -k 10 120 $R/apps/bin/perf_test 1 2 --sizes 4k --iters 200 > $OUT/r1.log 2>&1 &
MINI_NCCL_PORT=29611 timeout -k 10 150 rocprofv3 --kernel-trace --hip-trace --stats -d $OUT/trace -o run --output-format csv -- $R/apps/bin/perf_test 0 2 --sizes 4k --iters 200 > $OUT/r0.log 2>&1
rc=$?
wait
cat $OUT/r0.log | tail -3
echo "trace rc=$rc"
exit $rc
