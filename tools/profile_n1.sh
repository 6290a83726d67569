#!/bin/bash
# rocprofv3 evidence for bench.py at N=1 (run on the GPU box from the repo root):
#   1) --kernel-trace --stats of bench.py's headline (--no-alt: without the host-inclusive extra,
#      whose 64 MiB pieces run the same kernel and would mix into the per-launch numbers)
#   2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE in separate passes (TCC slots: MI355X_MICROARCH.md)
# Outputs under gpurun_out/$TAG/; tools/pmc_summary.py turns them into profiles/.
set -o pipefail
TAG=${1:-prof_n1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-alt > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-alt --steps 5 --warmup 1 > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-alt --steps 5 --warmup 1 > $OUT/write.log 2>&1 || exit 13
echo profile-done
