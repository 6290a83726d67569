#!/bin/bash
# rocprofv3 evidence for bench.py at N=1, all in ONE lease at one HEAD (run on the GPU box from the
# repo root; tools/pmc_summary.py turns gpurun_out/$TAG/ into profiles/):
#   0) python3 bench.py --gpus 1 as the driver runs it (the plain line, extras included)
#   1) the headline under rocprofv3 --kernel-trace --stats: its line (HIP events) and the trace come
#      from the SAME process (--no-alt: no host-inclusive pieces or proxy ranks mixing into the
#      per-launch numbers)
#   2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE in separate passes (TCC slots: MI355X_MICROARCH.md)
#   usage: tools/profile_n1.sh <tag> <head>
set -o pipefail
TAG=${1:-prof_n1}
HEAD=${2:-unknown}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
echo "$HEAD" > $OUT/head.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 $R/bench.py --gpus 1 > $OUT/line_plain.json 2> $OUT/plain.log || exit 10
echo plain-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --gpus 1 --no-cpu-baseline --no-alt > $OUT/line_traced.json 2> $OUT/trace.log || exit 11
echo trace-done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --gpus 1 --no-cpu-baseline --no-alt --steps 5 --warmup 1 > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --gpus 1 --no-cpu-baseline --no-alt --steps 5 --warmup 1 > $OUT/write.log 2>&1 || exit 13
echo profile-done
