set -o pipefail
R=$GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 4
cat gpurun_out/bench_n1.json
(export MINI_NCCL_PERF_DEVICE=0 MINI_NCCL_PORT=29911; timeout -k 5 120 apps/bin/perf_test 1 2 > gpurun_out/perf_test_r1.log 2>&1 & timeout -k 5 120 apps/bin/perf_test 0 2 > gpurun_out/perf_test_r0.log 2>&1; wait) ; echo "perf_test rc=$?"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_n1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_n1.log 2>&1; echo "prof rc=$?"
