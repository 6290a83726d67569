set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 python -m pytest tests/test_gpu.py -x -q -k "local_reduce" > gpurun_out/gpu_tests_lr.log 2>&1 || { tail -20 gpurun_out/gpu_tests_lr.log; exit 5; }
tail -2 gpurun_out/gpu_tests_lr.log
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 4
cat gpurun_out/bench_n1.json
bash tools/profile_n1.sh prof_n1_r1 || exit 6
find gpurun_out/prof_n1_r1 -name "*.csv" | head -20
