set -o pipefail
mkdir -p gpurun_out/r6_proxy
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "mismatch" > gpurun_out/r6_proxy/mismatch_tests.log 2>&1 || exit 10
tail -1 gpurun_out/r6_proxy/mismatch_tests.log
for n in 8 4; do
  timeout -k 10 600 python3 bench.py --gpus $n --same-device --no-sweep > gpurun_out/r6_proxy/bench_n$n.json 2> gpurun_out/r6_proxy/bench_n$n.err || exit $((20 + n))
  echo "n=$n"; cut -c1-200 gpurun_out/r6_proxy/bench_n$n.json
done
timeout -k 10 600 python -u tools/stress_mixed.py --ranks 8 --calls 200 --seed 61 > gpurun_out/r6_proxy/stress_n8.txt 2>&1 || exit 50
timeout -k 10 400 python -u tools/stress_mixed.py --ranks 3 --calls 200 --seed 62 > gpurun_out/r6_proxy/stress_n3.txt 2>&1 || exit 51
grep STRESS gpurun_out/r6_proxy/stress_n8.txt gpurun_out/r6_proxy/stress_n3.txt
