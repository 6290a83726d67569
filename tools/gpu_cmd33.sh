set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > gpurun_out/bench_n1_33.json 2> gpurun_out/bench_n1_33.err; rc=$?
echo "n1 rc=$rc lines=$(wc -l < gpurun_out/bench_n1_33.json)"; cut -c1-300 gpurun_out/bench_n1_33.json; [ $rc -ne 0 ] && exit 6
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_33.json 2> gpurun_out/bench_n2_33.err
rc=$?; echo "n2 rc=$rc lines=$(wc -l < gpurun_out/bench_n2_33.json)"; cut -c1-300 gpurun_out/bench_n2_33.json; exit $rc
