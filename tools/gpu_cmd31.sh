set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_same_31.json 2> gpurun_out/bench_n2_same_31.err
rc=$?; echo "bench n2 rc=$rc"; cat gpurun_out/bench_n2_same_31.json; [ $rc -ne 0 ] && exit 7
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --same-device > gpurun_out/bench_n4_same_31.json 2> gpurun_out/bench_n4_same_31.err
rc=$?; echo "bench n4 rc=$rc"; cat gpurun_out/bench_n4_same_31.json
exit $rc
