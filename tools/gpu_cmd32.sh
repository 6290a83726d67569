set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
MNCCL_BENCH_EXTRAS_S=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --same-device > gpurun_out/bench_n2_bail.json 2> gpurun_out/bench_n2_bail.err
rc=$?; echo "bench n2 bail rc=$rc"; cat gpurun_out/bench_n2_bail.json | cut -c1-600; [ $rc -ne 0 ] && exit 7
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; exit $rc
