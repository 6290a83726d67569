#!/bin/bash
# A round's evidence on the one GPU, step by step (each under its own time limit; the first failure
# ends the call): STEP=suite -> the whole -m gpu suite (one process) + smoke (PYTEST_K: a -k filter);
# STEP=n1 -> bench.py N=1 and its rocprofv3 evidence from the same lease (tools/profile_n1.sh,
# HEAD=<commit>); STEP=proxy -> the N > 1
# bench flow with NRS rank processes sharing the GPU; STEP=small -> small calls by rank count;
# STEP=stress -> the mixed-schedule stress at 8 and 3 ranks; STEP=inject -> the injected-abort
# rehearsal.  Outputs under gpurun_out/<RND>_<step>/ (RND: r6 by default).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for step in ${STEP:-suite}; do
  O=gpurun_out/${RND:-r6}_$step; mkdir -p $O
  case $step in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || exit 10
      tail -2 $O/gpu_tests.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
      tail -2 $O/smoke.log ;;
    n1)
      bash tools/profile_n1.sh ${RND:-r6}_n1 ${HEAD:-unknown} || exit 13
      cut -c1-400 gpurun_out/${RND:-r6}_n1/line_plain.json ;;
    proxy)
      for n in ${NRS:-2 4 8}; do
        GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --same-device ${BENCH_ARGS} \
          > $O/bench_n${n}_same_gpu.json 2> $O/bench_n${n}.err || exit $((20 + n))
        echo "n=$n"; cut -c1-300 $O/bench_n${n}_same_gpu.json
      done ;;
    small)
      ROUNDS="${ROUNDS:-1 2 3}" ITERS=500 timeout -k 10 600 bash tools/small_calls.sh > $O/small_calls.txt 2>&1 || exit 30
      python3 tools/ab_summary.py $O/small_calls.txt ;;
    stress)
      timeout -k 10 550 python -u tools/stress_mixed.py --ranks 8 --calls 200 --seed 11 > $O/stress_n8.txt 2>&1 || exit 50
      timeout -k 10 400 python -u tools/stress_mixed.py --ranks 3 --calls 200 --seed 12 > $O/stress_n3.txt 2>&1 || exit 51
      grep STRESS $O/stress_n8.txt $O/stress_n3.txt ;;
    inject)
      timeout -k 10 1100 bash tools/inject_check.sh > $O/inject_check.txt 2>&1 || exit 40
      tail -12 $O/inject_check.txt ;;
  esac
done
echo round-check-done
