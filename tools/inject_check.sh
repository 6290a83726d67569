#!/bin/bash
# an abort injected at EVERY stage of bench.py's N > 1 flow after the ring
# (MNCCL_BENCH_INJECT=<stage>: rank 0 calls abort() there, as a GPU fault would) must still
# print the one JSON line, with the schedules measured so far, roofline and cpu_baseline.
# 2 rank processes on the one GPU; one bench run per stage; summary per stage on stdout.
# SELF=1: the same through `python3 bench.py --gpus 2` starting its own rank processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/inject
port=29810
for stage in ${STAGES:-run_read probe standalone rccl sizes small_calls host_buffers sweep}; do
  port=$((port + 1))
  args="--no-sweep"
  [ $stage = sweep ] && args=""
  if [ -n "$SELF" ]; then  # bench.py starting its own rank processes (no launcher)
    MNCCL_BENCH_INJECT=$stage MNCCL_BENCH_C4=0 timeout -k 10 300 python3 bench.py --gpus 2 --same-device \
      --steps 5 --warmup 2 $args > gpurun_out/inject/$stage.json 2> gpurun_out/inject/$stage.err
  else
    MNCCL_BENCH_INJECT=$stage GPU_MAX_HW_QUEUES=2 MNCCL_BENCH_C4=0 timeout -k 10 300 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --same-device \
      --steps 5 --warmup 2 $args > gpurun_out/inject/$stage.json 2> gpurun_out/inject/$stage.err
  fi
  rc=$?
  python3 - "$stage" "$rc" gpurun_out/inject/$stage.json <<'EOF'
import json, sys
stage, rc, path = sys.argv[1], sys.argv[2], sys.argv[3]
lines = [l for l in open(path).read().splitlines() if l.strip().startswith("{")]
if len(lines) != 1:
    print(f"{stage}: rc={rc} JSON lines={len(lines)} -> FAIL")
    sys.exit(0)
d = json.loads(lines[0])
sch = {k: v.get("value", v.get("error", "?")) for k, v in d.get("schedules", {}).items()}
print(f"{stage}: rc={rc} one line, value={d.get('value')} result_check={d.get('config', {}).get('result_check', '-')[:60]!r} "
      f"schedules={sch} roofline.frac={d.get('roofline', {}).get('frac')} cpu_baseline={'yes' if d.get('cpu_baseline') else 'no'} "
      f"extras={[k for k in ('link', 'rccl_reference', 'sizes', 'small_calls', 'host_buffers', 'sweep') if k in d]}")
EOF
done
echo inject-check-done
