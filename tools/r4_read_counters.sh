#!/bin/bash
# where does the push-form read kernel lose HBM time on the one-GPU proxy?
# rocprofv3 counter passes (one run each: the hardware's per-block limits) on rank 0 of
# apps/bin/perf_test (1 GiB fp32), other ranks plain; configs: read (push form) at 2 and 4 ranks,
# the ring at 2 ranks (91-93 % of HBM on the same proxy) and a pure R=2 W=2 stream (mix_probe) as
# the comparisons.
# Summaries: tools/r4_counters_summary.py gpurun_out/<tag>.
set -o pipefail
TAG=${1:-r4_counters}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MINI_NCCL_PERF_DEVICE=0 GPU_MAX_HW_QUEUES=2
PASSES=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
  "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
  "TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
  "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE GRBM_GUI_ACTIVE"
  "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
)
run() {  # run <n> <algo> <pass-index>; algo "mix": tools/bin/mix_probe's R=2 W=2 sc0 sc1 stream alone
  local n=$1 algo=$2 k=$3
  if [ $algo = mix ]; then
    timeout -s KILL 60 rocprofv3 --pmc ${PASSES[$k]} --kernel-trace -d $OUT/mix_n1_p$k -o run --output-format csv -- $R/tools/bin/mix_probe 512 22s > $OUT/mix_n1_p$k.log 2>&1
    local rc=$?
    echo "mix_n1_p$k rc=$rc"
    return $rc
  fi
  local port=$((22000 + RANDOM % 20000))
  local tag=${algo}_n${n}_p$k
  for r in $(seq 1 $((n-1))); do
    MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -k 5 60 $R/apps/bin/perf_test $r $n --sizes 1024 --iters 10 --warmup 2 > $OUT/$tag.r$r.log 2>&1 &
  done
  MINI_NCCL_ALGO=$algo MINI_NCCL_PORT=$port timeout -s KILL 60 rocprofv3 --pmc ${PASSES[$k]} --kernel-trace -d $OUT/$tag -o run --output-format csv -- $R/apps/bin/perf_test 0 $n --sizes 1024 --iters 10 --warmup 2 > $OUT/$tag.log 2>&1
  local rc=$?
  wait
  echo "$tag rc=$rc"
  return $rc
}
for cfg in ${CFGS:-2:read 4:read 2:ring 1:mix}; do
  for k in ${PASS_SEL:-$(seq 0 $((${#PASSES[@]} - 1)))}; do
    run ${cfg%%:*} ${cfg#*:} $k || exit 10
  done
done
echo counters-done
