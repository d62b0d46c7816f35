#!/bin/bash
# Stall-breakdown PMC passes for the dense kernels (diagnostic): one counter
# group per rocprofv3 run (never combined with tracing), each under its own
# time limit; stops at the first failure.  Usage (GPU box, repo root):
#   [KB_ARGS="--nodes .. --dtype fp32"] tools/pmc_stalls.sh <tag> [kbench --only list]
R=${1:?tag}; ONLY=${2:-dense,nt,tn}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/stall_${R}_$i" -o run \
    -- python3 "$ROOT/tools/kbench.py" --only "$ONLY" --reps 1 $KB_ARGS \
    > "$OUT/stall_${R}_$i.log" 2>&1 || { echo "pass $i failed: $?"; exit 1; }
  echo "pass $i ok"
done
