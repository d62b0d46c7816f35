#!/bin/bash
# Clock / MFMA-busy comparison of library builds on the fp32 forward kernel:
# one counter group per rocprofv3 run (counters only, no tracing), per
# ab/lib_*.so (diagnostic; kbench prints the kernel times itself).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in $ROOT/ab/lib_*.so; do
  n=$(basename $lib .so)
  i=0
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS" \
             "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT"; do
    i=$((i + 1))
    SLDM_SAGE_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/f32ab_${n}_$i" -o run \
      -- python3 "$ROOT/tools/kbench.py" --only dense1 --reps 1 --dtype fp32 --edges 1000000 \
      > "$OUT/f32ab_${n}_$i.log" 2>&1 || { echo "$n pass $i failed: $?"; tail -3 "$OUT/f32ab_${n}_$i.log"; exit 1; }
    echo "$n pass $i ok"
  done
done
