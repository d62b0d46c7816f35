#!/bin/bash
# Real-workload diagnostics on the GPU box (repo root): the vehicle-step
# breakdown (tools/vehicle_breakdown.py) and rocprofv3 kernel stats of the
# vehicle and GRU bench lines.  usage: tools/prof_small.sh <tag>
R=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 240 python3 "$ROOT/tools/vehicle_breakdown.py" > "$OUT/vehicle_breakdown_$R.txt" 2>&1 \
  || { echo "breakdown failed: $?"; exit 1; }
echo "breakdown ok"
cd /tmp && export TMPDIR=/tmp
for cfg in vehicle gru; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${cfg}_$R" -o run \
    -- python3 "$ROOT/bench.py" --config $cfg --steps 20 --warmup 3 \
    > "$OUT/prof_${cfg}_$R.log" 2>&1 || { echo "$cfg stats pass failed: $?"; exit 1; }
  echo "$cfg stats pass ok"
done
