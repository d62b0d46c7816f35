#!/bin/bash
# Profiles for profiles/: run on the GPU box from the repo root, e.g.
#   gpurun -- 'tools/profile_round.sh r1'
# 1. rocprofv3 --kernel-trace --stats over the default bench command (C4);
# 2. separate PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit+miss) over
#    tools/kbench.py, one counter group per run (never combined with tracing).
# Each GPU step has its own time limit; the script stops at the first failure.
R=${1:?round tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$R" -o run \
  -- python3 "$ROOT/bench.py" --config c4 --steps 5 --warmup 2 --no-cpu-baseline \
  > "$OUT/prof_$R.log" 2>&1 || { echo "stats pass failed: $?"; exit 1; }
echo "stats pass ok"

i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${R}_$i" -o run \
    -- python3 "$ROOT/tools/kbench.py" --only gather,dense,nt,tn,post,gpost --reps 1 \
    > "$OUT/pmc_${R}_$i.log" 2>&1 || { echo "pmc pass $i ($ctr) failed: $?"; exit 1; }
  echo "pmc pass $i ($ctr) ok"
done
