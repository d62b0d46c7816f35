#!/bin/bash
# Every bench line of a round (GPU box, repo root): the default C4 line (CPU
# baseline at E/10), the locality variant, C5, C3 and C2 / C1 with CPU
# baselines on the full graph, the fp32 C4 line and the real-workload lines.
# Each run has its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r2}
: > gpurun_out/lines_$TAG.jsonl
for args in "" "--graph local --no-cpu-baseline" "--config c5 --cpu-frac 10" \
            "--config c3 --cpu-frac 1" "--config c2 --cpu-frac 1" "--config c1 --cpu-frac 1" \
            "--config c4 --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline" \
            "--config vehicle --steps 20 --warmup 5" "--config map --steps 50 --warmup 5" \
            "--config gru --steps 10 --warmup 3"; do
  timeout -k 10 400 python -u bench.py $args > gpurun_out/line.log 2>&1 || { echo "bench $args failed: $?"; tail -5 gpurun_out/line.log; exit 1; }
  grep -o '^{.*}' gpurun_out/line.log | tail -1 >> gpurun_out/lines_$TAG.jsonl
  echo "ok: $args"
done
