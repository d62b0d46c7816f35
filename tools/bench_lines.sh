set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r1}
: > gpurun_out/lines_$TAG.jsonl
for args in "" "--graph local --no-cpu-baseline" "--config c5 --no-cpu-baseline" "--config c3 --no-cpu-baseline" "--config c2"; do
  timeout -k 10 400 python -u bench.py $args > gpurun_out/line.log 2>&1 || { echo "bench $args failed: $?"; tail -5 gpurun_out/line.log; exit 1; }
  grep -o '^{.*}' gpurun_out/line.log | tail -1 >> gpurun_out/lines_$TAG.jsonl
  echo "ok: $args"
done
