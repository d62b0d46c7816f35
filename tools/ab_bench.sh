#!/bin/bash
# Same-box A/B of whole bench lines: bench.py <args> with every ab/lib_*.so
# in turn, two rounds; prints value, ms/step and the per-kernel averages.
# Usage: tools/ab_bench.sh "<bench args>"
ARGS=${1:-}
mkdir -p gpurun_out
for r in 1 2; do
  for lib in ab/lib_*.so; do
    echo "== $(basename $lib .so) run $r"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline \
      --no-torch-baseline $ARGS > gpurun_out/abb.log 2>&1 || { tail -5 gpurun_out/abb.log; exit 1; }
    python - <<'PY'
import json
for l in open("gpurun_out/abb.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(round(d["value"] / 1e9, 4), "G", d["ms_per_step"], "ms",
              {k: v["avg_ms"] for k, v in d.get("kernels", {}).items()})
PY
  done
done
