# Gather cache-policy modes on the C4 bench, uniform and locality graphs:
# SLDM_GATHER_NT = 1 (loads + stores non-temporal), s (stores only), 0 (none)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "gather" --timeout 120 --timeout-method thread > gpurun_out/gpar.log 2>&1 || { tail -30 gpurun_out/gpar.log; exit 1; }
tail -1 gpurun_out/gpar.log
for r in 1 2; do for g in uniform local; do for m in 1 s 0; do
  echo "== $g NT=$m run $r"
  SLDM_GATHER_NT=$m timeout -k 10 300 python -u bench.py --graph $g --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value']/1e9,4), d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if 'gather' in k})" || exit 1
done; done; done
