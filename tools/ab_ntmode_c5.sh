# Gather cache-policy modes on the C5 (power-law) bench: SLDM_GATHER_NT = s / 0 / 1
mkdir -p gpurun_out
for r in 1 2; do for m in s 0 1; do
  echo "== c5 NT=$m run $r"
  SLDM_GATHER_NT=$m timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value']/1e9,4), d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})" || exit 1
done; done
for m in s 0; do
  echo "== c4 NT=$m"
  SLDM_GATHER_NT=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value']/1e9,4), d['ms_per_step'])" || exit 1
done
