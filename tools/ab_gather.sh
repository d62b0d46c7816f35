# Non-temporal gather A/B (SLDM_GATHER_NT=0 vs 1) at C4 and at C3's table size, GPU parity
# with the default (auto) selection, then the C4 bench.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpar.log 2>&1 || { tail -30 gpurun_out/gpar.log; exit 1; }
tail -1 gpurun_out/gpar.log
for r in 1 2; do for nt in 0 1; do
  echo "== C4 NT=$nt run $r"
  SLDM_GATHER_NT=$nt timeout -k 10 200 python -u tools/kbench.py --only gather,gpost 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== C3-size NT=$nt run $r"
  SLDM_GATHER_NT=$nt timeout -k 10 200 python -u tools/kbench.py --nodes 1000000 --edges 10000000 --reps 20 --only gather,gpost 2>&1 | grep -v amdgpu.ids || exit 1
done; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b4.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b3.log 2>&1
