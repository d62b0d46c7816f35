mkdir -p gpurun_out
for t in 1 2 3; do
  SLDM_SAGE_LIB=$PWD/ab/lib_nt$t.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "gemm or dense or sageblock" --timeout 120 --timeout-method thread > gpurun_out/nt_t$t.log 2>&1 || { echo "parity fail $t"; tail -20 gpurun_out/nt_t$t.log; exit 1; }
  tail -1 gpurun_out/nt_t$t.log
done
for r in 1 2; do for t in 0 1 2 3; do
  echo "== nt$t run $r"
  SLDM_SAGE_LIB=$PWD/ab/lib_nt$t.so timeout -k 10 200 python -u tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only dense,nt 2>&1 | grep -v amdgpu.ids || exit 1
done; done
