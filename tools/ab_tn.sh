# dW (TN) A/B: ab/lib_tn0.so (previous) vs ab/lib_tn1.so, C2 fp32 and the C4 bf16 tile path
mkdir -p gpurun_out
SLDM_SAGE_LIB=$PWD/ab/lib_tn1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tn_par.log 2>&1 || { tail -20 gpurun_out/tn_par.log; exit 1; }
tail -1 gpurun_out/tn_par.log
for r in 1 2; do for lib in ab/lib_tn0.so ab/lib_tn1.so; do
  echo "== $lib run $r (C2 fp32)"
  SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only tn 2>&1 | grep "gemm_tn" || exit 1
  echo "== $lib run $r (C4 bf16)"
  SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --reps 3 --only tn 2>&1 | grep "gemm_tn" || exit 1
done; done
