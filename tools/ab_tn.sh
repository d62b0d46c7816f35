# dW (TN) A/B: ab/lib_tn0.so (previous) vs the in-tree library, C2 fp32 and C4 bf16
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "gemm or tn or sageblock" --timeout 120 --timeout-method thread > gpurun_out/tn_par.log 2>&1 || { tail -20 gpurun_out/tn_par.log; exit 1; }
tail -1 gpurun_out/tn_par.log
for r in 1 2; do
  for lib in ab/lib_tn0.so sldm-gnn_amd/sldm_sage/libsldm_sage.so; do
    echo "== $lib run $r (C2 fp32)"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only tn 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
