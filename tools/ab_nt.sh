# fp32 NT A/B at C2 shapes: ab/lib_nt_old.so vs the in-tree library (+ GPU parity of the new one)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_par.log 2>&1 || { tail -30 gpurun_out/nt_par.log; exit 1; }
tail -1 gpurun_out/nt_par.log
for r in 1 2; do for lib in ab/lib_nt_old.so sldm-gnn_amd/sldm_sage/libsldm_sage.so; do
  echo "== $lib run $r"
  SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only dense,nt 2>&1 | grep -v amdgpu.ids || exit 1
done; done
timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline > gpurun_out/b2.log 2>&1
