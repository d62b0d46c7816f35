# dW (TN) A/B: ab/lib_tn0.so (previous) vs the in-tree library; rocprof of slab_reduce
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tn_par.log 2>&1 || { tail -20 gpurun_out/tn_par.log; exit 1; }
tail -1 gpurun_out/tn_par.log
for r in 1 2; do
  for lib in ab/lib_tn0.so sldm-gnn_amd/sldm_sage/libsldm_sage.so; do
    for blk in 0 256; do
      echo "== $lib blocks=$blk run $r (C2 fp32)"
      SLDM_TN_BLOCKS=$blk SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only tn 2>&1 | grep -v amdgpu.ids || exit 1
    done
    echo "== $lib run $r (C4 bf16)"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --reps 5 --only tn 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_tn_new -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only tn > $GRAFT_REPO_ROOT/gpurun_out/prof_tn_new.log 2>&1
