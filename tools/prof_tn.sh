# rocprof kernel stats of the fp32 dW path at C2 shapes for several block targets
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for blk in 128 256 512; do
  SLDM_TN_BLOCKS=$blk timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_tn_$blk -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --nodes 100000 --edges 1000000 --feat 128 --dtype fp32 --reps 20 --only tn > $GRAFT_REPO_ROOT/gpurun_out/prof_tn_$blk.log 2>&1 || exit 1
  grep gemm_tn $GRAFT_REPO_ROOT/gpurun_out/prof_tn_$blk.log
done
