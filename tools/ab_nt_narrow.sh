# Gather cache-policy modes on the feature-sliced multi-GPU row widths (C4 graph, F/W columns):
# F = 32 (W = 8, 64-B rows, 640 MB table) and F = 64 (W = 4, 128-B rows, 1.28 GB table)
mkdir -p gpurun_out
for r in 1 2; do for f in 32 64; do for m in 0 s 1; do
  echo "== F=$f NT=$m run $r"
  SLDM_GATHER_NT=$m timeout -k 10 200 python -u tools/kbench.py --feat $f --reps 5 --only gather 2>&1 | grep "gather_fwd" || exit 1
done; done; done
