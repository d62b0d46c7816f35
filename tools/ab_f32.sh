#!/bin/bash
# Same-box A/B of library builds on the fp32 dense kernels: tools/kbench.py
# --dtype fp32 --only dense,nt with every ab/lib_*.so in turn, two rounds.
mkdir -p gpurun_out
for r in 1 2; do
  for lib in ab/lib_*.so; do
    echo "== $(basename $lib .so) run $r"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --dtype fp32 --edges 1000000 \
      --only "${1:-dense,nt}" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
