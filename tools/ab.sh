#!/bin/bash
# Same-box A/B of library builds (box-to-box variance, ~3-5 %, exceeds the
# effects measured): tools/kbench.py --only $1 with every ab/lib_*.so in turn,
# two rounds.  Usage: tools/ab.sh gather
ONLY=${1:?kbench --only list}
mkdir -p gpurun_out
for r in 1 2; do
  for lib in ab/lib_*.so; do
    echo "== $(basename $lib .so) run $r"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --only "$ONLY" 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done
done
