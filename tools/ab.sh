#!/bin/bash
# A/B of two builds of libsldm_sage.so in one GPU call (box-to-box variance is
# ~3-5 %, larger than the effects measured): kbench --only $1 alternating
# ab/lib_old.so and ab/lib_new.so, twice each.  Usage: tools/ab.sh gather
ONLY=${1:?kbench --only list}
mkdir -p gpurun_out
for r in 1 2; do
  for v in old new; do
    echo "== $v run $r"
    SLDM_SAGE_LIB=$PWD/ab/lib_$v.so timeout -k 10 200 python -u tools/kbench.py --only "$ONLY" 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done
done
