#!/bin/bash
# post_bwd A/B: tests on the default library, then kbench post with the
# default and each ab/lib_*.so (same box).
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "post or sageblock" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
for r in 1 2; do
  echo "== default run $r"; timeout -k 10 200 python -u tools/kbench.py --only ${1:-post} 2>&1 | grep -v amdgpu.ids
  for lib in ab/lib_*.so; do
    echo "== $(basename $lib .so) run $r"
    SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/kbench.py --only ${1:-post} 2>&1 | grep -v amdgpu.ids
  done
done
