#!/bin/bash
# One GPU call: default-suite check of the current library, the stream-kernel
# tests on an A/B variant, then the same-box kernel A/B (tools/ab.sh).
set -e
[ -n "$FULL" ] && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
for lib in ab/lib_f_da8.so; do
  SLDM_SAGE_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -k "stream_dense_fwd and stream or sageblock_bf16" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
done
timeout -k 10 900 tools/ab.sh ${1:-dense1}
