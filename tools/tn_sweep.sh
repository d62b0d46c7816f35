#!/bin/bash
# Split-count sweep of the fp32 dW (TN) kernel at C4 (diagnostic): SLDM_TN_BLOCKS =
# 512 .. 2048 through tools/kbench.py --dtype fp32 --only tn, one box.
for b in 512 768 1024 1536 2048; do echo "== TN_BLOCKS=$b"; SLDM_TN_BLOCKS=$b timeout -k 10 120 python -u tools/kbench.py --dtype fp32 --edges 1000000 --only tn 2>&1 | grep "gemm_tn " ; done
