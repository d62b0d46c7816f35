for b in 512 768 1024 1536 2048; do echo "== TN_BLOCKS=$b"; SLDM_TN_BLOCKS=$b timeout -k 10 120 python -u tools/kbench.py --dtype fp32 --edges 1000000 --only tn 2>&1 | grep "gemm_tn " ; done
