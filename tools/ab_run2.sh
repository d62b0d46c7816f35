set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "post" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
timeout -k 10 200 python -u tools/kbench.py --only postring,dense1 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/kbench.py --only postring 2>&1 | grep -v amdgpu.ids
