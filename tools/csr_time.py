"""Time ops.csr_build (with and without the transpose CSR) at per-batch and
large graph sizes on the GPU: python tools/csr_time.py"""
import sys, torch
sys.path.insert(0, "sldm-gnn_amd")
from sldm_sage import ops
dev = torch.device("cuda", 0)
def timed(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
for n, e in [(250, 5000), (8000, 160000), (8000, 20000), (100000, 1000000), (1000000, 10000000)]:
    ei = torch.randint(0, n, (2, e), device=dev)
    t = timed(lambda: ops.csr_build(ei, n, True))
    t1 = timed(lambda: ops.csr_build(ei, n, False))
    print(f"N={n} E={e}: csr_build with transpose {t:.3f} ms, forward only {t1:.3f} ms", flush=True)
