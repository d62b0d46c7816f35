"""Step time of a bench config with and without the per-op HIP-event timing
hook, and the CPU time per step (diagnostic: is the step host-bound?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from sldm_sage import SageBlock, ops  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
n, e, f, L, dtype, _ = cfg
dev = torch.device("cuda", 0)
ei, x = bench.make_graph(n, e, f, dtype, dev)
torch.manual_seed(0)
blk = SageBlock([f] * (L + 1), dropout=0.25, negative_slope=0.1).to(dev).train()
gout = torch.randn(n, f, device=dev).to(dtype)


def step():
    blk.zero_grad(set_to_none=True)
    xr = x.detach().requires_grad_(True)
    blk(xr, ei).backward(gout)


def run(k=30):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0, c0 = time.perf_counter(), time.process_time()
    for _ in range(k):
        step()
    c1 = time.process_time()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3, (c1 - c0) / k * 1e3


print("no hook: ms/step %.3f  cpu ms/step %.3f" % run())
timer = bench.KernelTimer()
ops.set_timing_hook(timer)
print("hook:    ms/step %.3f  cpu ms/step %.3f" % run())
ops.set_timing_hook(None)
s = timer.summary()
print("kernel sum ms/step", sum(v["avg_ms"] * v["launches"] for v in s.values()) / 35)
