"""Where the vehicle-batch step goes (diagnostic): collate, per-batch CSR
build, SageBlock fwd + bwd on a cached graph, and the reference's ATen op
sequence on the same batch; plus a kernel-count trace of one step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from sldm_sage import SageBlock, graph_cache  # noqa: E402
from sldm_sage.data import collate  # noqa: E402
from sldm_sage.graph import build_graph  # noqa: E402


def tm(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(0)
pool = [bench._synthetic_pack(gen, dev, 250, 128) for _ in range(32)]
torch.manual_seed(0)
blk = SageBlock([128, 96, 96], 0.25, 0.1).to(dev).train()
b = collate([dict(p) for p in pool])
h, ei = b.x, b.edge_index
print("nodes", h.size(0), "edges", ei.size(1))
print("collate ms", tm(lambda: collate([dict(p) for p in pool])))
print("csr build ms", tm(lambda: build_graph(ei, h.size(0))))
g = build_graph(ei, h.size(0))


def ours():
    blk.zero_grad(set_to_none=True)
    x = h.detach().requires_grad_(True)
    blk(x, g).backward(torch.ones(h.size(0), 96, device=dev))


def ours_fwd():
    with torch.no_grad():
        blk(h, g)


print("sageblock fwd+bwd (graph cached) ms", tm(ours))
print("sageblock fwd only ms", tm(ours_fwd))
print("torch ops fwd+bwd ms", bench.torch_ops_gpu_baseline(blk, ei, h, torch.ones(h.size(0), 96, device=dev), 3, 20) * 1e3)
import cProfile  # noqa: E402
import pstats  # noqa: E402

torch.autograd.set_multithreading_enabled(False)     # backward on this thread: profiled
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    ours()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(40)
