"""Diagnostic: bf16 vs fp32 GPU SageBlock vs the CPU oracle, every tensor."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from _helpers import oracle_block, run_oracle  # noqa: E402
from oracle.sage_ref import random_graph  # noqa: E402
from sldm_sage import SageBlock  # noqa: E402


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return f"maxabs={float((a - b).abs().max()):.4g} relnorm={float((a - b).norm() / b.norm()):.3g} " \
           f"refmax={float(b.abs().max()):.3g}"


def run(dtype, hd, layers_only=None):
    n, e = 1000, 5000
    ei, x = random_graph(n, e, hd[0], seed=0)
    x = x.bfloat16().float()
    gout = torch.randn(n, hd[-1], generator=torch.Generator().manual_seed(2))
    gout = gout.bfloat16().float()
    ref = oracle_block(hd, 0.1)
    out_r, dx_r, gr = run_oracle(ref, x, ei, gout)
    blk = SageBlock(hd, None, 0.1)
    blk.load_state_dict(ref.state_dict())
    blk = blk.cuda()
    xg = x.cuda().to(dtype).requires_grad_(True)
    out = blk(xg, ei.cuda())
    out.backward(gout.cuda().to(dtype))
    print(f"--- {dtype} hdims={hd}")
    print("out ", rel(out, out_r))
    print("dx  ", rel(xg.grad, dx_r))
    for k, p in blk.named_parameters():
        print(f"{k:28s}", rel(p.grad, gr[k]))


for hd in ([16, 16], [16, 16, 16]):
    run(torch.float32, hd)
    run(torch.bfloat16, hd)
