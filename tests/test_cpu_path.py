"""The SageBlock on CPU tensors (the reference's DEVICE='cpu' mode, main.py:58):
native host kernels (sldm_sage/cpu.py, csrc_cpu/sage_cpu.cpp) against the
oracle (oracle/sage_ref.py), forward and every gradient within 1e-4, plus the
drop-in contract (bad ids raise, dropout reproducible under manual_seed)."""
from __future__ import annotations

import pytest
import torch

from _helpers import oracle_block, run_oracle


@pytest.mark.parametrize("n,e,hdims,ns", [(1000, 5000, [16, 16, 16], 0.1),
                                          (600, 4000, [128, 96, 96], 0.1),
                                          (500, 2500, [16, 32, 32], None),
                                          (50, 0, [8, 8], 0.1)])
def test_cpu_sageblock_matches_oracle(n, e, hdims, ns):
    from oracle.sage_ref import random_graph
    from sldm_sage import SageBlock
    ei, x = random_graph(n, e, hdims[0], seed=3)
    gout = torch.randn(n, hdims[-1], generator=torch.Generator().manual_seed(4))
    ref = oracle_block(hdims, ns)
    with torch.no_grad():
        for post in ref.posts:
            post[0].bias.uniform_(-0.3, 0.3)
    out_r, dx_r, gr = run_oracle(ref, x, ei, gout)
    blk = SageBlock(hdims, None, ns)
    blk.load_state_dict(ref.state_dict())
    xr = x.clone().requires_grad_(True)
    out = blk(xr, ei)
    out.backward(gout)
    torch.testing.assert_close(out.detach(), out_r, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(xr.grad, dx_r, atol=1e-4, rtol=1e-4)
    for k, p in blk.named_parameters():
        s = max(1.0, gr[k].abs().max().item())
        torch.testing.assert_close(p.grad / s, gr[k] / s, atol=1e-4, rtol=1e-4)


def test_cpu_sageblock_contract():
    from sldm_sage import SageBlock
    blk = SageBlock([8, 8], dropout=0.25, negative_slope=0.1).train()
    x = torch.randn(20, 8)
    with pytest.raises(IndexError):
        blk(x, torch.tensor([[0, 25], [1, 2]]))
    ei = torch.randint(0, 20, (2, 60), generator=torch.Generator().manual_seed(1))
    torch.manual_seed(3)
    a = blk(x, ei)
    b = blk(x, ei)
    torch.manual_seed(3)
    assert torch.equal(blk(x, ei), a) and not torch.equal(a, b)
    kept = (a != 0).float().mean().item()
    assert 0.6 < kept < 0.9
    with torch.inference_mode():                 # rcv.py's inference mode
        blk.eval()
        out = blk(x, ei)
        assert out.shape == (20, 8)


def test_cpu_csr_build_ignores_padding_edges():
    """Edges (N, N) are padding on the CPU path as on the GPU: the block's
    output on a padded edge_index equals the output on the real edges."""
    from sldm_sage import SageBlock, cpu
    from oracle.sage_ref import random_graph
    n, e = 300, 2000
    ei, x = random_graph(n, e, 16, seed=9)
    padded = torch.cat([ei[:, :1000], torch.full((2, 57), n, dtype=torch.int64), ei[:, 1000:]], 1)
    a, b = cpu.csr_build(ei, n), cpu.csr_build(padded, n)
    for u, v, k in zip(a, b, (n + 1, e, n + 1, e)):
        assert torch.equal(u[:k], v[:k])
    torch.manual_seed(0)
    blk = SageBlock([16, 32], None, 0.1).eval()
    with torch.no_grad():
        assert torch.equal(blk(x, ei), blk(x, padded))
    with pytest.raises(IndexError):
        cpu.csr_build(torch.tensor([[n], [0]]), n)
