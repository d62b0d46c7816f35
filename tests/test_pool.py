"""Graph-level readout: global mean / max / mean||max
pooling over the batch vector.

CPU: the oracle (oracle/pool_ref.py, PyG 2.7.0's CPU op sequence) against
hand-computed answers, including torch's amax tie rule.  GPU: the HIP path
(pool.hip through the C ABI) against the oracle -- fp32 forward and input
gradient bit-exact when every graph has <= 256 nodes (sequential fp32 sums,
one division, same tie divisor), 1e-5 relative for longer graphs (per-piece
partial sums), bf16 within 1e-2 of the range.
"""
from __future__ import annotations

import pytest
import torch

from oracle import pool_ref as R

DEV = "cuda:0"


# ------------------------------------------------------------ oracle (CPU) --
def test_oracle_known_answers():
    x = torch.tensor([[1.0, 0.0], [3.0, 0.0], [3.0, -1.0], [2.0, -2.0], [5.0, -3.0]],
                     requires_grad=True)
    b = torch.tensor([0, 0, 0, 1, 1])
    out = R.global_mean_max_pool(x, b, size=3)
    exp = torch.tensor([[7 / 3, -1 / 3, 3.0, 0.0], [3.5, -2.5, 5.0, -2.0], [0, 0, 0, 0]])
    torch.testing.assert_close(out.detach(), exp)
    out.backward(torch.ones_like(out))
    # mean part: 1/3 and 1/2; max part: ties split, and the max of 0 (column
    # 1, graph 0) is divided by ties + 1 (torch counts the zero `self`)
    exp_g = torch.tensor([[1 / 3, 1 / 3 + 1 / 3], [1 / 3 + 1 / 2, 1 / 3 + 1 / 3], [1 / 3 + 1 / 2, 1 / 3],
                          [1 / 2, 1 / 2 + 1], [1 / 2 + 1, 1 / 2]])
    torch.testing.assert_close(x.grad, exp_g)


def test_oracle_batch_none_first_argmax():
    x = torch.tensor([[1.0, 2.0], [3.0, 2.0]], requires_grad=True)
    out = R.global_max_pool(x, None)
    out.sum().backward()
    assert torch.equal(out.detach(), torch.tensor([[3.0, 2.0]]))
    assert torch.equal(x.grad, torch.tensor([[0.0, 1.0], [1.0, 0.0]]))


def test_oracle_matches_loop_formulation():
    g = torch.Generator().manual_seed(0)
    n, f, B = 200, 5, 7
    x = torch.randn(n, f, generator=g, dtype=torch.float64)
    b = torch.randint(0, B, (n,), generator=g)
    out = R.global_mean_max_pool(x, b, size=B + 1)
    for s in range(B + 1):
        rows = x[b == s]
        if rows.numel() == 0:
            assert torch.all(out[s] == 0)
            continue
        torch.testing.assert_close(out[s, :f], rows.mean(0))
        torch.testing.assert_close(out[s, f:], rows.max(0)[0])


# ------------------------------------------- host library (CPU tensors) --
@pytest.mark.parametrize("mode", ["mean", "max", "double"])
def test_cpu_pool_matches_oracle(mode):
    """sldm_sage pooling on CPU tensors (the reference's DEVICE='cpu' mode,
    libsldm_sage_cpu.so): forward bit-equal to the oracle's scatter order,
    gradients equal (ties, maxima of 0, empty graphs, batch=None)."""
    import sldm_sage
    fn = sldm_sage.global_pool(mode)
    ref = {"mean": R.global_mean_pool, "max": R.global_max_pool,
           "double": R.global_mean_max_pool}[mode]
    g = torch.Generator().manual_seed(3)
    n, f, B = 300, 7, 9
    x = torch.randn(n, f, generator=g)
    x[::5] = x[::5].round()                     # ties
    x[:, 2] = -x[:, 2].abs()
    x[::3, 2] = 0.0                             # maxima of exactly 0
    b = torch.randint(0, B - 1, (n,), generator=g)     # graph B-1 stays empty
    for batch, size in ((b, B), (torch.sort(b).values, None), (None, None)):
        xa = x.clone().requires_grad_(True)
        xb = x.clone().requires_grad_(True)
        out = fn(xa, batch, size) if batch is not None else fn(xa, None)
        want = ref(xb, batch, size)
        if batch is None:       # x.mean(0) sums pairwise on the CPU: another order
            torch.testing.assert_close(out, want, atol=1e-6, rtol=1e-6)
        else:
            assert torch.equal(out, want)
        go = torch.randn(want.shape, generator=torch.Generator().manual_seed(4))
        out.backward(go)
        want.backward(go)
        torch.testing.assert_close(xa.grad, xb.grad, atol=1e-6, rtol=1e-6)


# -------------------------------------------------------------- GPU parity --
def _batch(sizes, seed=0, shuffle=False):
    b = torch.cat([torch.full((s,), i, dtype=torch.int64) for i, s in enumerate(sizes)])
    if shuffle:
        b = b[torch.randperm(b.numel(), generator=torch.Generator().manual_seed(seed))]
    return b


def _check(x, b, mode, size=None, exact=True, tol=None):
    from sldm_sage import pool
    fn_g = {"mean": pool.global_mean_pool, "max": pool.global_max_pool,
            "double": pool.global_mean_max_pool}[mode]
    fn_r = {"mean": R.global_mean_pool, "max": R.global_max_pool,
            "double": R.global_mean_max_pool}[mode]
    xr = x.clone().requires_grad_(True)
    out_r = fn_r(xr.float() if x.dtype != torch.float32 else xr, b, size)
    gout = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(3))
    out_r.backward(gout)
    xg = x.to(DEV).requires_grad_(True)
    out_g = fn_g(xg, b.to(DEV) if b is not None else None, size)
    out_g.backward(gout.to(DEV, x.dtype))
    torch.cuda.synchronize()
    if exact:
        assert torch.equal(out_g.cpu(), out_r.detach().to(x.dtype)), "forward differs"
        assert torch.equal(xg.grad.cpu(), xr.grad), "input grad differs"
    else:
        rng_o = out_r.detach().abs().max().item()
        rng_g = xr.grad.abs().max().item()
        assert (out_g.cpu().float() - out_r.detach()).abs().max().item() <= tol * max(rng_o, 1e-6)
        assert (xg.grad.cpu().float() - xr.grad.float()).abs().max().item() <= tol * max(rng_g, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mean", "max", "double"])
@pytest.mark.parametrize("feat", [1, 6, 32, 96, 256, 1000])
def test_pool_fp32_bit_exact(mode, feat):
    b = _batch([37, 0, 256, 1, 120, 200])     # an empty graph in the middle, one full piece
    x = torch.randn(b.numel(), feat, generator=torch.Generator().manual_seed(feat))
    _check(x, b, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["max", "double"])
def test_pool_ties_and_zero_max(mode):
    """ReLU-like input: many exact zeros and ties, the max-of-0 divisor rule."""
    b = _batch([50, 3, 200, 7])
    g = torch.Generator().manual_seed(1)
    x = torch.randint(-3, 3, (b.numel(), 64), generator=g).float().clamp(min=0)   # {0, 1, 2}
    _check(x, b, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mean", "max", "double"])
def test_pool_unsorted_batch_and_size(mode):
    b = _batch([10, 40, 0, 25], shuffle=True)
    x = torch.randn(b.numel(), 48, generator=torch.Generator().manual_seed(2))
    _check(x, b, mode, size=6)      # two trailing empty graphs


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mean", "max"])
def test_pool_batch_none(mode):
    x = torch.randn(500, 40, generator=torch.Generator().manual_seed(4))
    x[7, 3] = x[:, 3].max() + 1.0
    x[9, 3] = x[7, 3]                   # tie: x.max routes to the first row (7)
    # x.mean sums pairwise on the CPU: forward within fp32 rounding
    _check(x, None, mode, exact=(mode == "max"), tol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mean", "double"])
def test_pool_long_graph_pieces(mode):
    """Graphs far longer than a piece (one full-graph batch of 100k nodes)."""
    b = _batch([100_000, 3, 70_001])
    x = torch.randn(b.numel(), 64, generator=torch.Generator().manual_seed(5))
    _check(x, b, mode, exact=False, tol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mean", "max", "double"])
def test_pool_bf16(mode):
    b = _batch([30, 200, 1, 64])
    x = torch.randn(b.numel(), 128, generator=torch.Generator().manual_seed(6)).bfloat16()
    _check(x, b, mode, exact=False, tol=1e-2)
