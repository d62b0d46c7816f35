"""CPU tests of the oracle itself (no GPU).

The reference ships no tests or fixtures and its path (torch_geometric) cannot
run here, so the oracle is pinned by (a) an independent fp64 dense-matrix
formulation, (b) hand-computed known answers, (c) the C restatement of the
addressing, and (d) regression against the committed golden fixtures.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch

from _helpers import ref_agg_mean_f32, ref_csr
from oracle import dense_ref
from oracle.sage_ref import (RefSageBlock, khop_subgraph, pyg_sage_aggregate, pyg_scatter_mean,
                             random_graph, set_synthetic_params)


def _params(ref):
    out = []
    for conv, post in zip(ref.convs, ref.posts):
        out.append(dict(Wl=conv.lin_l.weight.detach().double().numpy(),
                        bl=conv.lin_l.bias.detach().double().numpy(),
                        Wr=conv.lin_r.weight.detach().double().numpy(),
                        g=post[0].weight.detach().double().numpy(),
                        b=post[0].bias.detach().double().numpy()))
    return out


EDGE_CASES = {
    "random": lambda n: random_graph(n, 4 * n, 1, seed=n)[0],
    "empty": lambda n: torch.empty(2, 0, dtype=torch.long),
    "dup_self_isolated": lambda n: torch.tensor([[0, 0, 2, 2, 3, 4], [1, 1, 2, 3, 3, 1]]),
    "star_in": lambda n: torch.stack([torch.arange(1, n), torch.zeros(n - 1, dtype=torch.long)]),
}


@pytest.mark.parametrize("case", list(EDGE_CASES))
@pytest.mark.parametrize("hdims,ns", [([6, 5, 4], 0.1), ([6, 8], None), ([6, 6, 6, 6], 0.2)])
def test_oracle_matches_dense_fp64(case, hdims, ns):
    n = 40
    ei = EDGE_CASES[case](n)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(n, hdims[0], generator=gen)
    gout = torch.randn(n, hdims[-1], generator=gen)
    ref = RefSageBlock(hdims, None, ns)
    set_synthetic_params(ref, seed=2)
    with torch.no_grad():  # non-trivial LayerNorm affine
        for post in ref.posts:
            post[0].weight.uniform_(0.5, 1.5, generator=gen)
            post[0].bias.uniform_(-0.5, 0.5, generator=gen)
    xr = x.clone().requires_grad_(True)
    out = ref(xr, ei)
    out.backward(gout)
    params = _params(ref)
    d_out, saved = dense_ref.forward(x.double().numpy(), ei.numpy(), params, ns)
    d_dx, d_grads = dense_ref.backward(gout.double().numpy(), params, saved)
    tol = dict(atol=2e-5, rtol=2e-5)
    np.testing.assert_allclose(out.detach().numpy(), d_out, **tol)
    np.testing.assert_allclose(xr.grad.numpy(), d_dx, **tol)
    for i, (conv, post) in enumerate(zip(ref.convs, ref.posts)):
        np.testing.assert_allclose(conv.lin_l.weight.grad.numpy(), d_grads[i]["Wl"], **tol)
        np.testing.assert_allclose(conv.lin_l.bias.grad.numpy(), d_grads[i]["bl"], **tol)
        np.testing.assert_allclose(conv.lin_r.weight.grad.numpy(), d_grads[i]["Wr"], **tol)
        np.testing.assert_allclose(post[0].weight.grad.numpy(), d_grads[i]["g"], **tol)
        np.testing.assert_allclose(post[0].bias.grad.numpy(), d_grads[i]["b"], **tol)


def test_known_answer_mean_aggregation():
    """Hand-computed: edges 0->2, 1->2, 2->0, 1->2 (duplicate counted), 3 isolated."""
    x = torch.tensor([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0], [7.0, 8.0]])
    ei = torch.tensor([[0, 1, 2, 1], [2, 2, 0, 2]])
    agg = pyg_sage_aggregate(x, ei)
    expect = torch.tensor([[5.0, 6.0], [0.0, 0.0], [(1 + 3 + 3) / 3, (2 + 4 + 4) / 3],
                           [0.0, 0.0]])
    assert torch.equal(agg, expect)
    assert torch.equal(pyg_scatter_mean(x[ei[0]], ei[1], 4), expect)


def test_known_answer_block():
    """One layer, W_l = I, b = 0, W_r = 0, LN affine identity, LeakyReLU(0.1)."""
    x = torch.tensor([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]])
    ei = torch.tensor([[2, 0, 1], [0, 2, 2]])
    blk = RefSageBlock([2, 2], None, 0.1)
    with torch.no_grad():
        blk.convs[0].lin_l.weight.copy_(torch.eye(2))
        blk.convs[0].lin_l.bias.zero_()
        blk.convs[0].lin_r.weight.zero_()
    out = blk(x, ei)
    # node 0: agg [5,6] -> LN [-1,1]*0.5/sqrt(0.25+1e-5); node 1: [0,0] -> 0; node 2: [2,3]
    s = 0.5 / (0.25 + 1e-5) ** 0.5
    expect = torch.tensor([[-0.1 * s, s], [0.0, 0.0], [-0.1 * s, s]])
    torch.testing.assert_close(out.detach(), expect, atol=1e-7, rtol=1e-6)


def test_oracle_raises_on_bad_index():
    x = torch.randn(3, 2)
    with pytest.raises(IndexError):
        pyg_sage_aggregate(x, torch.tensor([[0, 3], [1, 1]]))
    assert ref_csr(torch.tensor([[0, 3], [1, 1]]), 3) is None
    assert ref_csr(torch.tensor([[0, -1], [1, 1]]), 3) is None


@pytest.mark.parametrize("n,e", [(1, 0), (5, 0), (1, 7), (100, 1000), (3000, 30000)])
def test_c_csr_oracle_is_stable_sort(n, e):
    ei, _ = random_graph(n, e, 1, seed=e)
    rp, col, trp, tcol = ref_csr(ei, n)
    order = torch.argsort(ei[1], stable=True)
    assert np.array_equal(col, ei[0][order].numpy().astype(np.int32))
    assert np.array_equal(rp, torch.searchsorted(ei[1][order], torch.arange(n + 1)).numpy())
    t_order = torch.argsort(ei[0], stable=True)
    assert np.array_equal(tcol, ei[1][t_order].numpy().astype(np.int32))
    assert np.array_equal(trp, torch.searchsorted(ei[0][t_order], torch.arange(n + 1)).numpy())


@pytest.mark.parametrize("n,e,f", [(200, 1000, 16), (50, 0, 8), (300, 3000, 33)])
def test_c_agg_bit_equal_to_pyg_restatement(n, e, f):
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)  # scatter_add_ accumulation order per output element
    try:
        ei, x = random_graph(n, e, f, seed=f)
        rp, col, _, _ = ref_csr(ei, n)
        assert torch.equal(ref_agg_mean_f32(x, rp, col), pyg_sage_aggregate(x, ei))
    finally:
        torch.set_num_threads(nthreads)


def test_khop_subgraph_reproduces_full_graph():
    """The size-independent full-scale parity device used by the GPU tests."""
    n, e, hd = 3000, 15000, [8, 8, 8]
    ei, x = random_graph(n, e, hd[0], seed=11)
    ref = RefSageBlock(hd, None, 0.1)
    set_synthetic_params(ref, seed=1)
    targets = torch.tensor([5, 17, 2999, 1500])
    gfull = torch.zeros(n, hd[-1])
    gfull[targets] = torch.randn(len(targets), hd[-1], generator=torch.Generator().manual_seed(1))
    xr = x.clone().requires_grad_(True)
    out = ref(xr, ei)
    out.backward(gfull)
    full_grads = {k: p.grad.clone() for k, p in ref.named_parameters()}
    nodes, sub, tpos = khop_subgraph(ei, targets, len(hd) - 1, n)
    ref.zero_grad()
    xs = x[nodes].clone().requires_grad_(True)
    out_s = ref(xs, sub)
    out_s.backward(gfull[nodes])
    torch.testing.assert_close(out_s[tpos], out[targets], atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(xs.grad, xr.grad[nodes], atol=1e-6, rtol=1e-6)
    assert xr.grad.abs().sum() == pytest.approx(xs.grad.abs().sum().item(), rel=1e-5)
    for k, p in ref.named_parameters():
        torch.testing.assert_close(p.grad, full_grads[k], atol=1e-5, rtol=1e-5)


def _golden_files():
    return sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.parametrize("fn", _golden_files(), ids=os.path.basename)
def test_golden_fixture_matches_oracle(fn):
    z = np.load(fn)
    hdims = [int(v) for v in z["hdims"]]
    ns = float(z["negative_slope"]) if z["has_slope"] else None
    ref = RefSageBlock(hdims, None, ns)
    ref.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")})
    xr = torch.from_numpy(z["x"]).clone().requires_grad_(True)
    out = ref(xr, torch.from_numpy(z["edge_index"]))
    out.backward(torch.from_numpy(z["gout"]))
    # Sums over all rows (weight grads) depend on the CPU thread count's
    # reduction order: compare relative to each tensor's scale.
    tol = dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out.detach(), torch.from_numpy(z["out"]), **tol)
    torch.testing.assert_close(xr.grad, torch.from_numpy(z["dx"]), **tol)
    for k, p in ref.named_parameters():
        g = torch.from_numpy(z["grad." + k])
        s = max(1.0, g.abs().max().item())
        torch.testing.assert_close(p.grad / s, g / s, atol=5e-5, rtol=5e-5)


# ------------------------------------------------- bf16-storage oracle --
@pytest.mark.parametrize("case", list(EDGE_CASES))
@pytest.mark.parametrize("hdims,ns", [([6, 5, 4], 0.1), ([6, 8], None), ([6, 6, 6, 6], 0.2)])
def test_bf16_oracle_unrounded_equals_fp32_oracle(case, hdims, ns):
    """oracle/sage_bf16_ref.py with storage rounding off is the plain
    reference: its hand-written backward must equal sage_ref's autograd."""
    from oracle.sage_bf16_ref import block_params, sageblock_fwd_bwd
    n = 40
    ei = EDGE_CASES[case](n)
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(n, hdims[0], generator=gen)
    gout = torch.randn(n, hdims[-1], generator=gen)
    ref = RefSageBlock(hdims, None, ns)
    set_synthetic_params(ref, seed=2)
    with torch.no_grad():
        for post in ref.posts:
            post[0].weight.uniform_(0.5, 1.5, generator=gen)
            post[0].bias.uniform_(-0.5, 0.5, generator=gen)
    xr = x.clone().requires_grad_(True)
    out_r = ref(xr, ei)
    out_r.backward(gout)
    out, dx, grads = sageblock_fwd_bwd(block_params(ref), x, ei, gout, ns, store=None)
    tol = dict(atol=2e-5, rtol=2e-5)
    torch.testing.assert_close(out, out_r.detach(), **tol)
    torch.testing.assert_close(dx, xr.grad, **tol)
    for k, p in ref.named_parameters():
        torch.testing.assert_close(grads[k], p.grad, **tol, msg=lambda m: f"{k}: {m}")


def test_bf16_oracle_rounds_where_stored():
    """With rounding on: outputs and the input grad are bf16 values, and the
    result stays within bf16 resolution of the fp32 reference."""
    from oracle.sage_bf16_ref import block_params, branch_margin, sageblock_fwd_bwd
    hdims = [16, 16, 16]
    ei, x = random_graph(300, 1500, 16, seed=7)
    x = x.bfloat16().float()
    gout = torch.randn(300, 16, generator=torch.Generator().manual_seed(8)).bfloat16().float()
    ref = RefSageBlock(hdims, None, 0.1)
    set_synthetic_params(ref, seed=2)
    out, dx, grads = sageblock_fwd_bwd(block_params(ref), x, ei, gout, 0.1)
    assert torch.equal(out, out.bfloat16().float()) and torch.equal(dx, dx.bfloat16().float())
    out32, dx32, _ = sageblock_fwd_bwd(block_params(ref), x, ei, gout, 0.1, store=None)
    s = out32.abs().max()
    assert (out - out32).abs().max() < 2e-2 * s
    assert 0 < branch_margin(block_params(ref), x, ei, 0.1) < 1e-2


# --------------------------------------------------------------- GRU oracle --
@pytest.mark.parametrize("batch_first,bias,h0", [(True, True, False), (False, True, True),
                                                 (True, False, True)])
def test_gru_oracle_matches_torch_gru(batch_first, bias, h0):
    """oracle/gru_ref.py (aten's GRU cell unrolled) equals torch.nn.GRU on CPU,
    forward and every gradient (the reference's own op, grusage.py:66-71)."""
    from oracle.gru_ref import gru_ref
    torch.manual_seed(0)
    N, T, I, H = 7, 9, 6, 16
    gru = torch.nn.GRU(I, H, 1, bias=bias, batch_first=batch_first)
    x = torch.randn((N, T, I) if batch_first else (T, N, I), requires_grad=True)
    hx = torch.randn(1, N, H, requires_grad=True) if h0 else None
    out, hn = gru(x, hx)
    g1, g2 = torch.randn_like(out), torch.randn_like(hn)
    (out * g1).sum().add((hn * g2).sum()).backward()
    ref_grads = [p.grad.clone() for p in gru.parameters()] + [x.grad.clone()]
    if h0:
        ref_grads.append(hx.grad.clone())
    params = [p.detach().clone().requires_grad_(True) for p in gru.parameters()]
    x2 = x.detach().clone().requires_grad_(True)
    hx2 = hx.detach().clone().requires_grad_(True) if h0 else None
    w_ih, w_hh = params[0], params[1]
    b_ih, b_hh = (params[2], params[3]) if bias else (None, None)
    out2, hn2 = gru_ref(x2, w_ih, w_hh, b_ih, b_hh, hx2, batch_first)
    (out2 * g1).sum().add((hn2 * g2).sum()).backward()
    torch.testing.assert_close(out2, out, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(hn2, hn, atol=1e-6, rtol=1e-5)
    got = [p.grad for p in params] + [x2.grad] + ([hx2.grad] if h0 else [])
    for a, b in zip(got, ref_grads):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
