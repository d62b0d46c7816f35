"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact for the integer CSR build and for the fp32/bf16 aggregation sums
(same fp32 accumulation order as the reference's CPU scatter_add_); within
1e-4 (fp32) / 1e-2 (bf16) for the full SageBlock forward and every gradient.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest
import torch

from _helpers import TOL, oracle_block, ref_agg_mean_f32, ref_csr, run_oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(n, e, f, seed=0):
    from oracle.sage_ref import random_graph
    return random_graph(n, e, f, seed=seed)


# ------------------------------------------------------------------- CSR --
@pytest.mark.parametrize("n,e", [(1, 0), (7, 0), (1, 5), (1000, 5000), (3000, 40000),
                                 (100_000, 1_000_000)])
@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
def test_csr_build_bit_exact(n, e, idx_dtype):
    from sldm_sage import build_graph
    ei, _ = _graph(n, e, 1, seed=n + e)
    g = build_graph(ei.to(DEV, idx_dtype), n)
    rp, col, trp, tcol = ref_csr(ei, n)
    assert np.array_equal(g.rowptr.cpu().numpy(), rp)
    assert np.array_equal(g.col.cpu().numpy(), col)
    assert np.array_equal(g.t_rowptr.cpu().numpy(), trp)
    assert np.array_equal(g.t_col.cpu().numpy(), tcol)


def test_csr_power_law_hub():
    """One node with in-degree 10k plus duplicates and self loops."""
    from sldm_sage import build_graph
    n = 20_000
    gen = torch.Generator().manual_seed(5)
    src = torch.randint(0, n, (30_000,), generator=gen)
    dst = torch.randint(0, n, (30_000,), generator=gen)
    dst[:10_000] = 1234
    src[10_000:10_100] = dst[10_000:10_100]          # self loops
    ei = torch.stack([src, dst])
    ei = torch.cat([ei, ei[:, :500]], 1)             # duplicates
    g = build_graph(ei.to(DEV), n)
    rp, col, trp, tcol = ref_csr(ei, n)
    assert np.array_equal(g.rowptr.cpu().numpy(), rp) and np.array_equal(g.col.cpu().numpy(), col)
    assert np.array_equal(g.t_rowptr.cpu().numpy(), trp) and np.array_equal(g.t_col.cpu().numpy(), tcol)


@pytest.mark.parametrize("bad", [-1, 50])
def test_csr_bad_index_raises(bad):
    from sldm_sage import build_graph
    ei = torch.tensor([[0, 1, 2], [1, bad, 0]], device=DEV)
    with pytest.raises(IndexError):
        build_graph(ei, 50)


# ----------------------------------------------------------- aggregation --
@pytest.mark.parametrize("n,e,f", [(1000, 5000, 16), (500, 3000, 10), (300, 2000, 96),
                                   (4000, 40000, 128), (2000, 20000, 256), (100, 700, 3),
                                   (64, 300, 1000), (10, 0, 32)])
def test_gather_mean_fp32_bit_exact(n, e, f):
    from sldm_sage import build_graph, ops
    ei, x = _graph(n, e, f, seed=f)
    g = build_graph(ei.to(DEV), n)
    out = ops.gather_rows(x.to(DEV), g.rowptr, g.col, n, mean=True)
    rp, col, _, _ = ref_csr(ei, n)
    ref = ref_agg_mean_f32(x, rp, col)
    assert torch.equal(out.cpu(), ref)
    # and the C oracle is bit-equal to the PyG restatement itself
    from oracle.sage_ref import pyg_sage_aggregate
    assert torch.equal(pyg_sage_aggregate(x, ei), ref)


@pytest.mark.parametrize("n,e,f", [(1000, 5000, 16), (2000, 20000, 256), (300, 2000, 96),
                                   (100, 700, 6)])
def test_gather_mean_bf16_bit_exact(n, e, f):
    from sldm_sage import build_graph, ops
    ei, x = _graph(n, e, f, seed=f + 1)
    xb = x.bfloat16()
    g = build_graph(ei.to(DEV), n)
    out = ops.gather_rows(xb.to(DEV), g.rowptr, g.col, n, mean=True)
    rp, col, _, _ = ref_csr(ei, n)
    ref = ref_agg_mean_f32(xb.float(), rp, col).bfloat16()
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_transpose_sum_with_addend(dtype):
    """Backward form: out[j] = addend[j] + sum_{j->i} g[i] (g prescaled by 1/deg)."""
    from sldm_sage import build_graph, ops
    n, e, f = 3000, 30000, 64
    ei, g_in = _graph(n, e, f, seed=3)
    add = torch.randn(n, f, generator=torch.Generator().manual_seed(4))
    gr = build_graph(ei.to(DEV), n)
    d = g_in.to(DEV, dtype).clone()
    ops.scale_rows_by_inv_deg_(d, gr.rowptr)
    out = ops.gather_rows(d, gr.t_rowptr, gr.t_col, n, mean=False, addend=add.to(DEV, dtype))
    deg = torch.bincount(ei[1], minlength=n).clamp(min=1).float()
    gs = (g_in.to(dtype).float() / deg[:, None]).to(dtype).float()
    ref = add.to(dtype).float().index_add(0, ei[0], gs[ei[1]])
    torch.testing.assert_close(out.float().cpu(), ref, **TOL[dtype])


# ------------------------------------------------------------------ post --
@pytest.mark.parametrize("f", [16, 32, 96, 128, 256, 10])
@pytest.mark.parametrize("slope", [0.1, 0.0])
def test_post_fwd_bwd_vs_torch(f, slope):
    from sldm_sage import ops
    n = 777
    gen = torch.Generator().manual_seed(f)
    h = torch.randn(n, f, generator=gen) * 3 + 1
    b, gam, bet = (torch.randn(f, generator=gen) for _ in range(3))
    dout = torch.randn(n, f, generator=gen)
    out, xhat, rstd = ops.post_fwd(h.to(DEV), b.to(DEV), gam.to(DEV), bet.to(DEV), 1e-5, slope,
                                   0.0, 0, torch.float32, save=True)
    dh, dg, db, dbias = ops.post_bwd(dout.to(DEV), xhat, rstd, gam.to(DEV), bet.to(DEV), slope,
                                     0.0, 0, torch.float32)
    hr = h.clone().requires_grad_(True)
    br, gr, ber = (t.clone().requires_grad_(True) for t in (b, gam, bet))
    y = torch.nn.functional.layer_norm(hr + br, (f,), gr, ber, 1e-5)
    z = torch.nn.functional.leaky_relu(y, slope)
    z.backward(dout)
    tol = dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(out.cpu(), z.detach(), **tol)
    torch.testing.assert_close(dh.cpu(), hr.grad, **tol)
    torch.testing.assert_close(dbias.cpu(), br.grad, **tol)
    torch.testing.assert_close(dg.cpu(), gr.grad, **tol)
    torch.testing.assert_close(db.cpu(), ber.grad, **tol)


def test_dropout_statistics_and_backward_mask():
    from sldm_sage import ops
    n, f, p = 4096, 128, 0.25
    h = torch.randn(n, f, device=DEV)
    gam = torch.ones(f, device=DEV)
    bet = torch.full((f,), 5.0, device=DEV)          # y > 0 everywhere
    out, xhat, rstd = ops.post_fwd(h, None, gam, bet, 1e-5, 0.1, p, 1234, torch.float32, True)
    kept = out != 0
    rate = kept.float().mean().item()
    assert abs(rate - (1 - p)) < 0.01
    y = xhat * gam + bet
    torch.testing.assert_close(out[kept], y[kept] / (1 - p))
    dh, dg, db, _ = ops.post_bwd(torch.ones_like(out), xhat, rstd, gam, bet, 0.1, p, 1234,
                                 torch.float32)
    # d beta counts exactly the kept elements, scaled
    torch.testing.assert_close(db, kept.float().sum(0) / (1 - p))
    out2, _, _ = ops.post_fwd(h, None, gam, bet, 1e-5, 0.1, p, 1235, torch.float32, True)
    assert not torch.equal(out != 0, out2 != 0)


# -------------------------------------------------------------- SageBlock --
CASES = [
    # (N, E, hdims, negative_slope)
    (1000, 5000, [16, 16, 16], 0.1),
    (1000, 5000, [16, 32, 32], 0.1),
    (1000, 5000, [16, 16, 16], None),
    (1000, 5000, [16, 32, 32], None),
    (600, 4000, [128, 96, 96], 0.1),     # vehicle SageBlock shape (grusage.py:108)
    (500, 2500, [10, 8, 8], 0.1),        # map SageBlock default dims (mapencoder.py:18)
    (2000, 20000, [256, 256, 256, 256], 0.1),
]


@pytest.mark.parametrize("n,e,hdims,ns", CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sageblock_fwd_bwd(n, e, hdims, ns, dtype):
    from sldm_sage import SageBlock
    from oracle.sage_ref import random_graph
    ei, x = random_graph(n, e, hdims[0], seed=0)
    gout = torch.randn(n, hdims[-1], generator=torch.Generator().manual_seed(2))
    ref = oracle_block(hdims, ns)
    if dtype == torch.bfloat16:  # the reference sees the same bf16-rounded input
        x = x.bfloat16().float()
    out_r, dx_r, grads_r = run_oracle(ref, x, ei, gout)

    blk = SageBlock(hdims, dropout=None, negative_slope=ns)
    blk.load_state_dict(ref.state_dict())
    blk = blk.to(DEV)
    xg = x.to(DEV, dtype).requires_grad_(True)
    out = blk(xg, ei.to(DEV))
    out.backward(gout.to(DEV, dtype))
    tol = TOL[dtype]
    torch.testing.assert_close(out.float().cpu(), out_r, **tol)
    torch.testing.assert_close(xg.grad.float().cpu(), dx_r, **tol)
    for k, p in blk.named_parameters():
        g = grads_r[k]
        scale = max(1.0, g.abs().max().item())
        torch.testing.assert_close(p.grad.float().cpu() / scale, g / scale, **tol,
                                   msg=lambda m: f"{k}: {m}")


def test_sageblock_edge_cases():
    from sldm_sage import SageBlock
    hd = [8, 8, 8]
    ref = oracle_block(hd)
    blk = SageBlock(hd, None, 0.1)
    blk.load_state_dict(ref.state_dict())
    blk = blk.to(DEV)
    n = 50
    x = torch.randn(n, 8, generator=torch.Generator().manual_seed(9))
    edge_sets = {
        "empty": torch.empty(2, 0, dtype=torch.long),
        "isolated+dup+self": torch.tensor([[0, 0, 3, 3, 5, 7, 7], [1, 1, 3, 4, 5, 9, 9]]),
        "star-in": torch.stack([torch.arange(1, n), torch.zeros(n - 1, dtype=torch.long)]),
    }
    for name, ei in edge_sets.items():
        gout = torch.randn(n, 8, generator=torch.Generator().manual_seed(1))
        out_r, dx_r, gr = run_oracle(ref, x, ei, gout)
        xg = x.to(DEV).requires_grad_(True)
        blk.zero_grad(set_to_none=True)
        out = blk(xg, ei.to(DEV))
        out.backward(gout.to(DEV))
        torch.testing.assert_close(out.cpu(), out_r, atol=1e-4, rtol=1e-4, msg=name)
        torch.testing.assert_close(xg.grad.cpu(), dx_r, atol=1e-4, rtol=1e-4, msg=name)
        for k, p in blk.named_parameters():
            torch.testing.assert_close(p.grad.cpu(), gr[k], atol=1e-4, rtol=1e-4, msg=name + k)
    # identity block (len(hdims) == 1)
    ident = SageBlock([8]).to(DEV)
    xx = torch.randn(5, 8, device=DEV)
    assert ident(xx, torch.empty(2, 0, dtype=torch.long, device=DEV)) is xx


def test_golden_fixtures():
    """The committed oracle fixtures (tests/golden/*.npz) through the GPU path."""
    import glob
    import os

    from sldm_sage import SageBlock
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))
    assert files, "no golden fixtures"
    for fn in files:
        z = np.load(fn)
        hdims = [int(v) for v in z["hdims"]]
        ns = float(z["negative_slope"]) if z["has_slope"] else None
        blk = SageBlock(hdims, None, ns)
        sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")}
        blk.load_state_dict(sd)
        blk = blk.to(DEV)
        xg = torch.from_numpy(z["x"]).to(DEV).requires_grad_(True)
        out = blk(xg, torch.from_numpy(z["edge_index"]).to(DEV))
        out.backward(torch.from_numpy(z["gout"]).to(DEV))
        tol = dict(atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(out.detach().cpu(), torch.from_numpy(z["out"]), **tol)
        torch.testing.assert_close(xg.grad.cpu(), torch.from_numpy(z["dx"]), **tol)
        for k, p in blk.named_parameters():
            torch.testing.assert_close(p.grad.cpu(), torch.from_numpy(z["grad." + k]), **tol)


def test_inference_mode_and_thread():
    """Forward under inference_mode on a non-main thread (rcv.py:58-91 pattern)."""
    from sldm_sage import SageBlock
    from oracle.sage_ref import random_graph
    ei, x = random_graph(300, 1500, 16, seed=4)
    ref = oracle_block([16, 16, 16]).eval()
    blk = SageBlock([16, 16, 16], 0.25, 0.1)
    blk.load_state_dict(ref.state_dict())
    blk = blk.to(DEV).eval()
    res = {}

    def worker():
        with torch.inference_mode():
            res["out"] = blk(x.to(DEV), ei.to(DEV)).cpu()

    t = threading.Thread(target=worker)
    t.start()
    t.join()
    with torch.no_grad():
        expect = ref(x, ei)
    torch.testing.assert_close(res["out"], expect, atol=1e-4, rtol=1e-4)


def test_graph_cache_static_and_invalidate():
    from sldm_sage import SageBlock, graph_cache
    from oracle.sage_ref import random_graph
    graph_cache.clear()
    ei, x = random_graph(200, 800, 8, seed=6)
    blk = SageBlock([8, 8], None, 0.1).to(DEV)
    eid = ei.to(DEV)
    xd = x.to(DEV)
    a = blk(xd, eid)
    assert len(graph_cache) == 1
    b = blk(xd, eid)
    assert len(graph_cache) == 1 and torch.equal(a, b)
    eid[1, :10] = 0                     # in-place edit bumps _version -> rebuild
    c = blk(xd, eid)
    ref = oracle_block([8, 8])
    ref.load_state_dict(blk.state_dict())
    with torch.no_grad():
        torch.testing.assert_close(c.detach().cpu(), ref.to("cpu")(x, eid.cpu()), atol=1e-4,
                                   rtol=1e-4)
    del eid
    import gc
    gc.collect()
    assert len(graph_cache) == 0
