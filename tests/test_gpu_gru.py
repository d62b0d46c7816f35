"""The HIP GRU (sldm_sage.GRU, csrc/gru.hip) against torch.nn.GRU on the CPU
(the reference's own op, grusage.py:66-71,160-161; pinned to the restatement
oracle/gru_ref.py by tests/test_oracle.py): outputs, h_n and every gradient
within 1e-4 (fp32), for the model's shape and the edge cases of the API --
with the forward's recurrent product in split-bf16 form (default) and on the
exact fp32 MFMA."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True, params=["bf16x3", "fp32"])
def gru_kernel(request, monkeypatch):
    """Every test on both forward kernels: the split-bf16 recurrent product
    (default) and the exact fp32 MFMA one (SLDM_GRU_BF16X3=0)."""
    monkeypatch.setenv("SLDM_GRU_BF16X3", "1" if request.param == "bf16x3" else "0")
    return request.param


def _run_pair(N, T, I, H, batch_first=True, bias=True, h0=False, gout=True, gh=True,
              dx=True, seed=0):
    from sldm_sage import GRU
    torch.manual_seed(seed)
    ref = torch.nn.GRU(I, H, 1, bias=bias, batch_first=batch_first)
    ours = GRU(I, H, 1, bias=bias, batch_first=batch_first)
    ours.load_state_dict(ref.state_dict())
    ours = ours.to(DEV)
    g = torch.Generator().manual_seed(seed + 1)
    shape = (N, T, I) if batch_first else (T, N, I)
    x = torch.randn(shape, generator=g)
    hx = torch.randn(1, N, H, generator=g) if h0 else None
    go = torch.randn(shape[:2] + (H,), generator=g) if gout else None
    gn = torch.randn(1, N, H, generator=g) if gh else None

    def run(mod, dev):
        xx = x.detach().clone().to(dev).requires_grad_(dx)
        hh = hx.detach().clone().to(dev).requires_grad_(True) if h0 else None
        out, hn = mod(xx, hh)
        loss = 0
        if go is not None:
            loss = loss + (out * go.to(dev)).sum()
        if gn is not None:
            loss = loss + (hn * gn.to(dev)).sum()
        loss.backward()
        grads = {k: p.grad.detach().cpu() for k, p in mod.named_parameters()}
        if dx:
            grads["x"] = xx.grad.detach().cpu()
        if h0:
            grads["h0"] = hh.grad.detach().cpu()
        return out.detach().cpu(), hn.detach().cpu(), grads

    o_r, h_r, g_r = run(ref, "cpu")
    o_g, h_g, g_g = run(ours, DEV)
    tol = dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(o_g, o_r, **tol)
    torch.testing.assert_close(h_g, h_r, **tol)
    assert set(g_g) == set(g_r)
    for k in g_r:
        s = max(1.0, g_r[k].abs().max().item()) if k not in ("x", "h0") else 1.0
        torch.testing.assert_close(g_g[k] / s, g_r[k] / s, **tol, msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("H", [16, 32, 48, 64, 80, 96])
def test_gru_hidden_sizes(H):
    _run_pair(50, 12, 6, H)


@pytest.mark.parametrize("I", [1, 3, 4, 6, 9, 16])
def test_gru_input_sizes(I):
    _run_pair(33, 10, I, 32)


def test_gru_time_major_h0_no_bias():
    _run_pair(40, 15, 6, 48, batch_first=False, bias=False, h0=True)


def test_gru_only_h_n_gradient():
    """GruSage reads only hlast[-1] (grusage.py:160-161): no output gradient.
    The backward must then receive dout = None (the kernel's no-dout path),
    not a materialised [N, T, H] tensor of zeros."""
    from sldm_sage import gru as gru_mod
    gru_mod._GruFn.last_backward_had_dout = None
    _run_pair(64, 20, 6, 96, gout=False, dx=False)
    assert gru_mod._GruFn.last_backward_had_dout is False
    _run_pair(64, 20, 6, 96, gout=True, dx=False)
    assert gru_mod._GruFn.last_backward_had_dout is True


def test_gru_model_shape():
    """The vehicle batch: 32 packs x ~300 vehicles, T = 100 frames, 6 -> 96."""
    _run_pair(9600, 100, 6, 96, gout=False, dx=False, seed=3)


def test_gru_deterministic_and_unbatched():
    from sldm_sage import GRU
    torch.manual_seed(1)
    m = GRU(6, 32, batch_first=True).to(DEV)
    x = torch.randn(70, 8, 6, device=DEV)
    grads = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        out, hn = m(x)
        hn.sum().backward()
        grads.append(m.weight_hh_l0.grad.clone())
    assert torch.equal(grads[0], grads[1])
    o1, h1 = m(x[3])                      # unbatched [T, I]
    o2, h2 = m(x[3:4])
    torch.testing.assert_close(o1, o2[0])
    torch.testing.assert_close(h1, h2[:, 0])


def test_gru_rejects_unsupported():
    from sldm_sage import GRU
    with pytest.raises(ValueError):
        GRU(6, 100)
    with pytest.raises(ValueError):
        GRU(6, 32, num_layers=2)
    with pytest.raises(RuntimeError):
        GRU(6, 32)(torch.randn(2, 3, 6))   # CPU tensors: no fallback
