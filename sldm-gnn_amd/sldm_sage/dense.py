"""The dense part of a SAGEConv layer: one contraction
[agg | x] · [W_l | W_r]^T per layer, and its two backward contractions.

Interim implementation: PyTorch GEMMs (hipBLASLt on ROCm) in the layer's
storage dtype.  The hand-written MFMA kernels replace these functions.
"""
from __future__ import annotations

import torch


def sage_linear_fwd(agg: torch.Tensor, x: torch.Tensor, wl: torch.Tensor,
                    wr: torch.Tensor) -> torch.Tensor:
    """h = agg · W_l^T + x · W_r^T   (bias is added in the post kernel)."""
    dt = x.dtype
    h = torch.mm(agg, wl.to(dt).t())
    h.addmm_(x, wr.to(dt).t())
    return h


def sage_linear_bwd_data(dh: torch.Tensor, wl: torch.Tensor, wr: torch.Tensor):
    """(d_agg, dx_root) = (dh · W_l, dh · W_r)."""
    dt = dh.dtype
    return torch.mm(dh, wl.to(dt)), torch.mm(dh, wr.to(dt))


def sage_linear_bwd_weight(dh: torch.Tensor, agg: torch.Tensor, x: torch.Tensor):
    """(dW_l, dW_r) = (dh^T · agg, dh^T · x), fp32."""
    if dh.dtype == torch.float32:
        return torch.mm(dh.t(), agg), torch.mm(dh.t(), x)
    return torch.mm(dh.t(), agg).float(), torch.mm(dh.t(), x).float()
