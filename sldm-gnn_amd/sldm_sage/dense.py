"""The dense part of a SAGEConv layer on hand-written MFMA
kernels: one contraction [agg | x] · [W_l | W_r]^T per layer with the bias,
LayerNorm, activation and dropout fused in its epilogue, and the two backward
contractions (input grads with the 1/deg prescale fused; weight grads split
over the node dimension).
"""
from __future__ import annotations

import torch

from . import ops


def weight_cat(wl: torch.Tensor, wr: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[W_l | W_r] as [F_out, 2 F_in] in the compute dtype (parameter plumbing)."""
    return torch.cat([wl.detach(), wr.detach()], dim=1).to(dtype).contiguous()


def sage_layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed, save,
                   row_offset=0, outs=None, wcat=None):
    """out = dropout(act(LN(agg·W_l^T + b_l + x·W_r^T)))  -> (out, xhat, rstd).

    ``outs``: preallocated (out, xhat, rstd) row slices; ``wcat``: the
    [W_l | W_r] operand when the caller already built it."""
    if wcat is None:
        wcat = weight_cat(wl, wr, x.dtype)
    return ops.sage_dense_fwd(agg, x, wcat, bl, gamma, beta, eps, slope, drop_p, seed, save,
                              row_offset, outs=outs)


def sage_linear_bwd_data(dh: torch.Tensor, wl: torch.Tensor, wr: torch.Tensor,
                         rowptr: torch.Tensor, wcat: torch.Tensor | None = None):
    """[dAgg / deg | dx_root] = dh · [W_l | W_r] in one launch; returns the
    prescaled aggregate grad and the root-path grad as two contiguous [N, F_in]
    tensors (F_in % 4 == 0; otherwise column views of one [N, 2 F_in] buffer).
    ``wcat``: the forward's [W_l | W_r] operand (saves rebuilding it)."""
    fi = wl.size(1)
    if wcat is None or wcat.dtype != dh.dtype:
        wcat = weight_cat(wl, wr, dh.dtype)
    wcat_t = wcat.t().contiguous()                              # [2 F_in, F_out]
    if fi % 4 == 0:
        return ops.gemm_nt_rowscale(dh, wcat_t, rowptr, scale_cols=fi, split=True)
    buf = ops.gemm_nt_rowscale(dh, wcat_t, rowptr, scale_cols=fi)
    return buf[:, :fi], buf[:, fi:]


def sage_linear_bwd_data_blocked_ok(dh: torch.Tensor, fi: int, blk_cols: int) -> bool:
    return ops.gemm_nt_rowscale_blocked_ok(dh, 2 * fi, fi, blk_cols)


def sage_linear_bwd_data_blocked(dh: torch.Tensor, wcat_t: torch.Tensor, rowptr: torch.Tensor,
                                 fi: int, blk_cols: int, dx_root: torch.Tensor):
    """:func:`sage_linear_bwd_data` with dAgg / deg returned column-blocked
    (flat [fi // blk_cols][N][blk_cols], the send layout of a feature-sliced
    partition) and the root-path grad written into ``dx_root`` [N, F_in].
    ``wcat_t``: [W_l | W_r]^T, [2 F_in, F_out] contiguous."""
    blocked, _ = ops.gemm_nt_rowscale_blocked(dh, wcat_t, rowptr, fi, blk_cols, out2=dx_root)
    return blocked


def sage_linear_bwd_weight(dh: torch.Tensor, agg: torch.Tensor, x: torch.Tensor):
    """(dW_l, dW_r) = (dh^T · agg, dh^T · x), fp32, one launch + its reduce
    writing both (no slicing copies)."""
    return ops.gemm_tn(dh, agg, x, split=True)
