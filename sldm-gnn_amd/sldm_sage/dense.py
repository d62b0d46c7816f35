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


class SageLinearFn(torch.autograd.Function):
    """out = agg · W_l^T + b_l + x · W_r^T, the dense half of a stand-alone
    SAGEConv (PyG 2.7.0 ``SAGEConv.forward``: ``lin_l(out) + lin_r(x_r)``), on
    the library's MFMA GEMMs: one NT GEMM over [agg | x] forward, the dX GEMM
    and the row-streaming dW GEMM backward (no rocBLAS / hipBLASLt)."""

    @staticmethod
    def forward(ctx, agg, x, wl, bl, wr):
        wcat = weight_cat(wl, wr, x.dtype)                           # [F_out, 2 F_in]
        a = torch.cat([agg, x], dim=1)
        out = ops.gemm_nt_rowscale(a, wcat, None, 0)
        if bl is not None:
            out += bl.to(out.dtype)
        ctx.save_for_backward(agg, x, wcat)
        ctx.meta = (wl.dtype, wr.dtype, None if bl is None else bl.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        agg, x, wcat = ctx.saved_tensors
        wl_dt, wr_dt, bl_dt = ctx.meta
        fi = x.size(1)
        dout = dout.contiguous()
        dagg = dx = dwl = dbl = dwr = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            d = ops.gemm_nt_rowscale(dout, wcat.t().contiguous(), None, 0)   # [N, 2 F_in]
            dagg, dx = d[:, :fi], d[:, fi:]
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[4]:
            dwl, dwr = ops.gemm_tn(dout, agg, x, split=True)                 # fp32
            dwl, dwr = dwl.to(wl_dt), dwr.to(wr_dt)
        if bl_dt is not None and ctx.needs_input_grad[3]:
            dbl = dout.float().sum(0).to(bl_dt)
        return dagg, dx, dwl, dbl, dwr


def sage_linear_bwd_weight(dh: torch.Tensor, agg: torch.Tensor, x: torch.Tensor):
    """(dW_l, dW_r) = (dh^T · agg, dh^T · x), fp32, one launch + its reduce
    writing both (no slicing copies)."""
    return ops.gemm_tn(dh, agg, x, split=True)
