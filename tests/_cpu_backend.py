"""TEST INFRASTRUCTURE: a plain-torch CPU stand-in for sldm_sage.dist.HipBackend.

It implements the per-rank compute interface of the distributed SageBlock
(CSR build, gather, fused layer forward, post backward, the two backward
GEMMs) with ordinary torch ops so the multi-rank protocol (partitioning,
RCCL/gloo all-gathers, gradient all-reduce) can be checked over gloo on CPU.
The product never uses it.
"""
from __future__ import annotations

import torch


class CpuBackend:
    @staticmethod
    def csr(edge_index, num_nodes, transpose):
        src, dst = edge_index[0].long(), edge_index[1].long()

        def by(key, val):
            order = torch.argsort(key, stable=True)
            ptr = torch.searchsorted(key[order], torch.arange(num_nodes + 1))
            return ptr, val[order]

        rp, col = by(dst, src)
        trp, tcol = by(src, dst) if transpose else (None, None)
        return rp, col, trp, tcol

    @staticmethod
    def gather(x, rowptr, col, num_rows, mean, addend=None, rows=None, out=None, edges=None):
        full = CpuBackend._gather_all(x, rowptr, col, num_rows, mean, addend)
        if rows is None:
            if out is not None:
                out.copy_(full)
                return out
            return full
        if out is None:
            out = torch.full_like(full, float("nan"))     # untouched rows stay visible
        idx = rows.rows.long()
        out[idx] = full[idx]
        return out

    @staticmethod
    def _gather_all(x, rowptr, col, num_rows, mean, addend):
        rowptr = rowptr.long()
        base = rowptr[0]
        deg = rowptr[1:] - rowptr[:-1]
        seg = torch.repeat_interleave(torch.arange(num_rows), deg)
        cols = col[base: base + int(deg.sum())].long()
        out = torch.zeros(num_rows, x.size(1), dtype=torch.float32)
        out.index_add_(0, seg, x[cols].float())
        if mean:
            out = out / deg.clamp(min=1).float()[:, None]
        if addend is not None:
            out = addend.float() + out
        return out.to(x.dtype)

    @staticmethod
    def pick_rows(x, rowptr, idx):
        return x[idx.long()]

    @staticmethod
    def layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed, save, row_offset,
                  outs=None):
        res = CpuBackend._layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p)
        if outs is None:
            return res
        for dst, src in zip(outs, res):
            if dst is not None:
                dst.copy_(src)
        return outs

    @staticmethod
    def _layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p):
        assert drop_p == 0.0, "CPU test backend has no dropout"
        h = agg @ wl.detach().t() + bl.detach() + x @ wr.detach().t()
        mu = h.mean(1, keepdim=True)
        rstd = 1.0 / torch.sqrt(((h - mu) ** 2).mean(1, keepdim=True) + eps)
        xhat = (h - mu) * rstd
        y = xhat * gamma.detach() + beta.detach()
        out = torch.where(y > 0, y, y * slope)
        return out, xhat, rstd.squeeze(1)

    @staticmethod
    def post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed, zout, row_offset):
        dy = torch.where(zout > 0, dout, dout * slope)
        gx = dy * gamma.detach()
        r = rstd[:, None]
        dh = r * (gx - gx.mean(1, keepdim=True) - xhat * (gx * xhat).mean(1, keepdim=True))
        return dh, (dy * xhat).sum(0), dy.sum(0), dh.sum(0)

    @staticmethod
    def bwd_data(dh, wl, wr, rowptr):
        deg = (rowptr[1:] - rowptr[:-1]).clamp(min=1).float()
        return (dh @ wl.detach()) / deg[:, None], dh @ wr.detach()

    @staticmethod
    def bwd_weight(dh, agg, x):
        return dh.t() @ agg, dh.t() @ x

    @staticmethod
    def cols_pack(rows, nblk, cs):
        return rows.reshape(rows.size(0), nblk, cs).transpose(0, 1).contiguous().view(-1)

    @staticmethod
    def cols_unpack(blocks, n, nblk, cs, out, addend=None):
        src = blocks.view(nblk, n, cs).transpose(0, 1).reshape(n, nblk * cs)
        if addend is None:
            out.copy_(src)
        else:
            torch.add(addend, src, out=out)
        return out
