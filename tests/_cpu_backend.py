"""TEST INFRASTRUCTURE: a plain-torch CPU stand-in for sldm_sage.dist.HipBackend.

It implements the per-rank compute interface of the distributed SageBlock
(CSR build, gather, fused layer forward, post backward, the two backward
GEMMs) with ordinary torch ops so the multi-rank protocol (partitioning,
RCCL/gloo all-gathers, gradient all-reduce) can be checked over gloo on CPU.
The product never uses it.
"""
from __future__ import annotations

import numpy as np
import torch


def _hash32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def dropout_keep(seed: int, row0: int, rows: int, feat: int, p: float) -> torch.Tensor:
    """The kernels' counter-hash dropout mask, restated (csrc/common.hpp:
    dropout_row_key / dropout_keep): keep[i, j] for global rows row0 + i."""
    with np.errstate(over="ignore"):
        r = np.arange(row0, row0 + rows, dtype=np.uint64)
        lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
        inner = hi ^ _hash32((r & np.uint64(0xFFFFFFFF)).astype(np.uint32)) ^ (
            (r >> np.uint64(32)).astype(np.uint32) * np.uint32(0x9E3779B9))
        key = _hash32(lo ^ _hash32(inner))
        col = np.arange(feat, dtype=np.uint32)
        h = _hash32(key[:, None] + (col >> np.uint32(1))[None, :] * np.uint32(0x9E3779B9))
        v = np.where((col & np.uint32(1))[None, :] == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    thr = 65536 if p >= 1 else (0 if p <= 0 else int(np.float32(p) * np.float32(65536.0)
                                                   + np.float32(0.5)))
    return torch.from_numpy(v >= thr)


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
    def gather(x, rowptr, col, num_rows, mean, addend=None, rows=None, out=None, edges=None,
               hub=None):
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
        res = CpuBackend._layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed,
                                    row_offset)
        if outs is None:
            return res
        for dst, src in zip(outs, res):
            if dst is not None:
                dst.copy_(src)
        return outs

    @staticmethod
    def _layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed=0, row_offset=0):
        h = agg @ wl.detach().t() + bl.detach() + x @ wr.detach().t()
        mu = h.mean(1, keepdim=True)
        rstd = 1.0 / torch.sqrt(((h - mu) ** 2).mean(1, keepdim=True) + eps)
        xhat = (h - mu) * rstd
        y = xhat * gamma.detach() + beta.detach()
        out = torch.where(y > 0, y, y * slope)
        if drop_p > 0:
            keep = dropout_keep(seed, row_offset, out.size(0), out.size(1), drop_p)
            out = torch.where(keep, out * (1.0 / (1.0 - drop_p)), torch.zeros(()))
        return out, xhat, rstd.squeeze(1)

    @staticmethod
    def post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed, zout, row_offset):
        if drop_p > 0:
            keep = dropout_keep(seed, row_offset, dout.size(0), dout.size(1), drop_p)
            dout = torch.where(keep, dout * (1.0 / (1.0 - drop_p)), torch.zeros(()))
            y = xhat * gamma.detach() + beta.detach()       # dropped outputs lost their sign
            dy = torch.where(y > 0, dout, dout * slope)
        else:
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
