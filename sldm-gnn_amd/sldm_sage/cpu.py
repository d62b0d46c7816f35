"""The SageBlock path for CPU tensors: the reference's CPU mode.

The reference runs on ``DEVICE = 'cuda' if torch.cuda.is_available() else
'cpu'`` (/root/reference/main.py:58; test.py:18), so the drop-in must accept
CPU tensors too.  CUDA tensors always take the gfx950 library
(libsldm_sage.so; no fallback).  CPU tensors take this module: the same
algorithm in native host code (libsldm_sage_cpu.so, csrc_cpu/sage_cpu.cpp,
OpenMP over rows) -- CSR built once and cached, rows summed straight from
their source rows in CSR order (no [E, F] message tensor), LayerNorm /
activation / dropout fused per row with the GPU kernels' dropout hash, the
backward on the transpose CSR -- with the two GEMMs of a layer as plain
library GEMMs (torch.mm).  fp32 only, as in the reference.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
CPU_LIB_PATH = os.environ.get("SLDM_SAGE_CPU_LIB", os.path.join(_HERE, "libsldm_sage_cpu.so"))

_vp, _i64, _f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
_SIG = {
    "sldm_cpu_abi_version": (ctypes.c_int, []),
    "sldm_cpu_csr_build": (ctypes.c_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "sldm_cpu_gather_rows": (None, [_vp, _i64, _vp, _vp, _i64, _i64, ctypes.c_int, _vp, _i64,
                                    _vp, _i64]),
    "sldm_cpu_scale_rows_by_inv_deg": (None, [_vp, _i64, _vp, _i64, _i64]),
    "sldm_cpu_post_fwd": (None, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _f, _f, _f,
                                 ctypes.c_uint64, _i64, _vp, _vp, _vp]),
    "sldm_cpu_post_bwd": (None, [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _f, _f, ctypes.c_uint64,
                                 _i64, _vp, _vp, _vp, _vp]),
    "sldm_cpu_segment_pool": (None, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp,
                                     _vp]),
    "sldm_cpu_segment_pool_bwd": (None, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64,
                                         _vp, _i64, _vp, _vp, _vp, _i64]),
}
_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(CPU_LIB_PATH):
                raise RuntimeError(
                    f"libsldm_sage_cpu.so not found at {CPU_LIB_PATH}: build it with "
                    "`make -C sldm-gnn_amd/csrc` (CPU tensors need it; there is no "
                    "torch fallback)")
            lib = ctypes.CDLL(CPU_LIB_PATH)
            for name, (res, args) in _SIG.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            _lib = lib
    return _lib


def exported_symbols() -> list[str]:
    return list(_SIG)


def _p(t):
    return None if t is None else t.data_ptr()


def _f32(t):
    return None if t is None else t.detach().float().contiguous()


def csr_build(edge_index: torch.Tensor, num_nodes: int, transpose: bool = True):
    """edge_index [2, E] (CPU) -> (rowptr, col, t_rowptr, t_col) int32; raises
    IndexError on an id outside [0, num_nodes) (as the reference does)."""
    ei = edge_index.to(torch.int64).contiguous()
    E, N = ei.size(1), int(num_nodes)
    rowptr = torch.empty(N + 1, dtype=torch.int32)
    col = torch.empty(max(E, 1), dtype=torch.int32)[:E]
    t_rowptr = torch.empty(N + 1, dtype=torch.int32) if transpose else None
    t_col = torch.empty(max(E, 1), dtype=torch.int32)[:E] if transpose else None
    rc = load().sldm_cpu_csr_build(ei.data_ptr(), E, N, rowptr.data_ptr(),
                                   col.data_ptr() if E else rowptr.data_ptr(), _p(t_rowptr),
                                   (t_col.data_ptr() if E else t_rowptr.data_ptr())
                                   if transpose else None)
    if rc:
        raise IndexError(f"edge_index holds a node id outside [0, {num_nodes}) "
                         "(the reference's index_select/scatter would raise as well)")
    return rowptr, col, t_rowptr, t_col


def gather_rows(x, rowptr, col, num_rows, mean, addend=None):
    x = x.contiguous()
    F = x.size(1)
    out = torch.empty(num_rows, F, dtype=torch.float32)
    if num_rows == 0 or F == 0:
        return out
    add = addend.contiguous() if addend is not None else None
    load().sldm_cpu_gather_rows(x.data_ptr(), F, rowptr.data_ptr(),
                                col.data_ptr() if col.numel() else rowptr.data_ptr(), num_rows,
                                F, int(bool(mean)), _p(add), F, out.data_ptr(), F)
    return out


def as_f32(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != torch.float32:
        raise TypeError(f"SageBlock on CPU computes in float32 (the reference's dtype), "
                        f"got {x.dtype}")
    return x.contiguous()


def scale_rows_by_inv_deg_(g: torch.Tensor, rowptr: torch.Tensor) -> torch.Tensor:
    load().sldm_cpu_scale_rows_by_inv_deg(g.data_ptr(), g.size(1), rowptr.data_ptr(), g.size(0),
                                          g.size(1))
    return g


def layer_fwd(x, rowptr, col, wl, bl, wr, gamma, beta, slope, drop_p, seed, eps):
    """One SageBlock layer on the host kernels (sageblock.py:18-19): the CPU
    implementation of ``torch.ops.sldm.sage_layer`` -> (out, agg, xhat, rstd)."""
    n = x.size(0)
    agg = gather_rows(x, rowptr, col, n, True)
    h = torch.mm(agg, wl.detach().t())
    h.addmm_(x, wr.detach().t())
    fo = h.size(1)
    out = torch.empty(n, fo)
    xhat = torch.empty(n, fo)
    rstd = torch.empty(n)
    # bound to locals: a converted copy must outlive the C call
    bias_, gamma_, beta_ = _f32(bl), _f32(gamma), _f32(beta)
    load().sldm_cpu_post_fwd(h.data_ptr(), fo, n, fo, _p(bias_), gamma_.data_ptr(),
                             beta_.data_ptr(), float(eps), float(slope), float(drop_p),
                             seed & (2**64 - 1), 0, out.data_ptr(), xhat.data_ptr(),
                             rstd.data_ptr())
    return out, agg, xhat, rstd


def layer_bwd(dout, x, agg, xhat, rstd, rowptr, t_rowptr, t_col, wl, wr, gamma, beta, slope,
              drop_p, seed, need_dx):
    """CPU implementation of ``torch.ops.sldm.sage_layer_bwd`` ->
    (dx, dW_l, db_l, dW_r, dgamma, dbeta); dx has 0 elements unless need_dx."""
    n, fo = xhat.shape
    dout = dout.float().contiguous()
    dh = torch.empty(n, fo)
    dg, db, dbias = torch.empty(fo), torch.empty(fo), torch.empty(fo)
    gamma_, beta_ = _f32(gamma), _f32(beta)
    load().sldm_cpu_post_bwd(dout.data_ptr(), xhat.data_ptr(), rstd.data_ptr(), n, fo,
                             gamma_.data_ptr(), beta_.data_ptr(), float(slope),
                             float(drop_p), seed & (2**64 - 1), 0, dh.data_ptr(),
                             dg.data_ptr(), db.data_ptr(), dbias.data_ptr())
    dwl = torch.mm(dh.t(), agg)
    dwr = torch.mm(dh.t(), x)
    dx = x.new_empty(0)
    if need_dx:
        g = torch.mm(dh, wl.detach())
        scale_rows_by_inv_deg_(g, rowptr)
        dx_r = torch.mm(dh, wr.detach())
        dx = gather_rows(g, t_rowptr, t_col, n, False, addend=dx_r)
    return (dx, dwl.to(wl.dtype), dbias.to(wl.dtype), dwr.to(wr.dtype), dg.to(gamma.dtype),
            db.to(beta.dtype))


class PoolFn(torch.autograd.Function):
    """global mean / max / mean||max pooling of CPU tensors (pool.py's CPU
    mode): mode bit 1 mean, bit 2 max; ``first_arg``: batch=None routing of
    the max gradient (to the first maximal row)."""

    @staticmethod
    def forward(ctx, x, batch, num_segments: int, mode: int, first_arg: bool):
        x = as_f32(x)
        batch = batch.to(torch.int64).contiguous()
        if batch.numel() and (int(batch.min()) < 0 or int(batch.max()) >= num_segments):
            raise IndexError(f"batch holds a graph id outside [0, {num_segments})")
        n, F = x.shape
        B = int(num_segments)
        mean, mx = bool(mode & 1), bool(mode & 2)
        out = torch.empty(B, F * (2 if mean and mx else 1))
        meanv = out[:, :F] if mean else None
        maxv = out[:, F * (1 if mean else 0):] if mx else None
        div = torch.empty(B, F) if mx and not first_arg else None
        arg = torch.empty(B, F, dtype=torch.int32) if mx and first_arg else None
        load().sldm_cpu_segment_pool(x.data_ptr(), x.stride(0), batch.data_ptr(), n, B, F,
                                     _p(meanv), meanv.stride(0) if mean else 0, _p(maxv),
                                     maxv.stride(0) if mx else 0, _p(div), _p(arg))
        ctx.save_for_backward(x, batch, out)
        ctx.aux, ctx.cfg = (div, arg), (B, mode)
        return out

    @staticmethod
    def backward(ctx, gout):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        x, batch, out = ctx.saved_tensors
        div, arg = ctx.aux
        B, mode = ctx.cfg
        n, F = x.shape
        mean, mx = bool(mode & 1), bool(mode & 2)
        g = gout.float().contiguous()
        dmean = g[:, :F] if mean else None
        dmax = g[:, F * (1 if mean else 0):] if mx else None
        maxv = out[:, F * (1 if mean else 0):] if mx else None
        dx = torch.empty_like(x)
        load().sldm_cpu_segment_pool_bwd(
            x.data_ptr(), x.stride(0), batch.data_ptr(), n, B, F, _p(dmean),
            dmean.stride(0) if mean else 0, _p(maxv), maxv.stride(0) if mx else 0, _p(dmax),
            dmax.stride(0) if mx else 0, _p(div), _p(arg), dx.data_ptr(), dx.stride(0))
        return dx, None, None, None, None
