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


class _CpuLayerFn(torch.autograd.Function):
    """One SageBlock layer on the host kernels (sageblock.py:18-19)."""

    @staticmethod
    def forward(ctx, x, wl, bl, wr, gamma, beta, graph, slope, drop_p, seed, eps):
        n = x.size(0)
        agg = gather_rows(x, graph.rowptr, graph.col, n, True)
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
        ctx.save_for_backward(x, agg, xhat, rstd, wl, wr, gamma, beta)
        ctx.graph, ctx.cfg = graph, (slope, drop_p, seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, agg, xhat, rstd, wl, wr, gamma, beta = ctx.saved_tensors
        graph = ctx.graph
        slope, drop_p, seed = ctx.cfg
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
        dx = None
        if ctx.needs_input_grad[0]:
            g = torch.mm(dh, wl.detach())
            load().sldm_cpu_scale_rows_by_inv_deg(g.data_ptr(), g.size(1), graph.rowptr.data_ptr(),
                                                  n, g.size(1))
            dx_r = torch.mm(dh, wr.detach())
            dx = gather_rows(g, graph.t_rowptr, graph.t_col, n, False, addend=dx_r)
        return (dx, dwl.to(wl.dtype), dbias.to(wl.dtype), dwr.to(wr.dtype),
                dg.to(gamma.dtype), db.to(beta.dtype), None, None, None, None, None)
