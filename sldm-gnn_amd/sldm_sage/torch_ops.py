"""``torch.ops.sldm.*``: the SageBlock path as PyTorch custom operators.

libsldm_torch_ops.so (csrc/torch_ops.cpp) registers the operators with
``TORCH_LIBRARY(sldm, ...)`` and implements them for ROCm tensors over the C
ABI of libsldm_sage.so -- one C++ call per layer (or per stack) and direction.
This module loads it, registers the CPU implementations (the host kernels of
libsldm_sage_cpu.so, the reference's ``DEVICE = 'cpu'`` mode, main.py:58) so
the same operator serves both device types through the dispatcher, and wires
autograd with ``torch.library.register_autograd``:

    torch.ops.sldm.mean_aggregate(x, graph, meta)          PyG propagate + mean
    torch.ops.sldm.sage_layer(x, graph, meta, W_l, b_l, W_r, gamma, beta,
                              slope, p, seed, eps, save)   sageblock.py:18-19

``graph, meta`` is :meth:`sldm_sage.graph.SageGraph.packed`.  The whole-stack
operators (``sage_stack_fwd`` / ``sage_stack_bwd``, fused layer boundaries)
sit under one ``autograd.Function`` in sageblock.py.
"""
from __future__ import annotations

import os
import threading

import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
TORCH_LIB_PATH = os.environ.get("SLDM_TORCH_OPS_LIB", os.path.join(_HERE, "libsldm_torch_ops.so"))

_lock = threading.Lock()
_loaded = False


def load():
    """Load (once) libsldm_torch_ops.so and return ``torch.ops.sldm``; raises
    if the library (or libsldm_sage.so under it) is missing: no fallback."""
    global _loaded
    if _loaded:
        return torch.ops.sldm
    with _lock:
        if _loaded:
            return torch.ops.sldm
        _lib.load()                       # libsldm_sage.so first (the C ABI underneath)
        if not os.path.exists(TORCH_LIB_PATH):
            raise _lib.SldmError(
                f"libsldm_torch_ops.so not found at {TORCH_LIB_PATH}: build it with "
                "`make -C sldm-gnn_amd/csrc`")
        torch.ops.load_library(TORCH_LIB_PATH)
        ver = torch.ops.sldm.abi_version()
        if ver != _lib.ABI_VERSION:
            raise _lib.SldmError(f"libsldm_torch_ops.so sees ABI {ver}, expected "
                                 f"{_lib.ABI_VERSION}: rebuild")
        _register_cpu()
        _register_autograd()
        _loaded = True
    return torch.ops.sldm


# ------------------------------------------------------------ CPU kernels --
def _register_cpu() -> None:
    from . import cpu

    def unpack(graph):
        rowptr, col, t_rowptr, t_col = graph[:4]
        return rowptr, col, t_rowptr, t_col

    @torch.library.impl("sldm::mean_aggregate", "CPU")
    def _agg(x, graph, meta):
        rowptr, col, _, _ = unpack(graph)
        return cpu.gather_rows(cpu.as_f32(x), rowptr, col, x.size(0), True)

    @torch.library.impl("sldm::mean_aggregate_bwd", "CPU")
    def _agg_bwd(grad, graph, meta):
        rowptr, _, t_rowptr, t_col = unpack(graph)
        if not meta[0]:
            raise RuntimeError("SageGraph was built without its transpose; rebuild with "
                               "transpose=True for backward")
        g = grad.float().contiguous().clone()
        cpu.scale_rows_by_inv_deg_(g, rowptr)
        return cpu.gather_rows(g, t_rowptr, t_col, g.size(0), False)

    @torch.library.impl("sldm::sage_layer", "CPU")
    def _layer(x, graph, meta, wl, bl, wr, gamma, beta, slope, drop_p, seed, eps, save):
        rowptr, col, _, _ = unpack(graph)
        return cpu.layer_fwd(cpu.as_f32(x), rowptr, col, wl, bl, wr, gamma, beta, slope, drop_p,
                             seed, eps)

    @torch.library.impl("sldm::sage_layer_bwd", "CPU")
    def _layer_bwd(dout, x, agg, xhat, rstd, graph, meta, wl, wr, gamma, beta, slope, drop_p,
                   seed, need_dx):
        rowptr, _, t_rowptr, t_col = unpack(graph)
        if need_dx and not meta[0]:
            raise RuntimeError("SageGraph was built without its transpose; rebuild with "
                               "transpose=True for backward")
        return cpu.layer_bwd(dout, x, agg, xhat, rstd, rowptr, t_rowptr, t_col, wl, wr, gamma,
                             beta, slope, drop_p, seed, need_dx)


# ---------------------------------------------------------------- autograd --
def _register_autograd() -> None:
    def agg_setup(ctx, inputs, output):
        _, graph, meta = inputs
        ctx.graph, ctx.meta = graph, meta

    def agg_bwd(ctx, grad):
        return (torch.ops.sldm.mean_aggregate_bwd(grad, ctx.graph, ctx.meta),
                [None] * len(ctx.graph), None)

    torch.library.register_autograd("sldm::mean_aggregate", agg_bwd, setup_context=agg_setup)

    def layer_setup(ctx, inputs, output):
        x, graph, meta, wl, bl, wr, gamma, beta, slope, drop_p, seed, eps, save = inputs
        out, agg, xhat, rstd = output
        if not save:
            raise RuntimeError("sldm::sage_layer: differentiating needs save=True")
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(agg, xhat, rstd)
        ctx.save_for_backward(x, agg, xhat, rstd, wl, wr, gamma, beta)
        ctx.graph, ctx.meta = graph, meta
        ctx.cfg = (slope, drop_p, seed)
        ctx.has_bias = bl is not None

    def layer_bwd(ctx, dout, _dagg, _dxhat, _drstd):
        x, agg, xhat, rstd, wl, wr, gamma, beta = ctx.saved_tensors
        slope, drop_p, seed = ctx.cfg
        if dout is None:
            dout = torch.zeros_like(xhat)
        need_dx = ctx.needs_input_grad[0]
        dx, dwl, dbl, dwr, dgamma, dbeta = torch.ops.sldm.sage_layer_bwd(
            dout, x, agg, xhat, rstd, ctx.graph, ctx.meta, wl, wr, gamma, beta, slope, drop_p,
            seed, need_dx)
        return (dx if need_dx else None, [None] * len(ctx.graph), None, dwl,
                dbl if ctx.has_bias else None, dwr, dgamma, dbeta, None, None, None, None, None)

    torch.library.register_autograd("sldm::sage_layer", layer_bwd, setup_context=layer_setup)


# ------------------------------------------------------------------ timing --
def timing_set(on: bool, names=None) -> None:
    load().timing_set(bool(on), sorted(names) if names else [])


def timing_take():
    """[(name, ms, units)] of the launches recorded since the last call."""
    names, ms, units = load().timing_take()
    return list(zip(names, ms, units))
