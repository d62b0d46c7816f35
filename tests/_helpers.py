"""Shared helpers for the tests (oracle wiring, tolerances, C-oracle binding)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSR_REF_SO = os.path.join(ROOT, "oracle", "build", "libcsr_ref.so")

# Parity tolerances (BASELINE.json north_star): 1e-4 fp32, 1e-2 bf16.
TOL = {torch.float32: dict(atol=1e-4, rtol=1e-4), torch.bfloat16: dict(atol=1e-2, rtol=1e-2)}


def csr_ref():
    if not os.path.exists(CSR_REF_SO):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(CSR_REF_SO)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.csr_ref_build.argtypes = [vp, i64, i64, vp, vp, vp, vp]
    lib.csr_ref_build.restype = ctypes.c_int
    lib.agg_ref_mean_f32.argtypes = [vp, i64, i64, vp, vp, vp]
    lib.agg_ref_mean_f32.restype = None
    return lib


def ref_csr(edge_index: torch.Tensor, n: int):
    """C-oracle CSR: (rowptr, col, t_rowptr, t_col) as int32 numpy, or None if bad ids."""
    lib = csr_ref()
    ei = np.ascontiguousarray(edge_index.cpu().numpy().astype(np.int64))
    e = ei.shape[1]
    rp = np.zeros(n + 1, np.int32)
    col = np.zeros(max(e, 1), np.int32)
    trp = np.zeros(n + 1, np.int32)
    tcol = np.zeros(max(e, 1), np.int32)
    rc = lib.csr_ref_build(ei.ctypes.data, e, n, rp.ctypes.data, col.ctypes.data,
                           trp.ctypes.data, tcol.ctypes.data)
    if rc != 0:
        return None
    return rp, col[:e], trp, tcol[:e]


def ref_agg_mean_f32(x: torch.Tensor, rowptr: np.ndarray, col: np.ndarray) -> torch.Tensor:
    lib = csr_ref()
    xn = np.ascontiguousarray(x.detach().cpu().float().numpy())
    n, f = xn.shape
    out = np.zeros_like(xn)
    col_ = col if col.size else np.zeros(1, np.int32)
    lib.agg_ref_mean_f32(xn.ctypes.data, n, f, rowptr.ctypes.data, col_.ctypes.data,
                         out.ctypes.data)
    return torch.from_numpy(out)


def oracle_block(hdims, negative_slope=0.1, seed=1):
    from oracle.sage_ref import RefSageBlock, set_synthetic_params
    ref = RefSageBlock(hdims, dropout=None, negative_slope=negative_slope)
    set_synthetic_params(ref, seed=seed)
    return ref


def run_oracle(ref, x, edge_index, gout):
    xr = x.detach().float().clone().requires_grad_(True)
    ref.zero_grad(set_to_none=True)
    out = ref(xr, edge_index)
    out.backward(gout.float())
    grads = {k: p.grad.clone() for k, p in ref.named_parameters()}
    return out.detach(), xr.grad.detach(), grads
