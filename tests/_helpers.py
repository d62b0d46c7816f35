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


def bf16_oracle(ref, x, edge_index, gout, negative_slope, round_sum_first=False,
                act_masks=None, stats=None, check_rows=None, store="bf16",
                layer_inputs=None):
    """oracle/sage_bf16_ref.py on ``ref``'s parameters: (out, dx, grads).
    ``store="fp32"``: the same restatement without storage rounding."""
    from oracle.sage_bf16_ref import bf16_round, block_params, sageblock_fwd_bwd
    return sageblock_fwd_bwd(block_params(ref), x.detach().cpu().float(), edge_index.cpu(),
                             gout.detach().cpu().float(), negative_slope,
                             store=bf16_round if store == "bf16" else None,
                             round_sum_first=round_sum_first, act_masks=act_masks,
                             stats=stats, check_rows=check_rows,
                             layer_inputs=layer_inputs)


def assert_bf16_close(name, got, want, atol=1e-2, rtol=1e-2, reduction=None):
    """north_star's bf16 bar, element-wise: |got - want| <= atol + rtol |want|
    against the bf16-storage oracle (like-for-like rounding points).

    ``reduction``: the tensor is a sum over all node rows (a parameter
    gradient); its per-element error is set by the rows' bf16 rounding noise
    (~sqrt(N) ulp |dh| |h|), not by the element's own value, so atol scales
    with the tensor's range -- max(1, max |want|) -- as the fp32 tests do for
    the same tensors.  ``reduction=None`` infers it from the name."""
    if reduction is None:
        reduction = name.split(" ")[0] not in ("out", "dx")
    got = got.detach().float().cpu()
    want = want.detach().float().cpu()
    if reduction:
        atol = atol * max(1.0, want.abs().max().item())
    bad = (got - want).abs() > atol + rtol * want.abs()
    if bool(bad.any()):
        idx = bad.nonzero()[:5].tolist()
        raise AssertionError(
            f"{name}: {int(bad.sum())} of {bad.numel()} elements off by more than "
            f"{atol} + {rtol}|ref| (max abs diff {(got - want).abs().max().item():.4g}); "
            f"first at {idx}: got {[got[tuple(i)].item() for i in idx]}, "
            f"want {[want[tuple(i)].item() for i in idx]}")


def device_act_masks(blk, x, edge_index, rows=None):
    """The device run's activation branch per layer, (layer output > 0), from
    forwards of the block truncated after each layer (the same kernels, so
    the same bits as inside the full block; the last one is checked against
    the full forward by the caller).  For LeakyReLU / ReLU, output > 0 iff
    the pre-activation > 0.  ``rows``: keep only these rows (device index)."""
    import torch.nn as nn
    from sldm_sage import SageBlock
    hd = [blk.convs[0].in_channels] + [c.out_channels for c in blk.convs]
    ns = blk.posts[0][1].negative_slope if isinstance(blk.posts[0][1], nn.LeakyReLU) else None
    masks, outs = [], []
    sd = blk.state_dict()
    with torch.no_grad():
        for depth in range(1, len(hd)):
            part = SageBlock(hd[: depth + 1], None, ns)
            part.load_state_dict({k: v for k, v in sd.items()
                                  if int(k.split(".")[1]) < depth})
            part = part.to(x.device).eval()
            o = part(x.detach(), edge_index)
            if rows is not None:
                o = o[rows]
            masks.append((o > 0).cpu())
            outs.append(o)
    return masks, outs
