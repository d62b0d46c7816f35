"""ORACLE — test infrastructure only (see oracle/sage_ref.py for who may use it).

Independent fp64 numpy formulation of the same SageBlock (eval mode, no
dropout), written as dense linear algebra instead of index_select/scatter so
that it shares no code path with ``sage_ref.py``:

    A[i, j]  = (#edges j->i) / max(1, in_deg(i))          (mean aggregation)
    H        = A X W_l^T + 1 b_l^T + X W_r^T              (SAGEConv, PyG 2.7.0)
    Y        = LN(H) * gamma + beta, eps = 1e-5           (sageblock.py:11)
    Z        = leaky_relu(Y, ns) | relu(Y)                (sageblock.py:12)

and a hand-derived backward.  Used only on small graphs (dense N x N).
"""
from __future__ import annotations

import numpy as np


def mean_adjacency(edge_index: np.ndarray, n: int) -> np.ndarray:
    a = np.zeros((n, n), dtype=np.float64)
    for s, d in zip(edge_index[0].tolist(), edge_index[1].tolist()):
        a[d, s] += 1.0
    deg = a.sum(axis=1, keepdims=True)
    return a / np.maximum(deg, 1.0)


def forward(x, edge_index, params, negative_slope, eps=1e-5):
    """params: list of dicts with Wl [Fo,Fi], bl [Fo], Wr [Fo,Fi], g [Fo], b [Fo]."""
    a = mean_adjacency(edge_index, x.shape[0])
    tape = []
    h = x.astype(np.float64)
    slope = 0.0 if negative_slope is None else float(negative_slope)
    for p in params:
        agg = a @ h
        pre = agg @ p["Wl"].T + p["bl"] + h @ p["Wr"].T
        mu = pre.mean(axis=1, keepdims=True)
        var = ((pre - mu) ** 2).mean(axis=1, keepdims=True)
        rstd = 1.0 / np.sqrt(var + eps)
        xhat = (pre - mu) * rstd
        y = xhat * p["g"] + p["b"]
        z = np.where(y > 0, y, y * slope)
        tape.append((h, agg, xhat, rstd, y))
        h = z
    return h, (a, tape, slope)


def backward(dout, params, saved):
    """Returns (dx, [dict(Wl, bl, Wr, g, b) grads per layer])."""
    a, tape, slope = saved
    grads = [None] * len(params)
    d = dout.astype(np.float64)
    for li in reversed(range(len(params))):
        p = params[li]
        h, agg, xhat, rstd, y = tape[li]
        dy = np.where(y > 0, d, d * slope)
        dg = (dy * xhat).sum(axis=0)
        db = dy.sum(axis=0)
        gx = dy * p["g"]
        dpre = rstd * (gx - gx.mean(axis=1, keepdims=True)
                       - xhat * (gx * xhat).mean(axis=1, keepdims=True))
        dWl = dpre.T @ agg
        dbl = dpre.sum(axis=0)
        dWr = dpre.T @ h
        dagg = dpre @ p["Wl"]
        dh = dpre @ p["Wr"] + a.T @ dagg
        grads[li] = dict(Wl=dWl, bl=dbl, Wr=dWr, g=dg, b=db)
        d = dh
    return d, grads
