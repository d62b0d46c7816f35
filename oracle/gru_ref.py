"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the model's GRU (torch.nn.GRU, one layer, as built at
/root/reference/src/models/grusage.py:66-71 and called at :160-161): PyTorch's
cell (aten/src/ATen/native/RNN.cpp ``GRUCell``) unrolled over time in plain
fp32 torch ops --

    gi = x_t W_ih^T + b_ih,  gh = h W_hh^T + b_hh       (gate order r, z, n)
    r = sigmoid(gi_r + gh_r),  z = sigmoid(gi_z + gh_z)
    n = tanh(gi_n + r * gh_n),  h' = (h - n) * z + n

Pinned on CPU against torch.nn.GRU itself (the reference's op, available in
this image: tests/test_oracle.py), so the GPU tests may check the HIP GRU
against either.  Who may import this module: ``tests/`` only.
"""
from __future__ import annotations

import torch


def gru_ref(x: torch.Tensor, w_ih, w_hh, b_ih=None, b_hh=None, h0=None, batch_first=True):
    """Returns (out, h_n) like ``nn.GRU.forward`` (one layer); differentiable."""
    xb = x if batch_first else x.transpose(0, 1)
    N, T, _ = xb.shape
    H = w_hh.size(1)
    h = h0.reshape(N, H) if h0 is not None else xb.new_zeros(N, H)
    outs = []
    for t in range(T):
        gi = xb[:, t] @ w_ih.t()
        gh = h @ w_hh.t()
        if b_ih is not None:
            gi = gi + b_ih
        if b_hh is not None:
            gh = gh + b_hh
        i_r, i_z, i_n = gi.chunk(3, 1)
        h_r, h_z, h_n = gh.chunk(3, 1)
        r = torch.sigmoid(h_r + i_r)
        z = torch.sigmoid(h_z + i_z)
        n = torch.tanh(i_n + h_n * r)
        h = (h - n) * z + n
        outs.append(h)
    out = torch.stack(outs, 1)
    if not batch_first:
        out = out.transpose(0, 1)
    return out, h.unsqueeze(0)
