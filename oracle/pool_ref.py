"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the graph-level readout that follows the SageBlock in
the reference:

* selection: /root/reference/src/models/grusage.py:119-127
  ('mean' -> global_mean_pool, 'max' -> global_max_pool,
  'double' -> cat([mean, max], dim=1));
* call: grusage.py:185 ``x = self.global_pool(x, batch)``;
* the pools are torch-geometric==2.7.0 (uv.lock:1406-1407, absent here):
  ``global_mean_pool(x, batch, size)`` and ``global_max_pool`` reduce with
  ``torch_geometric.utils.scatter`` at ``dim_size = batch.max() + 1``; on the
  reference's CPU path (no torch_scatter) that is, op for op:

      mean: count = zeros(B).scatter_add_(0, batch, ones(N)).clamp(min=1)
            zeros(B,F).scatter_add_(0, batch[:,None].expand_as(x), x) / count[:,None]
      max:  zeros(B,F).scatter_reduce_(0, batch[:,None].expand_as(x), x,
                                       reduce='amax', include_self=False)

  ``batch=None`` pools every row into one graph: ``x.mean(dim=-2,
  keepdim=True)`` / ``x.max(dim=-2, keepdim=True)[0]`` (gradient to the
  first maximal row).  Autograd of these ops is the reference gradient (for
  amax: the evenly split tie gradient of torch's scatter_reduce backward).

Who may import this module: ``tests/`` only.  PARITY UNPINNED (no reference
fixtures exist): pinned by the hand-computed known answers in
tests/test_oracle.py.
"""
from __future__ import annotations

import torch


def _size(batch: torch.Tensor, size: int | None) -> int:
    if size is not None:
        return int(size)
    return int(batch.max()) + 1 if batch.numel() else 0


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    if batch is None:
        return x.mean(dim=-2, keepdim=True)
    B = _size(batch, size)
    count = x.new_zeros(B).scatter_add_(0, batch, x.new_ones(x.size(0))).clamp(min=1)
    idx = batch.view(-1, 1).expand_as(x)
    return x.new_zeros(B, x.size(1)).scatter_add_(0, idx, x) / count.view(-1, 1)


def global_max_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    if batch is None:
        return x.max(dim=-2, keepdim=True)[0]
    B = _size(batch, size)
    idx = batch.view(-1, 1).expand_as(x)
    return x.new_zeros(B, x.size(1)).scatter_reduce_(0, idx, x, reduce="amax",
                                                     include_self=False)


def global_mean_max_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    return torch.cat([global_mean_pool(x, batch, size), global_max_pool(x, batch, size)], dim=1)
