"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the reference's SageBlock hot path, in plain PyTorch fp32
(no torch_geometric), op for op:

* structure, parameter names, post stack:
  /root/reference/src/models/blocks/sageblock.py:4-20
* per-layer conv: torch-geometric==2.7.0 ``SAGEConv`` with default arguments
  (aggr='mean', normalize=False, root_weight=True, project=False, bias=True),
  instantiated at sageblock.py:8 and called at sageblock.py:18.  PyG is a
  third-party dependency pinned at /root/reference/uv.lock:1406-1407; it is
  absent from /root/reference and from this image, so its published
  algorithm is restated here:

      x_j   = x.index_select(0, edge_index[0])                 # MessagePassing._collect
      count = zeros(N).scatter_add_(0, dst, ones(E)).clamp(min=1)
      agg   = zeros(N,F).scatter_add_(0, dst[:,None].expand_as(x_j), x_j) / count[:,None]
      out   = lin_l(agg) + lin_r(x)                            # lin_l has the bias

  followed by LayerNorm(F_out) -> LeakyReLU(ns) | ReLU -> Dropout(p) | Identity
  (sageblock.py:9-15).

Who may import this module: ``tests/``, ``__graft_entry__.smoke()`` (as the
checker) and ``bench.py``'s ``cpu_baseline`` leg (as the timed CPU path).  The
product package ``sldm_sage`` never imports it.

PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors and its path cannot run here (torch_geometric is not
installed).  This restatement is cross-checked instead against
an independent fp64 dense-matrix formulation (``oracle/dense_ref.py``) and
hand-computed known-answer cases (``tests/test_oracle.py``).
"""
from __future__ import annotations

import torch
import torch.nn as nn


def pyg_scatter_mean(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    """torch_geometric/utils/_scatter.py ``scatter(..., reduce='mean')`` (PyG 2.7.0).

    fp32 count via scatter_add_ of ones, clamp(min=1), fp32 sums via an
    expanded-index scatter_add_, then one division.  Isolated nodes get 0,
    duplicate edges and self-loops are counted, an index >= dim_size raises.
    """
    count = src.new_zeros(dim_size)
    count.scatter_add_(0, index, src.new_ones(src.size(0)))
    count = count.clamp(min=1)
    idx = index.view(-1, 1).expand_as(src)
    out = src.new_zeros((dim_size, src.size(1))).scatter_add_(0, idx, src)
    return out / count.view(-1, 1)


def pyg_sage_aggregate(x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    """MessagePassing.propagate with flow='source_to_target' and MeanAggregation.

    Messages are rows ``x[edge_index[0]]``; they aggregate at ``edge_index[1]``;
    ``dim_size`` is ``x.size(0)`` (SAGEConv passes size=None, x=(x, x)).
    """
    n = x.size(0)
    if edge_index.numel() and (int(edge_index.min()) < 0 or int(edge_index.max()) >= n):
        raise IndexError("edge_index holds a node id outside [0, N)")
    x_j = x.index_select(0, edge_index[0])
    return pyg_scatter_mean(x_j, edge_index[1], n)


class RefSAGEConv(nn.Module):
    """PyG 2.7.0 ``SAGEConv(in, out)`` with default arguments (sageblock.py:8).

    ``lin_l`` (bias) is applied to the mean aggregate, ``lin_r`` (no bias) to
    the root features; no L2 normalisation, no projection.
    """

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin_l = nn.Linear(in_channels, out_channels, bias=True)
        self.lin_r = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        out = pyg_sage_aggregate(x, edge_index)
        out = self.lin_l(out)
        out = out + self.lin_r(x)
        return out


class RefSageBlock(nn.Module):
    """/root/reference/src/models/blocks/sageblock.py:4-20, verbatim in behaviour."""

    def __init__(self, hdims: list[int], dropout: float | None = None,
                 negative_slope: float | None = None):
        super().__init__()
        assert len(hdims) >= 1, "hdims must contain at least one element"
        self.convs = nn.ModuleList([RefSAGEConv(hdims[i], hdims[i + 1])
                                    for i in range(len(hdims) - 1)])
        self.posts = nn.ModuleList([
            nn.Sequential(
                nn.LayerNorm(hdims[i + 1]),
                nn.LeakyReLU(negative_slope=negative_slope) if negative_slope is not None else nn.ReLU(),
                nn.Dropout(p=dropout) if dropout is not None else nn.Identity(),
            ) for i in range(len(hdims) - 1)
        ])

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        for conv, post in zip(self.convs, self.posts):
            x = conv(x, edge_index)
            x = post(x)
        return x


def set_synthetic_params(block: nn.Module, seed: int = 1) -> None:
    """Deterministic weights for parity runs: lin weights and
    bias uniform ±1/sqrt(F_in) from ``torch.Generator().manual_seed(seed)``;
    LayerNorm weight 1, bias 0 (torch defaults).  Works on any module with the
    reference's state_dict layout."""
    g = torch.Generator().manual_seed(seed)
    sd = block.state_dict()
    new = {}
    for k, v in sd.items():
        if ".lin_" in k:
            fan_in = v.shape[-1] if v.dim() == 2 else sd[k.replace("bias", "weight")].shape[1]
            bound = 1.0 / fan_in ** 0.5
            new[k] = (torch.rand(v.shape, generator=g, dtype=torch.float32) * 2 - 1) * bound
        else:
            new[k] = v.clone()
    block.load_state_dict(new)


def random_graph(num_nodes: int, num_edges: int, feat: int, seed: int = 0):
    """Synthetic parity inputs: src, dst independent uniform
    randint(0, N, (E,)) stacked to int64 [2,E] (duplicates and self-loops
    allowed), x ~ N(0,1) [N,F] fp32, all from torch.Generator().manual_seed(seed)."""
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, num_nodes, (num_edges,), generator=g, dtype=torch.int64)
    dst = torch.randint(0, num_nodes, (num_edges,), generator=g, dtype=torch.int64)
    x = torch.randn(num_nodes, feat, generator=g, dtype=torch.float32)
    return torch.stack([src, dst]), x


def khop_subgraph(edge_index: torch.Tensor, targets: torch.Tensor, num_layers: int,
                  num_nodes: int):
    """In-neighbourhood subgraph that reproduces the targets' L-layer outputs.

    A node at in-hop distance h < L needs ALL its in-edges; nodes at hop L
    are leaves.  Returns (nodes, sub_edge_index, target_pos) where ``nodes``
    are global ids (targets first) and sub_edge_index is relabelled.  The
    aggregation of a node at hop h is exact up to layer L-h, so targets are
    exact at layer L, and for a loss that reads only target rows every
    parameter gradient and every input gradient of the full graph equals the
    subgraph's.
    """
    src, dst = edge_index[0], edge_index[1]
    order = torch.argsort(dst, stable=True)
    dst_sorted = dst[order]
    rowptr = torch.searchsorted(dst_sorted, torch.arange(num_nodes + 1))
    seen = {int(t): i for i, t in enumerate(targets.tolist())}
    nodes = [int(t) for t in targets.tolist()]
    frontier = list(nodes)
    keep_edges = []
    for _ in range(num_layers):
        nxt = []
        for v in frontier:
            lo, hi = int(rowptr[v]), int(rowptr[v + 1])
            eids = order[lo:hi]
            keep_edges.append(eids)
            for u in src[eids].tolist():
                if u not in seen:
                    seen[u] = len(nodes)
                    nodes.append(u)
                    nxt.append(u)
        frontier = nxt
    eids = torch.cat(keep_edges) if keep_edges else torch.empty(0, dtype=torch.int64)
    eids = torch.sort(eids).values          # keep the original edge order
    remap = torch.full((num_nodes,), -1, dtype=torch.int64)
    nodes_t = torch.tensor(nodes, dtype=torch.int64)
    remap[nodes_t] = torch.arange(len(nodes))
    sub = torch.stack([remap[src[eids]], remap[dst[eids]]])
    return nodes_t, sub, torch.arange(len(targets))
