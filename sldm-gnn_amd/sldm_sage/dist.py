"""Multi-GPU SageBlock: destination-row partition + RCCL halo exchange.

No reference counterpart (the reference has no distributed code, SURVEY.md
§2, §8e): a full-graph SageBlock forward/backward shards naturally by
destination node because the mean aggregation of row i reads only i's
in-edges, and the dense part, LayerNorm and activation are row-local.

Rank r owns the contiguous node rows [r*P, min((r+1)*P, N)), P = ceil(N/W):
  * its in-edges as a CSR by destination (rows = own nodes, col = GLOBAL
    source ids) for the forward aggregation;
  * its out-edges as a CSR by source (rows = own nodes, col = GLOBAL
    destination ids) for the backward (transpose) aggregation.
Per layer:
  forward   x_full = all_gather(x_local)          (RCCL, [W*P, F])
            agg    = gather-mean over own in-edges from x_full
            out    = dense + LayerNorm + act + dropout on own rows
  backward  dh, [dAgg/deg | dx_root] on own rows
            g_full = all_gather(dAgg/deg)          (RCCL, [W*P, F_in])
            dx     = dx_root + transpose gather over own out-edges from g_full
            weight grads: one bucketed all_reduce(SUM) per layer
The all-gathered buffer is laid out rank-major with P rows per rank, so a
global node id indexes it directly.  Rows are summed in the same CSR order
as on one GPU, and dropout keys use global row ids, so W ranks reproduce the
single-GPU result.

The per-rank compute goes through a backend object (default: the HIP ops);
the CPU tests plug a plain-torch backend in to run the same protocol over
gloo.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn as nn

from .graph import SageGraph


class HipBackend:
    """Per-rank compute on libsldm_sage.so (the product path)."""

    @staticmethod
    def csr(edge_index, num_nodes, transpose):
        from . import ops
        rowptr, col, t_rowptr, t_col, bad = ops.csr_build(edge_index, num_nodes, transpose)
        if edge_index.size(1) and int(bad.item()) != 0:
            raise IndexError(f"edge_index holds a node id outside [0, {num_nodes})")
        return rowptr, col, t_rowptr, t_col

    @staticmethod
    def gather(x, rowptr, col, num_rows, mean, addend=None):
        from . import ops
        return ops.gather_rows(x, rowptr, col, num_rows, mean=mean, addend=addend,
                               name="gather_fwd" if mean else "gather_bwd")

    @staticmethod
    def layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed, save, row_offset):
        from . import dense
        return dense.sage_layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed,
                                    save, row_offset=row_offset)

    @staticmethod
    def post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed, zout, row_offset):
        from . import ops
        return ops.post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed,
                            dh_dtype=xhat.dtype, zout=zout, row_offset=row_offset)

    @staticmethod
    def bwd_data(dh, wl, wr, rowptr):
        from . import dense
        return dense.sage_linear_bwd_data(dh, wl, wr, rowptr)

    @staticmethod
    def bwd_weight(dh, agg, x):
        from . import dense
        return dense.sage_linear_bwd_weight(dh, agg, x)


@dataclass
class GraphPartition:
    """One rank's share of a graph (see module docstring)."""

    rank: int
    world: int
    num_nodes: int
    rows_per_rank: int           # P
    row_begin: int
    row_end: int
    fwd: SageGraph               # rows = own nodes (local), col = global sources
    bwd: SageGraph               # rows = own nodes (local), col = global destinations
    num_local_edges: int         # in-edges of own rows

    @property
    def num_rows(self) -> int:
        return self.row_end - self.row_begin


def partition_graph(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                    backend=HipBackend) -> GraphPartition:
    """Build rank ``rank``'s partition from the full edge_index (same on every
    rank; it may live on any device the backend accepts)."""
    P = (num_nodes + world - 1) // world
    r0, r1 = min(rank * P, num_nodes), min((rank + 1) * P, num_nodes)
    src, dst = edge_index[0], edge_index[1]
    ein = edge_index[:, (dst >= r0) & (dst < r1)]     # original order kept
    eout = edge_index[:, (src >= r0) & (src < r1)]
    rp, col, _, _ = backend.csr(ein, num_nodes, False)
    _, _, trp, tcol = backend.csr(eout, num_nodes, True)
    n = r1 - r0
    fwd = SageGraph(n, int(ein.size(1)), rp[r0:r1 + 1], col, None, None)
    bwd = SageGraph(n, int(eout.size(1)), trp[r0:r1 + 1], tcol, None, None)
    return GraphPartition(rank, world, num_nodes, P, r0, r1, fwd, bwd, int(ein.size(1)))


def _all_gather_rows(x_local: torch.Tensor, part: GraphPartition, group) -> torch.Tensor:
    """[n_local, F] -> [W*P, F], rank-major, P rows per rank (tail padded)."""
    P, F = part.rows_per_rank, x_local.size(1)
    if x_local.size(0) != P:
        padded = x_local.new_zeros(P, F)
        padded[: x_local.size(0)] = x_local
        x_local = padded
    out = x_local.new_empty(part.world * P, F)
    dist.all_gather_into_tensor(out, x_local.contiguous(), group=group)
    return out


class _DistLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wl, bl, wr, gamma, beta, part: GraphPartition, group, backend,
                slope, drop_p, seed, eps):
        x_full = _all_gather_rows(x, part, group)
        agg = backend.gather(x_full, part.fwd.rowptr, part.fwd.col, part.num_rows, True)
        save = any(ctx.needs_input_grad[:6])
        out, xhat, rstd = backend.layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p,
                                            seed, save, part.row_begin)
        if save:
            ctx.save_for_backward(x, agg, xhat, rstd, wl, wr, gamma, beta, out)
            ctx.part, ctx.group, ctx.backend = part, group, backend
            ctx.cfg = (slope, drop_p, seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, agg, xhat, rstd, wl, wr, gamma, beta, out = ctx.saved_tensors
        part, group, be = ctx.part, ctx.group, ctx.backend
        slope, drop_p, seed = ctx.cfg
        dh, dgamma, dbeta, dbl = be.post_bwd(dout.contiguous(), xhat, rstd, gamma, beta, slope,
                                             drop_p, seed, out, part.row_begin)
        dwl, dwr = be.bwd_weight(dh, agg, x)
        # one bucketed all-reduce of this layer's weight gradients (fp32)
        flat = torch.cat([t.reshape(-1).float() for t in (dwl, dbl, dwr, dgamma, dbeta)])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        sizes = [t.numel() for t in (dwl, dbl, dwr, dgamma, dbeta)]
        dwl, dbl, dwr, dgamma, dbeta = (c.view_as(t) for c, t in zip(
            torch.split(flat, sizes), (dwl, dbl, dwr, dgamma, dbeta)))
        g, dx_r = be.bwd_data(dh, wl, wr, part.fwd.rowptr)
        g_full = _all_gather_rows(g.contiguous(), part, group)
        dx = be.gather(g_full, part.bwd.rowptr, part.bwd.col, part.num_rows, False,
                       addend=dx_r.contiguous())
        return (dx, dwl.to(wl.dtype), dbl.to(wl.dtype), dwr.to(wr.dtype), dgamma.to(gamma.dtype),
                dbeta.to(beta.dtype), None, None, None, None, None, None, None)


class DistSageBlock(nn.Module):
    """Runs a :class:`~sldm_sage.SageBlock`'s parameters over a partitioned graph.

    ``forward(x_local)`` takes this rank's rows [row_begin, row_end) of the
    node features and returns the same rows of the block's output; after
    ``backward`` every rank holds the full (summed) parameter gradients,
    identical to a single-device run.  Parameters are broadcast from rank 0
    at construction.
    """

    def __init__(self, block: nn.Module, partition: GraphPartition, group=None,
                 backend=HipBackend, broadcast_params: bool = True):
        super().__init__()
        self.block = block
        self.part = partition
        self.group = group
        self.backend = backend
        if broadcast_params and partition.world > 1:
            with torch.no_grad():
                for p in block.parameters():
                    dist.broadcast(p.data, src=0, group=group)

    def forward(self, x_local: torch.Tensor) -> torch.Tensor:
        from .sageblock import _act_slope, _drop_p, _new_seed
        x = x_local.contiguous()
        for conv, post in zip(self.block.convs, self.block.posts):
            ln, act, drop = post[0], post[1], post[2]
            p = _drop_p(drop)
            seed = _new_seed() if p > 0 else 0
            x = _DistLayerFn.apply(x, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight,
                                   ln.weight, ln.bias, self.part, self.group, self.backend,
                                   _act_slope(act), p, seed, float(ln.eps))
        return x
