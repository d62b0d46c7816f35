"""Multi-GPU SageBlock: destination-row partition + RCCL halo exchange.

No reference counterpart (the reference has no distributed code, SURVEY.md
§2, §8e): a full-graph SageBlock forward/backward shards naturally by
destination node because the mean aggregation of row i reads only i's
in-edges, and the dense part, LayerNorm and activation are row-local.

Rank r owns the contiguous node rows [r*P, min((r+1)*P, N)), P = ceil(N/W):
  * its in-edges as a CSR by destination (rows = own nodes) for the forward;
  * its out-edges as a CSR by source (rows = own nodes) for the backward.
Column ids are remapped at partition time into a per-rank *halo buffer*:
positions [0, n_own) are the rank's own rows, the rest are the remote rows it
actually references, grouped by owner (sorted).  A halo *plan* per direction
holds, for every peer, which of our rows it needs (send list) and how many of
its rows we receive; the lists are exchanged once, at partition time.
Per layer (RCCL ops are issued async and run on RCCL's stream):
  forward   buf = [x_own | all_to_all_v(x_own[send_idx])]      (in flight)
            agg = gather-mean, first over rows whose in-edges read only own
                  rows, then (after the wait) over rows that read halo rows
            out = dense + LayerNorm + act + dropout on own rows
  backward  dh, [dAgg/deg | dx_root] on own rows
            buf = [g_own | all_to_all_v(g_own[send_idx])]       (in flight)
            weight-grad GEMM + one bucketed all_reduce(SUM)      (in flight)
            dx  = dx_root + transpose gather, halo-free rows first, then the rest
Only referenced rows cross xGMI (on a uniform random graph with E/N = 10 and
8 ranks that is ~71% of the remote rows; on a partition-local graph far
fewer).  Each row's edges are summed in the same order as on one GPU and
dropout keys use global row ids, so W ranks reproduce the single-GPU result.

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
    def gather(x, rowptr, col, num_rows, mean, addend=None, rows=None, out=None):
        """Rows ``rows`` (a :class:`RowSubset`; all rows when None) of the CSR
        gather, written into ``out`` (allocated when None)."""
        from . import ops
        name = "gather_fwd" if mean else "gather_bwd"
        if rows is None:
            return ops.gather_rows(x, rowptr, col, num_rows, mean=mean, addend=addend, out=out,
                                   name=name)
        if out is None:
            out = torch.empty(num_rows, x.size(1), dtype=x.dtype, device=x.device)
        return ops.gather_rows(x, rowptr, col, rows.rows.numel(), mean=mean, addend=addend,
                               out=out, name=name, order=rows.rows, edges=rows.edges)

    @staticmethod
    def pick_rows(x, rowptr, idx):
        """x[idx] through the gather kernel (one-edge rows, no mean)."""
        from . import ops
        return ops.gather_rows(x, rowptr, idx, idx.numel(), mean=False, name="halo_pack")

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
class HaloPlan:
    """Which own rows go to which peer, and how many rows come back."""

    send_idx: torch.Tensor        # local row ids, grouped by destination peer
    send_rowptr: torch.Tensor     # identity CSR (arange) for the pack gather
    send_counts: list[int]
    recv_counts: list[int]

    @property
    def num_recv(self) -> int:
        return sum(self.recv_counts)


@dataclass
class RowSubset:
    rows: torch.Tensor            # int32 local row ids
    edges: int                    # in-edges of those rows


@dataclass
class RowSplit:
    """A partition graph's rows split by whether they read halo rows.

    ``resident`` rows read only own rows, so they are aggregated while the
    halo exchange is in flight; ``pending`` rows wait for it.  Each row is
    still summed in CSR order by one kernel, so results are unchanged."""

    resident: RowSubset
    pending: RowSubset


def _split_rows(g: SageGraph, n_own: int) -> RowSplit | None:
    n = g.num_nodes
    if n == 0 or g.num_edges == 0:
        return None
    dev = g.rowptr.device
    deg = (g.rowptr[1:] - g.rowptr[:-1]).long()
    row_of_edge = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    halo_edge = g.col[: g.num_edges].long() >= n_own
    if not bool(halo_edge.any()):
        return None
    has_halo = torch.zeros(n, dtype=torch.bool, device=dev)
    has_halo[row_of_edge[halo_edge]] = True
    pend = has_halo.nonzero().squeeze(1)
    res = (~has_halo).nonzero().squeeze(1)
    pend_edges = int(deg[pend].sum())
    return RowSplit(RowSubset(res.to(torch.int32), g.num_edges - pend_edges),
                    RowSubset(pend.to(torch.int32), pend_edges))


@dataclass
class GraphPartition:
    """One rank's share of a graph (see module docstring)."""

    rank: int
    world: int
    num_nodes: int
    rows_per_rank: int           # P
    row_begin: int
    row_end: int
    fwd: SageGraph               # rows = own nodes, col = halo-buffer positions (sources)
    bwd: SageGraph               # rows = own nodes, col = halo-buffer positions (destinations)
    fwd_plan: HaloPlan
    bwd_plan: HaloPlan
    fwd_split: RowSplit | None = None   # overlap schedule of the forward gather
    bwd_split: RowSplit | None = None   # ... and of the transpose gather

    @property
    def num_rows(self) -> int:
        return self.row_end - self.row_begin

    def halo_rows(self) -> tuple[int, int]:
        """(rows received in the forward exchange, in the backward exchange)."""
        return self.fwd_plan.num_recv, self.bwd_plan.num_recv


def _exchange_counts(counts: list[int], device, group) -> list[int]:
    world = len(counts)
    if world == 1:
        return list(counts)
    send = torch.tensor(counts, dtype=torch.int64, device=device)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv.tolist()


def _build_plan(ids: torch.Tensor, r0: int, r1: int, P: int, world: int, group):
    """ids: global node ids this rank references (any order, duplicates ok).

    Returns (remap, plan): remap(global ids) -> halo-buffer positions."""
    dev = ids.device
    uniq = torch.unique(ids)                                   # sorted
    remote = uniq[(uniq < r0) | (uniq >= r1)]                  # sorted => grouped by owner
    owner = torch.div(remote, P, rounding_mode="floor")
    need_counts = torch.bincount(owner, minlength=world)[:world].tolist()
    give_counts = _exchange_counts(need_counts, dev, group)
    # tell each owner which of its rows we need (global ids), learn what to send
    if world > 1:
        wanted = torch.empty(sum(give_counts), dtype=torch.int64, device=dev)
        dist.all_to_all_single(wanted, remote.to(torch.int64).contiguous(),
                               output_split_sizes=give_counts,
                               input_split_sizes=need_counts, group=group)
    else:
        wanted = remote.to(torch.int64)
    send_idx = (wanted - r0).to(torch.int32)
    n_own = r1 - r0

    def remap(g: torch.Tensor) -> torch.Tensor:
        own = (g >= r0) & (g < r1)
        pos = torch.searchsorted(remote, g)
        return torch.where(own, g - r0, n_own + pos).to(torch.int32)

    rowptr = torch.arange(send_idx.numel() + 1, dtype=torch.int32, device=dev)
    return remap, HaloPlan(send_idx, rowptr, give_counts, need_counts)


def partition_graph(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                    backend=HipBackend, group=None) -> GraphPartition:
    """Build rank ``rank``'s partition from the full edge_index (same on every
    rank).  Collective over ``group`` (the halo lists are exchanged here)."""
    P = (num_nodes + world - 1) // world
    r0, r1 = min(rank * P, num_nodes), min((rank + 1) * P, num_nodes)
    n = r1 - r0
    src, dst = edge_index[0], edge_index[1]
    ein = edge_index[:, (dst >= r0) & (dst < r1)]     # original order kept
    eout = edge_index[:, (src >= r0) & (src < r1)]
    remap_f, plan_f = _build_plan(ein[0], r0, r1, P, world, group)
    remap_b, plan_b = _build_plan(eout[1], r0, r1, P, world, group)
    n_buf_f = n + plan_f.num_recv
    n_buf_b = n + plan_b.num_recv
    # CSR by (local) destination over buffer-position sources, and by (local)
    # source over buffer-position destinations; stable, so edge order is kept.
    fin = torch.stack([remap_f(ein[0]).long(), (ein[1] - r0).long()])
    fout = torch.stack([(eout[0] - r0).long(), remap_b(eout[1]).long()])
    rp, col, _, _ = backend.csr(fin, max(n_buf_f, 1), False)
    _, _, trp, tcol = backend.csr(fout, max(n_buf_b, 1), True)
    fwd = SageGraph(n, int(ein.size(1)), rp[: n + 1], col, None, None)
    bwd = SageGraph(n, int(eout.size(1)), trp[: n + 1], tcol, None, None)
    return GraphPartition(rank, world, num_nodes, P, r0, r1, fwd, bwd, plan_f, plan_b,
                          _split_rows(fwd, n), _split_rows(bwd, n))


def _overlapped_gather(backend, buf, work, g: SageGraph, split: RowSplit | None, num_rows,
                       mean, addend=None):
    """The partition gather with the halo exchange ``work`` in flight: rows
    that read only own rows first, then (after ``work.wait()``) the rest."""
    if work is None or split is None:
        if work is not None:
            work.wait()
        return backend.gather(buf, g.rowptr, g.col, num_rows, mean, addend=addend)
    out = backend.gather(buf, g.rowptr, g.col, num_rows, mean, addend=addend,
                         rows=split.resident)
    work.wait()
    return backend.gather(buf, g.rowptr, g.col, num_rows, mean, addend=addend,
                          rows=split.pending, out=out)


def _halo_buffer(x_own: torch.Tensor, plan: HaloPlan, backend, group, async_op=False):
    """[x_own ; rows received from peers] (the layout the remapped CSR indexes).

    With ``async_op`` returns (buf, work): the exchange runs on RCCL's stream
    while the caller queues independent kernels; ``work.wait()`` before use."""
    n, F = x_own.shape
    if plan.num_recv == 0 and sum(plan.send_counts) == 0:
        return (x_own, None) if async_op else x_own   # nothing crosses: no copy
    buf = x_own.new_empty(n + plan.num_recv, F)
    buf[:n].copy_(x_own)
    work = None
    if plan.num_recv or sum(plan.send_counts):
        send = (backend.pick_rows(x_own, plan.send_rowptr, plan.send_idx)
                if plan.send_idx.numel() else x_own.new_empty(0, F))
        work = dist.all_to_all_single(buf[n:], send, output_split_sizes=plan.recv_counts,
                                      input_split_sizes=plan.send_counts, group=group,
                                      async_op=async_op)
    return (buf, work) if async_op else buf


class _DistLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wl, bl, wr, gamma, beta, part: GraphPartition, group, backend,
                slope, drop_p, seed, eps):
        # halo exchange on RCCL's stream; rows that read only own rows are
        # aggregated meanwhile (buf[:n] is already the own block)
        buf, work = _halo_buffer(x, part.fwd_plan, backend, group, async_op=True)
        agg = _overlapped_gather(backend, buf, work, part.fwd, part.fwd_split, part.num_rows,
                                 True)
        del buf
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
        # dAgg/deg first, so its halo exchange (RCCL stream) overlaps the
        # weight-gradient GEMM and all-reduce queued behind it.
        g, dx_r = be.bwd_data(dh, wl, wr, part.fwd.rowptr)
        buf, xwork = _halo_buffer(g.contiguous(), part.bwd_plan, be, group, async_op=True)
        dwl, dwr = be.bwd_weight(dh, agg, x)
        # one bucketed all-reduce of this layer's weight gradients (fp32)
        grads = (dwl, dbl, dwr, dgamma, dbeta)
        flat = torch.cat([t.reshape(-1).float() for t in grads])
        rwork = None
        if part.world > 1:
            rwork = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=True)
        dx = _overlapped_gather(be, buf, xwork, part.bwd, part.bwd_split, part.num_rows, False,
                                addend=dx_r.contiguous())
        if rwork is not None:
            rwork.wait()
        dwl, dbl, dwr, dgamma, dbeta = (c.view_as(t) for c, t in zip(
            torch.split(flat, [t.numel() for t in grads]), grads))
        return (dx, dwl.to(wl.dtype), dbl.to(wl.dtype), dwr.to(wr.dtype), dgamma.to(gamma.dtype),
                dbeta.to(beta.dtype), None, None, None, None, None, None, None)


class DistSageBlock(nn.Module):
    """Runs a :class:`~sldm_sage.SageBlock`'s parameters over a partitioned graph.

    ``forward(x_local)`` takes this rank's rows [row_begin, row_end) of the
    node features and returns the same rows of the block's output; after
    ``backward`` every rank holds the full (summed) parameter gradients,
    identical to a single-device run.  Parameters are broadcast from rank 0
    at construction.  Seed every rank identically (dropout draws).
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
