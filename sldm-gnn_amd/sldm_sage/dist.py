"""Multi-GPU SageBlock: destination-row partition + RCCL halo exchange.

No reference counterpart (the reference has no distributed code): a full-graph SageBlock forward/backward shards naturally by
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

A second strategy, *feature slicing* (:func:`partition_features`), serves
graphs where any row partition cuts nearly every edge (uniform random graphs:
the halo is ~71% of all rows at W = 8 and ~99% at W = 2).  Every rank keeps
the whole graph's CSR and aggregates ALL rows over its own slice of the
feature columns, so the gathers need no halo; the dense part stays on the
rank's row block, and layouts are switched by balanced all-to-alls:
  forward   x_cols = row->col(x_own)                   [N, F/W]
            agg_cols = gather-mean(x_cols)             all rows, own columns
            agg_own  = col->row(agg_cols)              [P, F]
            out = dense + LayerNorm + act + dropout on own rows
  backward  dh, [g = dAgg/deg | dx_root] on own rows
            g_cols = row->col(g)       (in flight with the weight-grad GEMM)
            dx = dx_root + col->row(transpose-gather(g_cols))
Per layer a rank moves 4 x (W-1)/W^2 x N x F x s bytes, against
2 x halo x F x s for the row partition (C4 at W = 8: 2.2 GB vs 6.4 GB), the
load is balanced by construction (power-law in-degrees included) and each
element is still summed in CSR order (fp32: bit-identical to one GPU; bf16:
the backward's two-term add rounds once more).  :func:`plan_partition`
picks the strategy with the lowest modelled time -- including *replicate*
(no sharding, every rank runs the whole block) for graphs where any
partition would move more bytes over xGMI than one GPU needs to do all the
work (a uniform random graph at W = 2: one link per peer).

The per-rank compute goes through a backend object (default: the HIP ops);
the CPU tests plug a plain-torch backend in to run the same protocol over
gloo.
"""
from __future__ import annotations

from dataclasses import dataclass

import os
import sys
import time

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
    def gather(x, rowptr, col, num_rows, mean, addend=None, rows=None, out=None, edges=None,
               hub=None):
        """Rows ``rows`` (a :class:`RowSubset`; all rows when None) of the CSR
        gather, written into ``out`` (allocated when None).  ``edges``: the
        edge count of a rowptr window (byte accounting only).  ``hub``: the
        high-degree split plan of all rows (a subset carries its own)."""
        from . import ops
        name = "gather_fwd" if mean else "gather_bwd"
        if rows is None:
            return ops.gather_rows(x, rowptr, col, num_rows, mean=mean, addend=addend, out=out,
                                   name=name, edges=edges, hub=hub)
        if out is None:
            out = torch.empty(num_rows, x.size(1), dtype=x.dtype, device=x.device)
        return ops.gather_rows(x, rowptr, col, rows.rows.numel(), mean=mean, addend=addend,
                               out=out, name=name, order=rows.rows, edges=rows.edges,
                               hub=rows.hub)

    @staticmethod
    def pick_rows(x, rowptr, idx):
        """x[idx] through the gather kernel (one-edge rows, no mean)."""
        from . import ops
        return ops.gather_rows(x, rowptr, idx, idx.numel(), mean=False, name="halo_pack")

    @staticmethod
    def layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed, save, row_offset,
                  outs=None):
        """Fused dense + post stack; ``outs`` = preallocated (out, xhat, rstd)."""
        from . import dense
        return dense.sage_layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope, drop_p, seed,
                                    save, row_offset=row_offset, outs=outs)

    @staticmethod
    def post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed, zout, row_offset):
        from . import ops
        return ops.post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed,
                            dh_dtype=xhat.dtype, row_offset=row_offset)

    @staticmethod
    def bwd_data(dh, wl, wr, rowptr):
        from . import dense
        return dense.sage_linear_bwd_data(dh, wl, wr, rowptr)

    @staticmethod
    def bwd_weight(dh, agg, x):
        from . import dense
        return dense.sage_linear_bwd_weight(dh, agg, x)

    @staticmethod
    def bwd_data_blocked_ok(dh, fi, cs):
        """Whether :meth:`bwd_data_blocked` takes this dtype / shape."""
        from . import dense
        return dense.sage_linear_bwd_data_blocked_ok(dh, fi, cs)

    @staticmethod
    def bwd_data_blocked(dh, wcat_t, rowptr, fi, cs, dx_root):
        """bwd_data on a row window with dAgg / deg written straight in the
        all-to-all's send layout (flat [F_in / cs][rows][cs])."""
        from . import dense
        return dense.sage_linear_bwd_data_blocked(dh, wcat_t, rowptr, fi, cs, dx_root)

    @staticmethod
    def cols_pack(rows, nblk, cs):
        """rows [n, nblk*cs] -> flat [nblk][n][cs] (layout.hip; torch for odd widths)."""
        from . import ops
        if ops.cols_layout_ok(rows, cs) and rows.stride(1) == 1:
            return ops.cols_pack(rows, nblk, cs)
        return rows.reshape(rows.size(0), nblk, cs).transpose(0, 1).contiguous().view(-1)

    @staticmethod
    def cols_unpack(blocks, n, nblk, cs, out, addend=None):
        """flat [nblk][n][cs] -> out [n, nblk*cs] (+ addend)."""
        from . import ops
        if ops.cols_layout_ok(out, cs):
            return ops.cols_unpack(blocks, n, nblk, cs, out, addend)
        src = blocks.view(nblk, n, cs).transpose(0, 1).reshape(n, nblk * cs)
        if addend is None:
            out.copy_(src)
        else:
            torch.add(addend, src, out=out)
        return out


# ---------------------------------------------------------------------------
# Collectives.  RCCL ("nccl") takes device tensors directly.  Under gloo (the
# CPU tests, and several ranks sharing one GPU in a rehearsal) device tensors
# are staged through host memory explicitly: ``.cpu()`` waits for the
# producing HIP stream, the collective runs on host tensors, and the result is
# copied back on the current stream.  Gloo's own CUDA path (its internal
# streams and pinned staging buffers, raced against our kernels on the current
# stream and the caching allocator) is never used.  Staged calls complete
# synchronously and return ``None`` as their work handle.
# ---------------------------------------------------------------------------
def _host_staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None,
                      async_op: bool = False):
    """``dist.all_to_all_single`` with gloo host staging (module note above)."""
    if _host_staged(out, group):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=group)
        out.copy_(o)
        return None
    return dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                                  input_split_sizes=in_splits, group=group, async_op=async_op)


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None, async_op: bool = False):
    """In-place ``dist.all_reduce`` with gloo host staging."""
    if _host_staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
        return None
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def broadcast(t: torch.Tensor, src: int = 0, group=None) -> None:
    """In-place ``dist.broadcast`` with gloo host staging."""
    if _host_staged(t, group):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
        return
    dist.broadcast(t, src=src, group=group)


# ---------------------------------------------------------------------------
# Row blocks.  Rank r owns the contiguous node rows [bounds[r], bounds[r+1]).
# "rows": equal row counts (P = ceil(N/W)); "cost": cut by the cumulative
# per-node cost (in-degree + out-degree + the dense part's row cost in
# edge-equivalents), a split by cumulative in-degree for
# power-law graphs -- a 10k-in-degree hub then weighs as much as ~10k rows'
# edges instead of one row.
# ---------------------------------------------------------------------------
# dense part per row (13 F s bytes at ~4 TB/s) vs one gathered edge (F s + 4
# bytes at ~5.3 TB/s): ~17 edge-equivalents per row (two gathers per layer).
_ROW_COST_EDGES = 17.0


_TRACE = os.environ.get("SLDM_DIST_TRACE") == "1"
_T0 = time.perf_counter()


def _trace(msg: str) -> None:
    """Per-rank setup timing on stderr (SLDM_DIST_TRACE=1; diagnostics)."""
    if _TRACE:
        r = dist.get_rank() if dist.is_initialized() else 0
        mem = ""
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            free, total = torch.cuda.mem_get_info()
            mem = (f"  [gpu free {free / 2**30:.0f} of {total / 2**30:.0f} GiB,"
                   f" reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB]")
        print(f"[dist r{r}] {time.perf_counter() - _T0:8.2f} s  {msg}{mem}", file=sys.stderr,
              flush=True)


def row_bounds(edge_index: torch.Tensor, num_nodes: int, world: int,
               balance: str = "cost") -> list[int]:
    """[W+1] row offsets of the W contiguous row blocks (same on every rank:
    edge_index is the same everywhere).  ``balance`` = "rows" or "cost"."""
    if balance == "rows" or world == 1 or num_nodes == 0:
        P = (num_nodes + world - 1) // world
        return [min(r * P, num_nodes) for r in range(world + 1)]
    if balance != "cost":
        raise ValueError(f"unknown balance {balance!r} (rows, cost)")
    dev = edge_index.device
    # integer costs (exact, and bincount's int64 atomics are native; fp64
    # index_add_ was the slowest step of partitioning with ranks sharing a GPU)
    w = torch.full((num_nodes,), int(_ROW_COST_EDGES), dtype=torch.int64, device=dev)
    if edge_index.numel():
        w += torch.bincount(edge_index[1].long(), minlength=num_nodes)[:num_nodes]
        w += torch.bincount(edge_index[0].long(), minlength=num_nodes)[:num_nodes]
    cum = torch.cumsum(w, 0)
    total = int(cum[-1])
    targets = torch.tensor([total * r // world for r in range(1, world)], dtype=torch.int64,
                           device=dev)
    cuts = torch.searchsorted(cum, targets).tolist() if world > 1 else []
    bounds = [0] + [min(int(c) + 1, num_nodes) for c in cuts] + [num_nodes]
    for r in range(1, world + 1):        # monotone (empty blocks allowed)
        bounds[r] = max(bounds[r], bounds[r - 1])
    return bounds


def _owner(ids: torch.Tensor, bounds: list[int]) -> torch.Tensor:
    b = torch.tensor(bounds[1:-1], dtype=ids.dtype, device=ids.device)
    return torch.searchsorted(b, ids, right=True)


@dataclass
class HaloPlan:
    """Which own rows go to which peer, and how many rows come back.

    ``active`` is global: whether ANY rank sends or receives anything in this
    exchange (all ranks agree, so they all issue the collective or all skip
    it -- a locally decided skip would desynchronise the process group)."""

    send_idx: torch.Tensor        # local row ids, grouped by destination peer
    send_rowptr: torch.Tensor     # identity CSR (arange) for the pack gather
    send_counts: list[int]
    recv_counts: list[int]
    active: bool = True

    @property
    def num_recv(self) -> int:
        return sum(self.recv_counts)


@dataclass
class RowSubset:
    rows: torch.Tensor            # int32 local row ids
    edges: int                    # in-edges of those rows
    hub: object | None = None     # graph.HubPlan of the subset's high-degree rows


@dataclass
class RowSplit:
    """A partition graph's rows split by whether they read halo rows.

    ``resident`` rows read only own rows, so they are aggregated while the
    halo exchange is in flight; ``pending`` rows wait for it.  Each row is
    still summed in CSR order by one kernel, so results are unchanged."""

    resident: RowSubset
    pending: RowSubset


def _hub_threshold(num_nodes: int, num_edges: int, device) -> int | None:
    """The single-GPU path's high-degree rule (graph.build_graph) for the
    WHOLE graph, so a partition splits exactly the rows one GPU would split,
    into the same chunks: the W-rank sums then equal the one-GPU bits.  None:
    no split (small graphs, the host backend's CPU tensors, SLDM_SKEW)."""
    from . import graph as graph_mod
    if (device.type != "cuda" or num_edges < graph_mod.HUB_MIN_EDGES
            or graph_mod._skew_mode() != "split"):
        return None
    return graph_mod.hub_threshold(num_nodes, num_edges)


def _split_rows(g: SageGraph, n_own: int, hub_thr: int | None = None) -> RowSplit | None:
    """Rows by whether they read halo rows (None: none do).  ``hub_thr``: rows
    above this degree are split into edge chunks (graph.hub_plan); sets
    ``g.hub`` (all rows) and each subset's own plan."""
    from .graph import hub_plan
    n = g.num_nodes
    if n == 0 or g.num_edges == 0:
        return None
    dev = g.rowptr.device
    deg = (g.rowptr[1:] - g.rowptr[:-1]).long()
    skewed = hub_thr is not None and int(deg.max()) > hub_thr
    if skewed:
        g.hub = hub_plan(g.rowptr, hub_thr)
    row_of_edge = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    halo_edge = g.col[: g.num_edges].long() >= n_own
    if not bool(halo_edge.any()):
        return None
    has_halo = torch.zeros(n, dtype=torch.bool, device=dev)
    has_halo[row_of_edge[halo_edge]] = True
    pend = has_halo.nonzero().squeeze(1)
    res = (~has_halo).nonzero().squeeze(1)
    pend_edges = int(deg[pend].sum())
    res_hub = hub_plan(g.rowptr, hub_thr, row_mask=~has_halo) if skewed else None
    pend_hub = hub_plan(g.rowptr, hub_thr, row_mask=has_halo) if skewed else None
    return RowSplit(RowSubset(res.to(torch.int32), g.num_edges - pend_edges, res_hub),
                    RowSubset(pend.to(torch.int32), pend_edges, pend_hub))


@dataclass
class GraphPartition:
    """One rank's share of a graph (see module docstring)."""

    rank: int
    world: int
    num_nodes: int
    bounds: list[int]            # [W+1] row-block offsets (row_bounds)
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

    def exchange_bytes_per_layer(self, feat: int, elem: int) -> int:
        """Bytes this rank sends per layer (forward x rows + backward dAgg rows)."""
        return (sum(self.fwd_plan.send_counts) + sum(self.bwd_plan.send_counts)) * feat * elem


def _exchange_counts(counts: list[int], device, group) -> list[int]:
    world = len(counts)
    if world == 1:
        return list(counts)
    send = torch.tensor(counts, dtype=torch.int64, device=device)
    recv = torch.empty_like(send)
    all_to_all_single(recv, send, None, None, group=group)
    return recv.tolist()


def _build_plan(ids: torch.Tensor, r0: int, r1: int, bounds: list[int], world: int, group):
    """ids: global node ids this rank references (any order, duplicates ok).

    Returns (remap, plan): remap(global ids) -> halo-buffer positions."""
    dev = ids.device
    _trace("build_plan: unique")
    uniq = torch.unique(ids)                                   # sorted
    _trace("build_plan: remote")
    remote = uniq[(uniq < r0) | (uniq >= r1)]                  # sorted => grouped by owner
    owner = _owner(remote, bounds)
    _trace("build_plan: owner counts")
    need_counts = torch.bincount(owner, minlength=world)[:world].tolist()
    _trace("build_plan: exchange counts")
    give_counts = _exchange_counts(need_counts, dev, group)
    _trace("build_plan: exchange ids")
    # tell each owner which of its rows we need (global ids), learn what to send
    if world > 1:
        wanted = torch.empty(sum(give_counts), dtype=torch.int64, device=dev)
        all_to_all_single(wanted, remote.to(torch.int64).contiguous(), give_counts,
                          need_counts, group=group)
        # global decision: does any rank move anything in this exchange?
        tot = torch.tensor([sum(need_counts) + sum(give_counts)], dtype=torch.int64, device=dev)
        all_reduce(tot, group=group)
        active = int(tot.item()) > 0
    else:
        wanted = remote.to(torch.int64)
        active = False
    send_idx = (wanted - r0).to(torch.int32)
    n_own = r1 - r0

    def remap(g: torch.Tensor) -> torch.Tensor:
        own = (g >= r0) & (g < r1)
        pos = torch.searchsorted(remote, g)
        return torch.where(own, g - r0, n_own + pos).to(torch.int32)

    rowptr = torch.arange(send_idx.numel() + 1, dtype=torch.int32, device=dev)
    return remap, HaloPlan(send_idx, rowptr, give_counts, need_counts, active)


def partition_graph(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                    backend=HipBackend, group=None, balance: str = "cost") -> GraphPartition:
    """Build rank ``rank``'s partition from the full edge_index (same on every
    rank).  Collective over ``group`` (the halo lists are exchanged here).
    ``balance``: row blocks of equal size ("rows") or of equal modelled cost
    ("cost", :func:`row_bounds`)."""
    _trace("partition_graph: row bounds")
    bounds = row_bounds(edge_index, num_nodes, world, balance)
    _trace("partition_graph: masks")
    r0, r1 = bounds[rank], bounds[rank + 1]
    n = r1 - r0
    src, dst = edge_index[0], edge_index[1]
    ein = edge_index[:, (dst >= r0) & (dst < r1)]     # original order kept
    eout = edge_index[:, (src >= r0) & (src < r1)]
    _trace("partition_graph: plans")
    remap_f, plan_f = _build_plan(ein[0], r0, r1, bounds, world, group)
    remap_b, plan_b = _build_plan(eout[1], r0, r1, bounds, world, group)
    n_buf_f = n + plan_f.num_recv
    n_buf_b = n + plan_b.num_recv
    # CSR by (local) destination over buffer-position sources, and by (local)
    # source over buffer-position destinations; stable, so edge order is kept.
    fin = torch.stack([remap_f(ein[0]).long(), (ein[1] - r0).long()])
    fout = torch.stack([(eout[0] - r0).long(), remap_b(eout[1]).long()])
    _trace("partition_graph: csr")
    rp, col, _, _ = backend.csr(fin, max(n_buf_f, 1), False)
    _, _, trp, tcol = backend.csr(fout, max(n_buf_b, 1), True)
    _trace("partition_graph: split rows")
    fwd = SageGraph(n, int(ein.size(1)), rp[: n + 1], col, None, None)
    bwd = SageGraph(n, int(eout.size(1)), trp[: n + 1], tcol, None, None)
    thr = _hub_threshold(num_nodes, int(edge_index.size(1)), edge_index.device)
    return GraphPartition(rank, world, num_nodes, bounds, r0, r1, fwd, bwd, plan_f, plan_b,
                          _split_rows(fwd, n, thr), _split_rows(bwd, n, thr))


def _overlapped_gather(backend, buf, work, g: SageGraph, split: RowSplit | None, num_rows,
                       mean, addend=None):
    """The partition gather with the halo exchange ``work`` in flight: rows
    that read only own rows first, then (after ``work.wait()``) the rest."""
    if work is None or split is None:
        if work is not None:
            work.wait()
        return backend.gather(buf, g.rowptr, g.col, num_rows, mean, addend=addend, hub=g.hub)
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
    if not plan.active:
        # no rank moves anything (decided globally at partition time): every
        # rank skips the collective together
        return (x_own, None) if async_op else x_own
    buf = x_own.new_empty(n + plan.num_recv, F)
    buf[:n].copy_(x_own)
    send = (backend.pick_rows(x_own, plan.send_rowptr, plan.send_idx)
            if plan.send_idx.numel() else x_own.new_empty(0, F))
    work = all_to_all_single(buf[n:], send, plan.recv_counts, plan.send_counts, group=group,
                             async_op=async_op)
    if work is not None and async_op:
        # the caching allocator may hand `send`'s block to the next allocation
        # on this stream; keep it alive until the caller waits
        work = _KeepAlive(work, send)
    return (buf, work) if async_op else buf


class _KeepAlive:
    """A collective's work handle that also holds its input buffer."""

    __slots__ = ("work", "keep")

    def __init__(self, work, keep):
        self.work, self.keep = work, keep

    def wait(self):
        self.work.wait()
        self.keep = None


# ---------------------------------------------------------------------------
# Feature slicing (module docstring, second strategy)
# ---------------------------------------------------------------------------
def _even_split(n: int, parts: int, align: int = 1) -> list[int]:
    """``parts`` sizes summing to n, as equal as possible in units of ``align``."""
    units, tail = divmod(n, align)
    base, rem = divmod(units, parts)
    sizes = [(base + (i < rem)) * align for i in range(parts)]
    sizes[-1] += tail
    return sizes


@dataclass
class FeaturePartition:
    """One rank's view of a feature-sliced graph.

    Node rows are relabelled into a *chunk-major* order pi: for chunk j of K,
    for rank q in order, rank q's j-th sub-range of its own rows.  Then the
    rows of one chunk are contiguous in every column-sliced buffer and, inside
    the chunk, grouped by owning rank -- each chunk's layout switch is one
    balanced all-to-all straight out of / into those buffers.  The CSR pair is
    built over pi-labels (sources and destinations), stable, so each row's
    edges keep their original order."""

    rank: int
    world: int
    num_nodes: int
    rows_per_rank: int
    row_begin: int
    row_end: int
    graph: SageGraph                  # full graph, pi-labelled, with transpose
    own_rowptr: torch.Tensor          # int32 [n_own+1]: in-degree prefix of own rows (natural order)
    chunk_rows: list[list[int]]       # [K][W]: rows of rank q in chunk j
    chunk_start: list[int]            # [K+1]: pi-row offset of chunk j
    chunk_edges: list[int]            # [K]: in-edges of chunk j's rows
    chunk_t_edges: list[int]          # [K]: out-edges of chunk j's rows
    own_chunk: list[int]              # [K+1]: own-row offsets of the chunks

    @property
    def num_rows(self) -> int:
        return self.row_end - self.row_begin

    @property
    def num_chunks(self) -> int:
        return len(self.chunk_rows)

    def col_sizes(self, feat: int) -> list[int]:
        """Column slice widths of a ``feat``-wide layer, one per rank (16-B
        multiples where F allows: whole vectors per lane in the gather)."""
        align = 8 if feat >= 8 * self.world else 1
        return _even_split(feat, self.world, align)

    def exchange_bytes_per_layer(self, feat: int, elem: int) -> int:
        """Bytes this rank sends per layer (fwd + bwd, 4 layout switches)."""
        cs = self.col_sizes(feat)
        own = self.num_rows
        return 4 * sum(own * cs[c] for c in range(self.world) if c != self.rank) * elem


def _chunk_bounds(n_own: int, chunks: int) -> list[int]:
    return [(j * n_own) // chunks for j in range(chunks + 1)]


def partition_features(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                       backend=HipBackend, chunks: int = 4) -> FeaturePartition:
    """Feature-sliced partition (no collective: every rank holds edge_index)."""
    P = (num_nodes + world - 1) // world
    dev = edge_index.device
    begins = [min(q * P, num_nodes) for q in range(world)]
    ends = [min((q + 1) * P, num_nodes) for q in range(world)]
    k = max(1, min(chunks, max(e - b for b, e in zip(begins, ends))))
    bounds = [_chunk_bounds(e - b, k) for b, e in zip(begins, ends)]
    chunk_rows = [[bounds[q][j + 1] - bounds[q][j] for q in range(world)] for j in range(k)]
    chunk_start = [0]
    for j in range(k):
        chunk_start.append(chunk_start[-1] + sum(chunk_rows[j]))
    # pi: natural id -> chunk-major id, built piecewise
    pi = torch.empty(num_nodes, dtype=torch.int64, device=dev)
    pos = 0
    for j in range(k):
        for q in range(world):
            a, b = begins[q] + bounds[q][j], begins[q] + bounds[q][j + 1]
            pi[a:b] = torch.arange(pos, pos + b - a, device=dev)
            pos += b - a
    ei = torch.stack([pi[edge_index[0].long()], pi[edge_index[1].long()]]) \
        if edge_index.numel() else edge_index.long()
    rp, col, trp, tcol = backend.csr(ei, max(num_nodes, 1), True)
    g = SageGraph(num_nodes, int(edge_index.size(1)), rp, col, trp, tcol)
    deg_rp = rp.long()
    t_rp = trp.long()
    chunk_edges = [int(deg_rp[chunk_start[j + 1]] - deg_rp[chunk_start[j]]) for j in range(k)]
    chunk_t_edges = [int(t_rp[chunk_start[j + 1]] - t_rp[chunk_start[j]]) for j in range(k)]
    r0, r1 = begins[rank], ends[rank]
    # own rows' in-degrees in natural order (1/deg of the bwd-data GEMM)
    own_pi = pi[r0:r1]
    own_deg = (deg_rp[own_pi + 1] - deg_rp[own_pi]).to(torch.int32)
    own_rowptr = torch.zeros(r1 - r0 + 1, dtype=torch.int32, device=dev)
    if r1 > r0:
        own_rowptr[1:] = torch.cumsum(own_deg, 0).to(torch.int32)
    return FeaturePartition(rank, world, num_nodes, P, r0, r1, g, own_rowptr, chunk_rows,
                            chunk_start, chunk_edges, chunk_t_edges, bounds[rank])


def _a2a(out, inp, out_splits, in_splits, group):
    return all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=True)


def _rows_to_cols(part: FeaturePartition, src: torch.Tensor, j: int, dst_cols: torch.Tensor,
                  group, backend):
    """Chunk j of this rank's rows of ``src`` [n_own, F] -> rows
    [chunk_start[j], chunk_start[j+1]) of the column-sliced ``dst_cols``
    [N, F_r] on every rank.  Returns (work, keep-alive)."""
    W, r = part.world, part.rank
    a, b = part.own_chunk[j], part.own_chunk[j + 1]
    cs = part.col_sizes(src.size(1))
    if W == 1:
        dst_cols[part.chunk_start[j]: part.chunk_start[j + 1]].copy_(src[a:b])
        return None, None
    rows = b - a
    if all(c == cs[0] for c in cs):
        send = backend.cols_pack(src[a:b], W, cs[0]) if rows else src.new_empty(0)
    else:
        send = torch.cat([src[a:b, sum(cs[:c]): sum(cs[:c + 1])].reshape(-1)
                          for c in range(W)]) if rows else src.new_empty(0)
    recv = dst_cols[part.chunk_start[j]: part.chunk_start[j + 1]]
    work = _a2a(recv.view(-1), send.view(-1), [n * cs[r] for n in part.chunk_rows[j]],
                [rows * c for c in cs], group)
    return work, send


def _cols_to_rows(part: FeaturePartition, src_cols: torch.Tensor, j: int, feat: int, group):
    """Rows [chunk_start[j], chunk_start[j+1]) of the column-sliced ``src_cols``
    -> this rank's chunk-j rows, all columns, as (work, recv, sizes); finish
    with :func:`_cols_to_rows_finish`."""
    W, r = part.world, part.rank
    cs = part.col_sizes(feat)
    s0, s1 = part.chunk_start[j], part.chunk_start[j + 1]
    rows = part.own_chunk[j + 1] - part.own_chunk[j]
    if W == 1:
        return None, src_cols[s0:s1], cs
    recv = src_cols.new_empty(rows * feat)
    work = _a2a(recv, src_cols[s0:s1].reshape(-1), [rows * c for c in cs],
                [n * cs[r] for n in part.chunk_rows[j]], group)
    return work, recv, cs


def _cols_to_rows_finish(part, recv, cs, rows, out_rows, backend, addend=None):
    """Interleave the per-rank column blocks of ``recv`` into ``out_rows``
    [rows, F] (+ ``addend`` rows, one rounding)."""
    if rows == 0:
        return
    if part.world == 1:
        if addend is None:
            out_rows.copy_(recv)
        else:
            torch.add(addend, recv, out=out_rows)
        return
    if all(c == cs[0] for c in cs):
        backend.cols_unpack(recv, rows, part.world, cs[0], out_rows, addend)
        return
    off, col = 0, 0
    for c in cs:
        piece = recv[off: off + rows * c].view(rows, c)
        if addend is None:
            out_rows[:, col:col + c].copy_(piece)
        else:
            torch.add(addend[:, col:col + c], piece, out=out_rows[:, col:col + c])
        off += rows * c
        col += c


def _feat_gather(backend, src_cols, rowptr, col, part, j, mean, out_cols, edges):
    s0, s1 = part.chunk_start[j], part.chunk_start[j + 1]
    if s1 > s0 and src_cols.size(1):
        backend.gather(src_cols, rowptr[s0: s1 + 1], col, s1 - s0, mean,
                       out=out_cols[s0:s1], edges=edges)


def _feat_aggregate_to_rows(backend, part, src_cols, rowptr, col, mean, feat, chunk_edges,
                            group, addend=None):
    """Aggregate all rows over this rank's columns, chunk by chunk, and bring
    each finished chunk back to row layout while the next chunk is gathered
    (+ ``addend`` rows: the backward's root-path gradient)."""
    out_cols = src_cols.new_empty(part.num_nodes, src_cols.size(1))
    out_rows = src_cols.new_empty(part.num_rows, feat)
    pending = []
    for j in range(part.num_chunks):
        _feat_gather(backend, src_cols, rowptr, col, part, j, mean, out_cols, chunk_edges[j])
        pending.append((j,) + _cols_to_rows(part, out_cols, j, feat, group))
    for j, work, recv, cs in pending:
        if work is not None:
            work.wait()
        a, b = part.own_chunk[j], part.own_chunk[j + 1]
        _cols_to_rows_finish(part, recv, cs, b - a, out_rows[a:b], backend,
                             addend[a:b] if addend is not None else None)
    return out_rows


def _feat_rows_to_cols(part, x_rows, group, backend):
    """Column-sliced copy [N, F_r] of the row-partitioned ``x_rows``; returns
    (buffer, works) -- wait on every work before reading the buffer."""
    cs = part.col_sizes(x_rows.size(1))
    buf = x_rows.new_empty(part.num_nodes, cs[part.rank])
    works = []
    for j in range(part.num_chunks):
        w, keep = _rows_to_cols(part, x_rows, j, buf, group, backend)
        if w is not None:
            works.append((w, keep))
    return buf, works


def _wait_all(works):
    for w, _ in works:
        w.wait()


class _FeatLayerFn(torch.autograd.Function):
    """One feature-sliced layer, pipelined per row chunk j:
    gather(j) || col->row(j-1) on the RCCL stream; then, as each chunk's
    aggregate arrives, dense + LayerNorm on its rows and (when a next layer
    follows) row->col(j) of its output, which runs while later chunks compute
    -- the next layer's column-sliced input is already in flight when this
    layer returns (handed over in ``carry``)."""

    @staticmethod
    def forward(ctx, x, wl, bl, wr, gamma, beta, part: FeaturePartition, group, backend,
                slope, drop_p, seed, eps, carry: dict):
        g = part.graph
        F = x.size(1)
        fo = wl.size(0)
        pre = carry.pop("cols", None)
        x_cols, works = pre if pre is not None else _feat_rows_to_cols(part, x, group,
                                                                        backend)
        _wait_all(works)
        out_cols = x_cols.new_empty(part.num_nodes, x_cols.size(1))
        pending = []
        for j in range(part.num_chunks):
            _feat_gather(backend, x_cols, g.rowptr, g.col, part, j, True, out_cols,
                         part.chunk_edges[j])
            pending.append(_cols_to_rows(part, out_cols, j, F, group))
        save = any(ctx.needs_input_grad[:6])
        n = part.num_rows
        agg = x.new_empty(n, F)
        out = x.new_empty(n, fo)
        xhat = x.new_empty(n, fo) if save else None
        rstd = x.new_empty(n, dtype=torch.float32) if save else None
        nxt = None
        if carry.get("next_layer"):
            cs = part.col_sizes(fo)
            nxt = (x.new_empty(part.num_nodes, cs[part.rank]), [])
        for j, (work, recv, cs_in) in enumerate(pending):
            a, b = part.own_chunk[j], part.own_chunk[j + 1]
            if work is not None:
                work.wait()
            _cols_to_rows_finish(part, recv, cs_in, b - a, agg[a:b], backend)
            if b > a:
                backend.layer_fwd(agg[a:b], x[a:b], wl, bl, wr, gamma, beta, eps, slope, drop_p,
                                  seed, save, part.row_begin + a,
                                  outs=(out[a:b], xhat[a:b] if save else None,
                                        rstd[a:b] if save else None))
            if nxt is not None:
                w, keep = _rows_to_cols(part, out, j, nxt[0], group, backend)
                if w is not None:
                    nxt[1].append((w, keep))
        del x_cols, out_cols, pending
        if nxt is not None:
            carry["cols"] = nxt
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
        gr = part.graph
        F = x.size(1)
        dh, dgamma, dbeta, dbl = be.post_bwd(dout.contiguous(), xhat, rstd, gamma, beta, slope,
                                             drop_p, seed, out, part.row_begin)
        cs = part.col_sizes(F)
        blocked = (part.world > 1 and all(c == cs[0] for c in cs)
                   and getattr(be, "bwd_data_blocked_ok", None) is not None
                   and be.bwd_data_blocked_ok(dh, F, cs[0]))
        if blocked:
            # the dX GEMM writes dAgg/deg chunk by chunk in the all-to-all's send
            # layout (no packing copy); each chunk's exchange starts behind its GEMM
            from .dense import weight_cat
            wcat_t = weight_cat(wl, wr, dh.dtype).t().contiguous()
            dx_r = dh.new_empty(part.num_rows, F)
            g_cols = dh.new_empty(part.num_nodes, cs[part.rank])
            works = []
            for j in range(part.num_chunks):
                a, b = part.own_chunk[j], part.own_chunk[j + 1]
                send = (be.bwd_data_blocked(dh[a:b], wcat_t, part.own_rowptr[a: b + 1], F, cs[0],
                                            dx_r[a:b]) if b > a else dh.new_empty(0))
                recv = g_cols[part.chunk_start[j]: part.chunk_start[j + 1]]
                w = _a2a(recv.view(-1), send, [n * cs[part.rank] for n in part.chunk_rows[j]],
                         [(b - a) * c for c in cs], group)
                if w is not None:                  # None: a staged (synchronous) exchange
                    works.append((w, send))
        else:
            g, dx_r = be.bwd_data(dh, wl, wr, part.own_rowptr)
            # dAgg/deg to column layout (RCCL stream) while the weight-grad GEMM runs
            g_cols, works = _feat_rows_to_cols(part, g, group, be)
        dwl, dwr = be.bwd_weight(dh, agg, x)
        grads = (dwl, dbl, dwr, dgamma, dbeta)
        flat = torch.cat([t.reshape(-1).float() for t in grads])
        rwork = None
        if part.world > 1:
            rwork = all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=True)
        _wait_all(works)
        # dx = dx_root + the gathered gradient, added as the blocks are unpacked
        dx = _feat_aggregate_to_rows(be, part, g_cols, gr.t_rowptr, gr.t_col, False, F,
                                     part.chunk_t_edges, group, addend=dx_r.contiguous())
        if rwork is not None:
            rwork.wait()
        dwl, dbl, dwr, dgamma, dbeta = (c.view_as(t) for c, t in zip(
            torch.split(flat, [t.numel() for t in grads]), grads))
        return (dx, dwl.to(wl.dtype), dbl.to(wl.dtype), dwr.to(wr.dtype), dgamma.to(gamma.dtype),
                dbeta.to(beta.dtype), None, None, None, None, None, None, None, None)


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
            rwork = all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=True)
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
                    broadcast(p.data, src=0, group=group)

    @property
    def strategy(self) -> str:
        if isinstance(self.part, ReplicaPartition):
            return "replicate"
        return "feature" if isinstance(self.part, FeaturePartition) else "halo"

    def forward(self, x_local: torch.Tensor) -> torch.Tensor:
        from .sageblock import _act_slope, _cpu_seed, _drop_p, _new_seed
        if isinstance(self.part, ReplicaPartition):
            # every rank runs the whole block: gradients are complete and
            # identical on every rank, nothing crosses xGMI
            return self.block(x_local, self.part.graph)
        feat = isinstance(self.part, FeaturePartition)
        x = x_local.contiguous()
        layers = list(zip(self.block.convs, self.block.posts))
        carry: dict = {}
        for i, (conv, post) in enumerate(layers):
            ln, act, drop = post[0], post[1], post[2]
            p = _drop_p(drop)
            # CPU tensors (the gloo / host-backend path) draw from torch's CPU
            # generator, as SageBlock's CPU mode does; the device generator
            # would need (and initialise) a GPU
            seed = 0 if p <= 0 else (_cpu_seed() if x.device.type == "cpu"
                                     else _new_seed(x.device))
            args = (x, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight, ln.weight, ln.bias,
                    self.part, self.group, self.backend, _act_slope(act), p, seed, float(ln.eps))
            if feat:
                carry["next_layer"] = i + 1 < len(layers)
                x = _FeatLayerFn.apply(*args, carry)
            else:
                x = _DistLayerFn.apply(*args)
        return x


# ---------------------------------------------------------------------------
# Strategy planner
# ---------------------------------------------------------------------------
# Cost-model constants (MI355X, measured on one GPU):
#   gather rate by gathered row width, uniform random rows of a multi-GB
#   table (tools/gather_probe.py, profiles/r1_gather_probe.txt);
#   xGMI: one link per peer, ~50 GB/s achieved per direction (conservative
#   share of the 76.8 GB/s per-direction link rate).
_GATHER_TBPS = ((64, 3.7e12), (128, 5.5e12), (256, 5.3e12), (512, 5.7e12), (1 << 30, 5.2e12))
_LINK_BPS = 50e9


def _gather_rate(row_bytes: int) -> float:
    for limit, rate in _GATHER_TBPS:
        if row_bytes <= limit:
            return rate
    return _GATHER_TBPS[-1][1]


def _remote_unique(ids: torch.Tensor, r0: int, r1: int) -> int:
    if ids.numel() == 0:
        return 0
    u = torch.unique(ids)
    return int(((u < r0) | (u >= r1)).sum())


# dense part (fwd GEMM + LN, LN backward, dX, dW) per layer and row, in units
# of F*s bytes at the stream kernels' measured rate (~13 F s per row)
_DENSE_BYTES_PER_ROW_FS = 13.0
_DENSE_BPS = 4.0e12
_FEAT_CHUNKS = 4          # partition_features' default pipeline depth
# A partition is chosen only when the model has it faster than one GPU doing
# all the work (replicate) by this factor: the xGMI and kernel rates above are
# estimates (~ +-20 %), and a strong-scaling run slower than one GPU is the
# outcome to rule out (C4 uniform at W = 4: feature 32.0 vs 34.8 ms per layer
# modelled -> replicate; at W = 8: 9.0 vs 34.8 -> feature).
_PARTITION_MARGIN = 1.2


def choose_strategy(info: dict) -> str:
    """The planner's pick from :func:`estimate_strategies`' modelled times."""
    best = min(("halo", "feature"), key=lambda k: info[f"{k}_s"])
    return best if info[f"{best}_s"] * _PARTITION_MARGIN < info["replicate_s"] else "replicate"


def measure_link_bps(device: torch.device, group=None, per_peer_bytes: int = 32 << 20,
                     reps: int = 3) -> float | None:
    """Achieved per-peer rate (bytes/s, one direction) of a balanced
    all_to_all over RCCL on this node: every rank sends ``per_peer_bytes`` to
    every peer at once (the feature-slicing switch pattern), timed after one
    warm-up call, max over ranks.  None when the group is not NCCL / RCCL or
    has one rank (the planner then keeps ``_LINK_BPS``)."""
    world = dist.get_world_size(group)
    if world < 2 or dist.get_backend(group) != "nccl" or device.type != "cuda":
        return None
    n = per_peer_bytes // 4
    inp = torch.empty(world * n, dtype=torch.float32, device=device).normal_()
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=group)          # warm-up (connections)
    torch.cuda.synchronize(device)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_to_all_single(out, inp, group=group)
    torch.cuda.synchronize(device)
    t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return per_peer_bytes / float(t)


def estimate_strategies(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                        feat: int, elem: int, group=None, link_bps: float | None = None,
                        balance: str = "cost") -> dict:
    """Modelled per-layer time (s) of the halo, feature-sliced and replicated
    strategies: exchange bytes / xGMI + gather bytes / measured gather rate +
    dense bytes / stream rate, max over ranks (collective over ``group`` when
    world > 1, so every rank gets the same numbers).  ``link_bps``: the
    per-peer xGMI rate to price exchanges at (:func:`measure_link_bps`;
    default ``_LINK_BPS``).  ``balance``: the row-block rule the halo strategy
    would be built with ("cost" or "rows"), so the model prices the blocks
    :func:`partition_graph` cuts."""
    hb_ = row_bounds(edge_index, num_nodes, world, balance)    # partition_graph's blocks
    h0, h1 = hb_[rank], hb_[rank + 1]
    src, dst = edge_index[0], edge_index[1]
    in_mask = (dst >= h0) & (dst < h1)
    out_mask = (src >= h0) & (src < h1)
    halo_f = _remote_unique(src[in_mask], h0, h1)
    halo_b = _remote_unique(dst[out_mask], h0, h1)
    e_in, e_out = int(in_mask.sum()), int(out_mask.sum())
    link = max(world - 1, 1) * (link_bps or _LINK_BPS)
    row = feat * elem
    halo_t = ((halo_f + halo_b) * row / link
              + (e_in + e_out) * (row + 4) / _gather_rate(row)
              + _DENSE_BYTES_PER_ROW_FS * (h1 - h0) * row / _DENSE_BPS)
    P = (num_nodes + world - 1) // world                       # partition_features' blocks
    r0, r1 = min(rank * P, num_nodes), min((rank + 1) * P, num_nodes)
    dense_own = _DENSE_BYTES_PER_ROW_FS * (r1 - r0) * row / _DENSE_BPS
    fc = max(1, feat // world)
    e = int(edge_index.size(1))
    # feature slicing pipelines its switches over `chunks` row chunks: the
    # exchange overlaps the gathers / dense of other chunks, one chunk's worth
    # of it stays exposed (the halo path overlaps only halo-free rows: additive)
    feat_comm = 4 * (world - 1) * (r1 - r0) * fc * elem / link
    # layout copies per layer (each reads and writes the rank's rows once): x
    # and dAgg/deg packed for their exchanges, agg unpacked, dx unpacked + added,
    # the dropout-free copy of the carried layer output; the bf16 F = 256 dX GEMM
    # writes dAgg/deg in send layout itself (dense.sage_linear_bwd_data_blocked)
    copies = 4 if (elem == 2 and feat == 256 and fc in (32, 64, 128)) else 5
    feat_comp = (2 * e * (fc * elem + 4) / _gather_rate(fc * elem) + dense_own
                 + copies * 2 * (r1 - r0) * row / _DENSE_BPS)
    feat_t = max(feat_comm, feat_comp) + feat_comm / _FEAT_CHUNKS
    rep_t = (2 * e * (row + 4) / _gather_rate(row)
             + _DENSE_BYTES_PER_ROW_FS * num_nodes * row / _DENSE_BPS)
    v = torch.tensor([halo_t, feat_t, rep_t, float(halo_f), float(halo_b)], dtype=torch.float64,
                     device=edge_index.device)
    if world > 1:
        all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    halo_t, feat_t, rep_t, hf, hb = v.tolist()
    return {"halo_s": halo_t, "feature_s": feat_t, "replicate_s": rep_t,
            "halo_rows_fwd_max": int(hf), "halo_rows_bwd_max": int(hb),
            "link_bps": float(link_bps or _LINK_BPS)}


@dataclass
class ReplicaPartition:
    """No sharding: every rank holds the whole graph and runs the whole block.
    Chosen by the planner when any partition is modelled slower than one GPU
    doing all the work (a random graph over a single xGMI link: W = 2)."""

    rank: int
    world: int
    num_nodes: int
    graph: SageGraph

    row_begin = 0

    @property
    def row_end(self) -> int:
        return self.num_nodes

    @property
    def num_rows(self) -> int:
        return self.num_nodes

    def exchange_bytes_per_layer(self, feat: int, elem: int) -> int:
        return 0


def partition_replicated(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                         backend=HipBackend) -> ReplicaPartition:
    if backend is HipBackend:
        from .graph import build_graph
        g = build_graph(edge_index, num_nodes)      # with the skew schedules (C5)
    else:
        rp, col, trp, tcol = backend.csr(edge_index, max(num_nodes, 1), True)
        g = SageGraph(num_nodes, int(edge_index.size(1)), rp, col, trp, tcol)
    return ReplicaPartition(rank, world, num_nodes, g)


def plan_partition(edge_index: torch.Tensor, num_nodes: int, world: int, rank: int,
                   feat: int, elem: int, strategy: str = "auto", backend=HipBackend,
                   group=None, chunks: int = 4, balance: str = "cost",
                   link_bps: float | None = None):
    """Partition with ``strategy`` in {"auto", "halo", "feature", "replicate"};
    "auto" takes :func:`choose_strategy` of :func:`estimate_strategies`
    (every rank gets the same answer: the estimate is max-reduced).  Returns
    (partition, info).  With "replicate" every rank runs the whole graph: the
    caller passes all rows of x (``partition.row_begin/row_end`` span them)."""
    info = {}
    if strategy == "auto":
        if world == 1:
            strategy = "halo"
        else:
            _trace("plan: estimate")
            info = estimate_strategies(edge_index, num_nodes, world, rank, feat, elem, group,
                                       link_bps, balance)
            _trace("plan: estimated")
            strategy = choose_strategy(info)
    info["strategy"] = strategy
    if strategy == "feature":
        return partition_features(edge_index, num_nodes, world, rank, backend, chunks), info
    if strategy == "replicate":
        return partition_replicated(edge_index, num_nodes, world, rank, backend), info
    if strategy == "halo":
        return partition_graph(edge_index, num_nodes, world, rank, backend, group,
                               balance), info
    raise ValueError(f"unknown partition strategy {strategy!r} "
                     "(auto, halo, feature, replicate)")
