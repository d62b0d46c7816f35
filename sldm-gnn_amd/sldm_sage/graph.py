"""Graph ingest: edge_index [2,E] -> CSR by destination (+ transpose), cached.

The reference hands SageBlock a raw COO ``edge_index`` every call
(sageblock.py:16-18; produced by src/gbuilder.py:85-112 and batched by PyG
collate, main.py:166) and PyG re-derives its addressing per SAGEConv call.
Here the CSR is built once per graph on the GPU (``ops.csr_build``) and cached
against the *tensor object*: a weak reference plus its ``_version`` counter,
so the static lane-map graph (mapencoder.py:12, a registered buffer) pays
once, a per-batch graph pays once per batch, an in-place edit invalidates the
entry, and nothing outlives the edge_index tensor it describes.
"""
from __future__ import annotations

import os
import threading
import weakref
from dataclasses import dataclass

import torch

from . import ops


@dataclass
class HubPlan:
    """High-degree rows of one CSR, split into fixed-length edge chunks for
    ``sldm_gather_rows_split`` (include/sldm_sage.h): rows with degree >
    ``max_deg`` are summed chunk by chunk by separate row groups (fp32
    partials, combined in chunk order) instead of serially by one."""

    hub_rows: torch.Tensor          # int32 [H]
    chunk_ptr: torch.Tensor         # int32 [H+1]: chunks of hub h
    chunk_row: torch.Tensor         # int32 [C]
    chunk_beg: torch.Tensor         # int32 [C]: first CSR position of chunk c
    num_hubs: int
    num_chunks: int
    chunk_len: int
    max_deg: int


@dataclass
class SageGraph:
    """CSR of one graph on one device (int32)."""

    num_nodes: int
    num_edges: int
    rowptr: torch.Tensor            # [N+1] by destination
    col: torch.Tensor               # [E]   sources, original edge order per row
    t_rowptr: torch.Tensor | None   # [N+1] by source (backward)
    t_col: torch.Tensor | None      # [E]   destinations
    hub: HubPlan | None = None            # high-degree split of rowptr rows (skewed graphs)
    t_hub: HubPlan | None = None          # same for t_rowptr
    _packed: tuple | None = None
    bad: torch.Tensor | None = None       # device range flag of a build that could not read it

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def packed(self) -> tuple[list, list]:
        """The graph as the ``(Tensor[12], int[9])`` pair the ``torch.ops.sldm``
        operators take: [rowptr, col, t_rowptr, t_col, then the hub plan of
        the rows and of the transpose rows (hub_rows, chunk_ptr, chunk_row,
        chunk_beg each)] -- absent entries have 0 elements -- and
        [has_transpose, num_hubs, num_chunks, chunk_len, max_deg, and the
        same four for the transpose].  Built once per graph."""
        if self._packed is None:
            none = self.rowptr.new_empty(0)
            ts = [self.rowptr, self.col,
                  self.t_rowptr if self.t_rowptr is not None else none,
                  self.t_col if self.t_col is not None else none]
            meta = [int(self.t_rowptr is not None)]
            for h in (self.hub, self.t_hub):
                if h is None:
                    ts += [none] * 4
                    meta += [0, 0, 1, 0]
                else:
                    ts += [h.hub_rows, h.chunk_ptr, h.chunk_row, h.chunk_beg]
                    meta += [h.num_hubs, h.num_chunks, h.chunk_len, h.max_deg]
            self._packed = (ts, meta)
        return self._packed

    def in_degree(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]

    def check(self) -> None:
        """Raise IndexError if the build found a node id out of range: for
        graphs built under HIP graph capture, whose build leaves the flag on
        the device (call after a replay has finished; one host sync)."""
        if self.bad is not None and int(self.bad) != 0:
            raise IndexError(f"edge_index holds a node id outside [0, {self.num_nodes})")


# Skew handling (power-law graphs).  Graphs below HUB_MIN_EDGES are
# launch-bound (per-batch vehicle graphs: ~10^4 edges) and skip it -- and its
# host sync -- entirely.  SLDM_SKEW: "split" (default: hub rows split into
# chunks) or "none".
HUB_MIN_EDGES = int(os.environ.get("SLDM_HUB_MIN_EDGES", str(1 << 20)))
# Largest edge count whose CSR build may be recorded into a HIP graph: above
# it the radix sort inside sldm_csr_build clears its histograms with memset
# nodes (rocPRIM's one-sweep path), which a captured graph must not hold.
CAPTURE_MAX_EDGES = 1 << 20
HUB_CHUNK = 256          # edges per hub chunk (one row group sums one chunk)


def _skew_mode() -> str:
    return os.environ.get("SLDM_SKEW", "split")


def hub_threshold(num_nodes: int, num_edges: int) -> int:
    """Rows with more in-edges than this are hubs: max(1024, 32 x mean degree)."""
    return max(1024, int(32 * num_edges / max(num_nodes, 1)))


def build_graph(edge_index: torch.Tensor, num_nodes: int, transpose: bool = True,
                validate: bool = True) -> SageGraph:
    """Build the CSR pair on edge_index's device.

    ``validate`` reads back the device-side range flag and raises IndexError
    on a node id outside [0, num_nodes) -- the reference raises too (PyG
    index_select / scatter bounds checks).  That read is the build's only
    host sync for graphs below HUB_MIN_EDGES; larger graphs read their
    maximum degrees in the same sync (and a skewed one a second time, for
    the hub plan's size).  While the current stream is capturing a HIP graph
    nothing can be read back: the build (up to CAPTURE_MAX_EDGES edges) is
    recorded with the range flag left on the device (``SageGraph.bad``,
    ``SageGraph.check()``).  An edge whose two ends both equal ``num_nodes``
    is padding and is ignored (fixed-shape edge_index buffers).
    """
    E = int(edge_index.size(1))
    if edge_index.device.type == "cpu":
        # the reference's CPU mode (main.py:58): host kernels (cpu.py), which
        # validate the ids as they count
        from . import cpu
        rowptr, col, t_rowptr, t_col = cpu.csr_build(edge_index, num_nodes, transpose)
        return SageGraph(num_nodes, E, rowptr, col, t_rowptr, t_col)
    if torch.cuda.is_current_stream_capturing():
        # recorded into a HIP graph (a per-batch edge_index buffer refilled
        # between replays): no host read is possible, so the range flag stays
        # on the device (SageGraph.check; the kernels clamp a bad id to node 0)
        # and rows are never split -- per-batch graphs are far below that size
        if E > CAPTURE_MAX_EDGES:
            raise RuntimeError(
                f"a graph of {E} edges cannot be built under HIP graph capture (limit "
                f"{CAPTURE_MAX_EDGES}): build it before the capture (sldm_sage.build_graph) "
                "and pass the SageGraph")
        rowptr, col, t_rowptr, t_col, bad = ops.csr_build(edge_index, num_nodes, transpose)
        return SageGraph(num_nodes, E, rowptr, col, t_rowptr, t_col, bad=bad)
    rowptr, col, t_rowptr, t_col, bad = ops.csr_build(edge_index, num_nodes, transpose)
    g = SageGraph(num_nodes, E, rowptr, col, t_rowptr, t_col)
    mode = _skew_mode()
    skew_check = E >= HUB_MIN_EDGES and num_nodes > 0 and mode != "none"
    if not (validate and E > 0) and not skew_check:
        return g
    stats = [bad.to(torch.int64).view(1)]
    if skew_check:
        stats.append((rowptr[1:] - rowptr[:-1]).max().to(torch.int64).view(1))
        if t_rowptr is not None:
            stats.append((t_rowptr[1:] - t_rowptr[:-1]).max().to(torch.int64).view(1))
    vals = torch.cat(stats).tolist()                    # the one host sync
    if validate and E > 0 and vals[0] != 0:
        raise IndexError(
            f"edge_index holds a node id outside [0, {num_nodes}) "
            "(the reference's index_select/scatter would raise as well)")
    if skew_check:
        thr = hub_threshold(num_nodes, E)
        if vals[1] > thr:
            g.hub = hub_plan(rowptr, thr)
        if t_rowptr is not None and vals[2] > thr:
            g.t_hub = hub_plan(t_rowptr, thr)
    return g


def hub_plan(rowptr: torch.Tensor, max_deg: int, chunk_len: int = HUB_CHUNK,
             row_mask: torch.Tensor | None = None) -> HubPlan | None:
    """Chunk table of the rows with degree > max_deg (None if there are none).
    ``row_mask`` (bool [N]): only the hubs among these rows (a row subset's
    plan; the launch still skips every row above max_deg)."""
    deg = (rowptr[1:] - rowptr[:-1]).long()
    is_hub = deg > max_deg
    if row_mask is not None:
        is_hub &= row_mask
    hubs = is_hub.nonzero().squeeze(1)
    nch = (deg[hubs] + chunk_len - 1) // chunk_len
    ptr = torch.zeros(hubs.numel() + 1, dtype=torch.int64, device=rowptr.device)
    torch.cumsum(nch, 0, out=ptr[1:])
    total = int(ptr[-1])                                # sync (hubs only)
    if hubs.numel() == 0:
        return None
    chunk_row = torch.repeat_interleave(hubs, nch, output_size=total)
    local = (torch.arange(total, device=rowptr.device)
             - torch.repeat_interleave(ptr[:-1], nch, output_size=total))
    chunk_beg = rowptr.long()[chunk_row] + local * chunk_len
    i32 = torch.int32
    return HubPlan(hubs.to(i32), ptr.to(i32), chunk_row.to(i32), chunk_beg.to(i32),
                   int(hubs.numel()), total, chunk_len, max_deg)


class _GraphCache:
    def __init__(self, max_entries: int = 64):
        self._lock = threading.RLock()  # weakref callbacks may fire under the lock
        self._entries: dict[int, tuple] = {}
        self._max = max_entries

    def _drop(self, key: int) -> None:
        with self._lock:
            self._entries.pop(key, None)

    def get(self, edge_index: torch.Tensor, num_nodes: int, transpose: bool) -> SageGraph:
        if edge_index.is_inference() or (edge_index.device.type == "cuda"
                                         and torch.cuda.is_current_stream_capturing()):
            # Inference tensors carry no version counter: an in-place edit
            # would go unseen, so they are never cached (rcv.py builds a new
            # graph per pack anyway).  A build recorded into a HIP graph has
            # not run yet: its arrays hold nothing until a replay, so no
            # eager call may find it in the cache.
            return build_graph(edge_index, num_nodes, transpose=transpose)
        key = id(edge_index)
        ver = edge_index._version
        with self._lock:
            ent = self._entries.get(key)
        if ent is not None:
            ref, e_ver, e_n, graph = ent
            if ref() is edge_index and e_ver == ver and e_n == num_nodes and (
                    graph.t_rowptr is not None or not transpose):
                return graph
        graph = build_graph(edge_index, num_nodes, transpose=transpose)
        try:
            ref = weakref.ref(edge_index, lambda _r, k=key: self._drop(k))
        except TypeError:  # not weak-referenceable: do not cache
            return graph
        with self._lock:
            if len(self._entries) >= self._max:
                self._entries.pop(next(iter(self._entries)))
            self._entries[key] = (ref, ver, num_nodes, graph)
        return graph

    def put(self, edge_index: torch.Tensor, num_nodes: int, graph: SageGraph) -> None:
        """Register a CSR built elsewhere (e.g. at collate time) for this
        edge_index tensor, so the next SageBlock call skips the GPU build."""
        if edge_index.is_inference() or graph.device != edge_index.device or (
                edge_index.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            return
        key = id(edge_index)
        try:
            ref = weakref.ref(edge_index, lambda _r, k=key: self._drop(k))
        except TypeError:
            return
        with self._lock:
            if len(self._entries) >= self._max and key not in self._entries:
                self._entries.pop(next(iter(self._entries)))
            self._entries[key] = (ref, edge_index._version, num_nodes, graph)

    def clear(self) -> None:
        with self._lock:
            self._entries.clear()

    def __len__(self) -> int:
        return len(self._entries)


graph_cache = _GraphCache()


def get_graph(edge_index: torch.Tensor, num_nodes: int, transpose: bool = True) -> SageGraph:
    if isinstance(edge_index, SageGraph):
        return edge_index
    return graph_cache.get(edge_index, num_nodes, transpose)
