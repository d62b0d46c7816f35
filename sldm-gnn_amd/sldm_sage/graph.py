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
class SageGraph:
    """CSR of one graph on one device (int32)."""

    num_nodes: int
    num_edges: int
    rowptr: torch.Tensor            # [N+1] by destination
    col: torch.Tensor               # [E]   sources, original edge order per row
    t_rowptr: torch.Tensor | None   # [N+1] by source (backward)
    t_col: torch.Tensor | None      # [E]   destinations
    order: torch.Tensor | None = None     # longest-first schedule of rowptr rows (skewed graphs)
    t_order: torch.Tensor | None = None   # same for t_rowptr

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def in_degree(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]


def build_graph(edge_index: torch.Tensor, num_nodes: int, transpose: bool = True,
                validate: bool = True) -> SageGraph:
    """Build the CSR pair on edge_index's device.

    ``validate`` reads back the device-side range flag (one host sync) and
    raises IndexError on a node id outside [0, num_nodes) — the reference
    raises too (PyG index_select / scatter bounds checks).
    """
    rowptr, col, t_rowptr, t_col, bad = ops.csr_build(edge_index, num_nodes, transpose)
    if validate and edge_index.size(1) > 0 and int(bad.item()) != 0:
        raise IndexError(
            f"edge_index holds a node id outside [0, {num_nodes}) "
            "(the reference's index_select/scatter would raise as well)")
    g = SageGraph(num_nodes, int(edge_index.size(1)), rowptr, col, t_rowptr, t_col)
    g.order = _schedule(rowptr, g.num_edges)
    if t_rowptr is not None:
        g.t_order = _schedule(t_rowptr, g.num_edges)
    return g


def _schedule(rowptr: torch.Tensor, num_edges: int):
    """Longest-first row order when the degree distribution is skewed
    (max > max(64, 8 x mean)), e.g. power-law in-degrees; None otherwise."""
    n = rowptr.numel() - 1
    if n <= 0 or num_edges == 0 or os.environ.get("SLDM_NO_SCHEDULE") == "1":
        return None
    max_deg = int((rowptr[1:] - rowptr[:-1]).max().item())
    if max_deg <= max(64, 8 * num_edges / n):
        return None
    return ops.degree_order(rowptr)


class _GraphCache:
    def __init__(self, max_entries: int = 64):
        self._lock = threading.RLock()  # weakref callbacks may fire under the lock
        self._entries: dict[int, tuple] = {}
        self._max = max_entries

    def _drop(self, key: int) -> None:
        with self._lock:
            self._entries.pop(key, None)

    def get(self, edge_index: torch.Tensor, num_nodes: int, transpose: bool) -> SageGraph:
        if edge_index.is_inference():
            # Inference tensors carry no version counter: an in-place edit
            # would go unseen, so they are never cached (rcv.py builds a new
            # graph per pack anyway).
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
        if edge_index.is_inference() or graph.device != edge_index.device:
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
