"""PyG-free batching of the reference's graphs, emitting the SageBlock CSR at
collate time.

Replaces ``torch_geometric.loader.DataLoader`` / ``Batch.from_data_list``
as used by the reference (main.py:3, :166-167; test.py:9; utils.py:2, :218,
:249) for the graphs ``src/gbuilder.py`` emits (gbuilder.py:85-131: ``x``
[n, T, 6], ``xsttype`` [n], ``xdims`` [n, 2], ``edge_index`` [2, e],
``edge_attr`` [e, 4], ``y`` [L]; ``pos_raw`` [n, T, 2] added by
dataset.py:85):

* tensors are concatenated along dim 0, ``edge_index`` (any key containing
  "index") along dim -1 and offset by the running node count -- PyG's
  ``__cat_dim__`` / ``__inc__`` defaults; 0-dim tensors are stacked; numbers
  become a tensor, anything else a list;
* ``batch`` [N] (graph id per node), ``ptr`` [B+1] and ``num_graphs`` as in
  PyG, so ``batch.y.view(batch.num_graphs, L)`` (utils.py:222) works;
* for graphs on the host, each graph's CSR pair (by destination, and by
  source for the backward) is built once on the host (stable counting order = the GPU builder's order,
  bit for bit) and cached on the graph object; the batch's CSR is the
  concatenation of its graphs' CSRs with offsets -- equal to building it from
  the batched edge_index -- and ``GraphBatch.to(device)`` registers it for
  the moved ``edge_index`` in the SageBlock's graph cache, so the per-batch
  GPU CSR build vanishes.
"""
from __future__ import annotations

import weakref
from collections.abc import Mapping

import numpy as np
import torch

from .graph import SageGraph, graph_cache

_CSR_ATTR = "_sldm_csr"


def _items(data) -> dict:
    if isinstance(data, Mapping):
        return dict(data)
    if hasattr(data, "to_dict"):            # PyG Data
        return dict(data.to_dict())
    return {k: v for k, v in vars(data).items() if not k.startswith("_")}


def _num_nodes(d: dict) -> int:
    if d.get("num_nodes") is not None:
        return int(d["num_nodes"])
    for k in ("x", "pos_raw", "xsttype", "xdims"):
        v = d.get(k)
        if isinstance(v, torch.Tensor) and v.dim() > 0:
            return int(v.size(0))
    ei = d.get("edge_index")
    if isinstance(ei, torch.Tensor) and ei.numel():
        return int(ei.max()) + 1
    return 0


def host_csr(edge_index: torch.Tensor, num_nodes: int):
    """(rowptr, col, t_rowptr, t_col) int32 numpy: CSR by destination with
    sources in original edge order, and by source with destinations in
    original order -- the order ``sldm_csr_build`` produces."""
    ei = edge_index.detach().cpu().numpy().astype(np.int64, copy=False)
    src, dst = ei[0], ei[1]
    if ei.shape[1] and (min(src.min(), dst.min()) < 0 or max(src.max(), dst.max()) >= num_nodes):
        raise IndexError(f"edge_index holds a node id outside [0, {num_nodes})")

    def by(key, val):
        order = np.argsort(key, kind="stable")
        ptr = np.zeros(num_nodes + 1, np.int32)
        np.cumsum(np.bincount(key, minlength=num_nodes), out=ptr[1:])
        return ptr, val[order].astype(np.int32)

    rp, col = by(dst, src)
    trp, tcol = by(src, dst)
    return rp, col, trp, tcol


def graph_csr(data, edge_index: torch.Tensor, num_nodes: int):
    """The graph's host CSR pair, cached on the graph object when possible.

    The entry is keyed on the edge_index tensor itself -- a weak reference
    plus its ``_version`` counter, as the SageBlock's graph cache does -- so a
    replaced edge_index, or one edited in place (augmentation, rewiring),
    is rebuilt even when its edge count is unchanged."""
    cached = getattr(data, _CSR_ATTR, None) if not isinstance(data, Mapping) else \
        data.get(_CSR_ATTR)
    versioned = not edge_index.is_inference()
    if (cached is not None and versioned and cached[0] == num_nodes
            and cached[1]() is edge_index and cached[2] == edge_index._version):
        return cached[3]
    csr = host_csr(edge_index, num_nodes)
    if not versioned:           # inference tensors carry no version counter
        return csr
    try:
        ref = weakref.ref(edge_index)
    except TypeError:
        return csr
    entry = (num_nodes, ref, edge_index._version, csr)
    try:
        if isinstance(data, Mapping):
            data[_CSR_ATTR] = entry
        else:
            object.__setattr__(data, _CSR_ATTR, entry)
    except (AttributeError, TypeError):
        pass
    return csr


class GraphBatch:
    """A batch of graphs with PyG ``Batch`` attribute access (``batch.x``,
    ``batch.edge_index``, ``batch.batch``, ``batch.ptr``, ``batch.num_graphs``,
    ``batch.to(device)``), plus the batch CSR."""

    def __init__(self, store: dict, num_graphs: int, csr=None, graph: SageGraph | None = None):
        object.__setattr__(self, "_store", store)
        object.__setattr__(self, "num_graphs", num_graphs)
        object.__setattr__(self, "_csr", csr)   # host (N, E, rowptr, col, t_rowptr, t_col)
        object.__setattr__(self, "_graph", graph)   # device SageGraph (GPU batching path)

    def __getattr__(self, key):
        try:
            return self._store[key]
        except KeyError:
            raise AttributeError(key) from None

    def __setattr__(self, key, value):
        self._store[key] = value

    def __getitem__(self, key):
        return self._store[key]

    def __contains__(self, key):
        return key in self._store

    def keys(self):
        return list(self._store.keys())

    @property
    def num_nodes(self) -> int:
        return int(self._store["ptr"][-1])

    @property
    def num_edges(self) -> int:
        ei = self._store.get("edge_index")
        return int(ei.size(1)) if isinstance(ei, torch.Tensor) else 0

    def sage_graph(self, device=None) -> SageGraph | None:
        """The batch CSR as a :class:`SageGraph` on ``device`` (default: where
        ``edge_index`` lives)."""
        dev = torch.device(device) if device is not None else self._store["edge_index"].device
        if self._graph is not None and self._graph.device == dev:
            return self._graph
        if self._csr is None:
            return None
        n, e, rp, col, trp, tcol = self._csr
        t = [torch.as_tensor(a).to(dev) for a in (rp, col, trp, tcol)]
        return SageGraph(n, e, t[0], t[1], t[2], t[3])

    def to(self, device, non_blocking: bool = False) -> "GraphBatch":
        store = {k: (v.to(device, non_blocking=non_blocking) if isinstance(v, torch.Tensor) else v)
                 for k, v in self._store.items()}
        ei = store.get("edge_index")
        g = self._graph if (self._graph is not None and isinstance(ei, torch.Tensor)
                            and ei.device == self._graph.device) else None
        out = GraphBatch(store, self.num_graphs, self._csr, g)
        if g is not None:
            graph_cache.put(ei, g.num_nodes, g)
            return out
        if self._csr is not None and isinstance(ei, torch.Tensor) and ei.device.type == "cuda":
            graph_cache.put(ei, self._csr[0], out.sage_graph(ei.device))
        return out

    def __repr__(self) -> str:
        parts = [f"{k}={list(v.shape) if isinstance(v, torch.Tensor) else type(v).__name__}"
                 for k, v in self._store.items()]
        return f"GraphBatch(num_graphs={self.num_graphs}, {', '.join(parts)})"


def _device_batch(items, counts):
    """The fused GPU batching path (ops.batch_graphs) when every graph's
    edge_index is an int64 [2, E] tensor on one GPU and no graph exceeds the
    kernel's node limit; None otherwise (host path below)."""
    eis = [d.get("edge_index") for d in items]
    if not eis or not all(isinstance(e, torch.Tensor) for e in eis):
        return None
    dev = eis[0].device
    if dev.type != "cuda" or any(
            e.device != dev or e.dtype != torch.int64 or e.dim() != 2 or e.size(0) != 2
            or (e.size(1) > 1 and e.stride(1) != 1) for e in eis):
        return None
    from . import _lib, ops
    if max(counts) > _lib.load().sldm_batch_graphs_max_nodes():
        return None
    ei, batch, ptr, rowptr, col, t_rowptr, t_col, bad = ops.batch_graphs(eis, counts)
    if int(bad.item()):                       # the batch's one host sync
        raise IndexError("edge_index holds a node id outside its graph's [0, num_nodes) "
                         "(the reference's index_select/scatter would raise as well)")
    graph = SageGraph(int(sum(counts)), int(ei.size(1)), rowptr, col, t_rowptr, t_col)
    return ei, batch, ptr, graph


def collate(data_list) -> GraphBatch:
    """``Batch.from_data_list`` semantics (module docstring) + the batch CSR."""
    items = [_items(d) for d in data_list]
    if not items:
        raise ValueError("collate: empty data list")
    keys = [k for k in items[0] if k != _CSR_ATTR and k != "num_nodes"]
    counts = [_num_nodes(d) for d in items]
    offs = np.zeros(len(items) + 1, np.int64)
    np.cumsum(counts, out=offs[1:])
    store: dict = {}
    fused = _device_batch(items, counts)
    if fused is not None:
        # graphs on the GPU: edge_index + batch + ptr + the batch CSR pair in
        # one kernel (ops.batch_graphs), registered for the SageBlock
        store["edge_index"], store["batch"], store["ptr"] = fused[:3]
        keys = [k for k in keys if k != "edge_index"]
    for k in keys:
        vals = [d[k] for d in items]
        v0 = vals[0]
        if isinstance(v0, torch.Tensor):
            if "index" in k:
                vals = [v + int(offs[i]) for i, v in enumerate(vals)]
                store[k] = torch.cat(vals, dim=-1)
            elif v0.dim() == 0:
                store[k] = torch.stack(vals)
            else:
                store[k] = torch.cat(vals, dim=0)
        elif isinstance(v0, (int, float, bool)) and not isinstance(v0, np.generic):
            store[k] = torch.tensor(vals)
        else:
            store[k] = vals
    N = int(offs[-1])
    if fused is not None:
        graph_cache.put(store["edge_index"], N, fused[3])
        return GraphBatch(store, len(items), None, fused[3])
    dev = next((v.device for v in store.values() if isinstance(v, torch.Tensor)),
               torch.device("cpu"))
    store["batch"] = torch.repeat_interleave(
        torch.arange(len(items), device=dev), torch.tensor(counts, device=dev),
        output_size=N)
    store["ptr"] = torch.as_tensor(offs, device=dev)
    csr = None
    # The batch CSR is assembled on the host from per-graph host CSRs when the
    # graphs live on the host (the DataLoader-worker case).  Graphs on the GPU
    # (dataset.py:77 loads with map_location=DEVICE) took the fused path above;
    # the rest (e.g. int32 ids) leave the CSR to the SageBlock's GPU build.
    if "edge_index" in items[0] and all(
            getattr(d.get("edge_index"), "device", torch.device("cpu")).type == "cpu"
            for d in items):
        parts = [graph_csr(data_list[i], items[i]["edge_index"], counts[i])
                 for i in range(len(items))]
        e_offs = np.zeros(len(items) + 1, np.int64)
        np.cumsum([p[1].size for p in parts], out=e_offs[1:])
        rp = np.concatenate([p[0][:-1] + e_offs[i] for i, p in enumerate(parts)] +
                            [np.array([e_offs[-1]])]).astype(np.int32)
        trp = np.concatenate([p[2][:-1] + e_offs[i] for i, p in enumerate(parts)] +
                             [np.array([e_offs[-1]])]).astype(np.int32)
        col = np.concatenate([p[1] + offs[i] for i, p in enumerate(parts)]).astype(np.int32)
        tcol = np.concatenate([p[3] + offs[i] for i, p in enumerate(parts)]).astype(np.int32)
        csr = (N, int(e_offs[-1]), rp, col, trp, tcol)
    return GraphBatch(store, len(items), csr)


class GraphLoader(torch.utils.data.DataLoader):
    """``torch_geometric.loader.DataLoader(dataset, batch_size, shuffle)``
    (main.py:166-167) without PyG: batches with :func:`collate`."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, **kwargs):
        kwargs.pop("collate_fn", None)
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle, collate_fn=collate,
                         **kwargs)
