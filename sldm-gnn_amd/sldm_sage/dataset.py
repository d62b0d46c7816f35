"""PyG-free ingest of the reference's ``pack_*.pt`` graphs.

The reference loads each pack with ``torch.load(path, map_location=device)``
under ``safe_globals([DataEdgeAttr, DataTensorAttr, GlobalStorage])``
(/root/reference/src/dataset.py:64-89), which needs torch_geometric to
rebuild the pickled ``torch_geometric.data.Data``.  Here the same files load
without PyG: ``torch.load(..., weights_only=True)`` -- torch's restricted
unpickler, which executes nothing from the file -- with the four PyG class
paths such a pickle names mapped to inert local records
(:class:`PackGraph` for ``Data``, a plain storage for ``GlobalStorage``,
markers for the two attr classes).  Every other global still raises.  The
result is a :class:`PackGraph` with PyG ``Data`` attribute access
(``g.x``, ``g.edge_index``, ``g.num_nodes``, ``g.to(device)``) that
:func:`sldm_sage.data.collate` batches directly.

:class:`PackDataset` mirrors ``MapGraph`` (dataset.py:13-149): same
constructor arguments, ``len`` / ``get`` / ``__getitem__``, the z-score of
``x[..., :-1]`` and ``xdims`` with ``pos_raw`` saved first (innerGet,
dataset.py:75-89), ``computeMuSigma`` (dataset.py:107-149, over present
frames only) and the ``usingRawData`` context.
"""
from __future__ import annotations

import contextlib
import json
from pathlib import Path

import torch

_PYG_DATA = "torch_geometric.data.data.Data"
_PYG_STORAGE = "torch_geometric.data.storage.GlobalStorage"
_PYG_EDGE_ATTR = "torch_geometric.data.data.DataEdgeAttr"
_PYG_TENSOR_ATTR = "torch_geometric.data.data.DataTensorAttr"


class PackGraph:
    """A graph record with PyG ``Data`` attribute access (module docstring)."""

    def __init__(self, **fields):
        self.__dict__.update(fields)

    # restricted-unpickler hook: the pickled Data's state is its __dict__,
    # whose '_store' is a GlobalStorage holding the attribute mapping
    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:      # (dict, slots)
            state = {**(state[0] or {}), **(state[1] or {})}
        store = state.get("_store") if isinstance(state, dict) else None
        mapping = getattr(store, "_mapping", None) if store is not None else None
        if mapping is None and isinstance(state, dict):
            mapping = {k: v for k, v in state.items() if not k.startswith("_")}
        self.__dict__.update(dict(mapping or {}))

    def to_dict(self) -> dict:
        return {k: v for k, v in self.__dict__.items() if not k.startswith("_")}

    def keys(self) -> list[str]:
        return list(self.to_dict())

    def __getitem__(self, key):
        return self.__dict__[key]

    def __setitem__(self, key, value):
        self.__dict__[key] = value

    def __contains__(self, key) -> bool:
        return key in self.__dict__

    @property
    def num_nodes(self) -> int:
        for k in ("x", "pos_raw", "xsttype", "xdims"):
            v = self.__dict__.get(k)
            if isinstance(v, torch.Tensor) and v.dim() > 0:
                return int(v.size(0))
        ei = self.__dict__.get("edge_index")
        return int(ei.max()) + 1 if isinstance(ei, torch.Tensor) and ei.numel() else 0

    @property
    def num_edges(self) -> int:
        ei = self.__dict__.get("edge_index")
        return int(ei.size(1)) if isinstance(ei, torch.Tensor) else 0

    def to(self, device, non_blocking: bool = False) -> "PackGraph":
        return PackGraph(**{k: (v.to(device, non_blocking=non_blocking)
                                if isinstance(v, torch.Tensor) else v)
                            for k, v in self.to_dict().items()})

    def clone(self) -> "PackGraph":
        return PackGraph(**{k: (v.clone() if isinstance(v, torch.Tensor) else v)
                            for k, v in self.to_dict().items()})

    def __repr__(self) -> str:
        parts = [f"{k}={list(v.shape) if isinstance(v, torch.Tensor) else v!r}"
                 for k, v in self.to_dict().items()]
        return f"PackGraph({', '.join(parts)})"


class _Storage:
    """Stand-in for ``GlobalStorage``: keeps its state (``_mapping`` etc.)."""

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:
            state = {**(state[0] or {}), **(state[1] or {})}
        self.__dict__.update(state if isinstance(state, dict) else {})


class _EdgeAttrMarker:
    """Stand-in for the ``DataEdgeAttr`` class reference a Data pickle holds."""


class _TensorAttrMarker:
    """Stand-in for the ``DataTensorAttr`` class reference a Data pickle holds."""


_SAFE = [(PackGraph, _PYG_DATA), (_Storage, _PYG_STORAGE), (_EdgeAttrMarker, _PYG_EDGE_ATTR),
         (_TensorAttrMarker, _PYG_TENSOR_ATTR)]


def load_pack(path, device="cpu") -> PackGraph:
    """One ``pack_*.pt`` (a pickled PyG ``Data``) as a :class:`PackGraph`,
    without torch_geometric (dataset.py:77: ``torch.load(..., map_location=
    device)``).  Only torch's weights-only unpickler runs; a file naming any
    global outside tensors and the four PyG paths raises."""
    with torch.serialization.safe_globals(_SAFE):
        obj = torch.load(path, map_location=device, weights_only=True)
    if isinstance(obj, PackGraph):
        return obj
    if isinstance(obj, dict):
        return PackGraph(**obj)
    raise TypeError(f"{path}: expected a pickled torch_geometric Data, got {type(obj).__name__}")


def _meta_get(metadata, key):
    return metadata[key] if isinstance(metadata, dict) else getattr(metadata, key)


class PackDataset(torch.utils.data.Dataset):
    """``MapGraph`` (dataset.py:13-149) without torch_geometric."""

    def __init__(self, graphs_dirpath, *, device: str = "cpu", transform=None,
                 normalizeZScore: bool = True, metadata=None, zscore_mu_sigma=None):
        graphs_dirpath = Path(graphs_dirpath)
        if metadata is None:
            with open(graphs_dirpath / "metadata.json", encoding="utf-8") as fh:
                metadata = json.load(fh)
        self.frames_num = _meta_get(metadata, "frames_num")
        labels = _meta_get(metadata, "active_labels")
        self.active_labels = set(labels) if labels is not None else None
        # MetaData.n_node_temporal_features (utils.py:130-132): 3 + 1 + 2
        self.n_temp_feats = (getattr(metadata, "n_node_temporal_features", None)
                             if not isinstance(metadata, dict) else None) or 6
        self.transform = transform
        self.dirpath = graphs_dirpath.resolve()
        self.paths = list(sorted(self.dirpath.glob("*.pt")))
        self.device = device
        self.normalizeZScore = normalizeZScore
        self.mu = self.sigma = None
        if normalizeZScore:
            if zscore_mu_sigma is not None:
                self.mu, self.sigma = zscore_mu_sigma
            else:
                self.mu, self.sigma = self.computeMuSigma()

    def getMuSigma(self):
        if self.mu is None or self.sigma is None:
            self.mu, self.sigma = self.computeMuSigma()
        return self.mu, self.sigma

    def len(self) -> int:
        return len(self.paths)

    def __len__(self) -> int:
        return self.len()

    def get(self, idx: int) -> PackGraph:
        return self.innerGet(idx)

    def __getitem__(self, idx: int) -> PackGraph:
        return self.innerGet(idx)

    def getRawByPid(self, pid: int) -> PackGraph:
        fname = (self.dirpath / f"pack_{pid}.pt").resolve()
        if not fname.exists():
            raise FileNotFoundError(f"Graph file for pack id {pid} not found at path: {fname}")
        return load_pack(fname, self.device)

    def innerGet(self, idx: int) -> PackGraph:
        """dataset.py:75-89: load, transform, then z-score with pos_raw saved."""
        graph = load_pack(self.paths[idx], self.device)
        if self.transform:
            graph = self.transform(graph)
        if self.normalizeZScore:
            graph.pos_raw = graph.x[:, :, :2].clone()
            graph.x[:, :, :-1] = (graph.x[:, :, :-1] - self.mu["x"]) / self.sigma["x"]
            graph.xdims = (graph.xdims - self.mu["xdims"]) / self.sigma["xdims"]
        return graph

    @property
    def usingRawData(self):
        """Context that disables normalisation and transforms (dataset.py:91-105)."""
        @contextlib.contextmanager
        def ctx():
            prev = (self.normalizeZScore, self.transform)
            self.normalizeZScore, self.transform = False, None
            try:
                yield
            finally:
                self.normalizeZScore, self.transform = prev
        return ctx()

    def computeMuSigma(self):
        """dataset.py:107-149: mean / std of x[..., :-1] over present frames
        (presence = last feature > 0.5) and of xdims over vehicles, fp32
        sums; sigma_x clamped at 1e-8."""
        nfeats = self.n_temp_feats - 1
        sum_x = torch.zeros((1, 1, nfeats), device=self.device, dtype=torch.float)
        sum_x2 = torch.zeros_like(sum_x)
        sum_xd = torch.zeros((1, 2), device=self.device)
        sum_xd2 = torch.zeros_like(sum_xd)
        tot_cnt = 0
        vcnt = 0
        with self.usingRawData:
            for i in range(self.len()):
                g = self.innerGet(i)
                pres = g.x[:, :, -1] > 0.5                       # [V, T]
                # absent frames are dropped, whatever they hold (the reference
                # indexes them away, dataset.py:127-131: a NaN / inf there must
                # not reach the sums)
                feats = torch.where(pres[:, :, None], g.x[:, :, :-1],
                                    torch.zeros((), dtype=g.x.dtype, device=g.x.device))
                sum_x += feats.sum(dim=(0, 1), keepdim=True)
                sum_x2 += (feats ** 2).sum(dim=(0, 1), keepdim=True)
                tot_cnt += int(pres.sum())
                sum_xd += g.xdims.sum(dim=0, keepdim=True)
                sum_xd2 += (g.xdims ** 2).sum(dim=0, keepdim=True)
                vcnt += g.xdims.size(0)
        mu_xd = sum_xd / vcnt
        sigma_xd = ((sum_xd2 / vcnt) - mu_xd ** 2).sqrt()
        mu_x = sum_x / tot_cnt
        sigma_x = ((sum_x2 / tot_cnt) - mu_x ** 2).sqrt().clamp(min=1e-8)
        return {"x": mu_x, "xdims": mu_xd}, {"x": sigma_x, "xdims": sigma_xd}
