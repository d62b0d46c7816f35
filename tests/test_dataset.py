"""PyG-free ``.pt`` ingest (sldm_sage.dataset) on CPU.

torch_geometric is not installed here, so the pickles are
written with stand-in classes registered under PyG's module paths, shaped
like PyG 2.x's ``Data`` / ``GlobalStorage`` pickle state (a ``_store``
storage holding the attribute ``_mapping`` and a back-reference to its
parent, plus the ``DataEdgeAttr`` / ``DataTensorAttr`` class references
``Data.__init__`` keeps); the stand-ins are removed from ``sys.modules``
before loading, exactly as on a box without PyG.  Parity with PyG's own
pickles is therefore unpinned (no PyG-written fixture exists in the
reference or here).
"""
from __future__ import annotations

import json
import sys
import types
import weakref

import pytest
import torch


def _install_fake_pyg():
    """Stand-ins for torch_geometric.data.{data,storage} (PyG 2.x pickle shape)."""
    root = types.ModuleType("torch_geometric")
    data_pkg = types.ModuleType("torch_geometric.data")
    data_mod = types.ModuleType("torch_geometric.data.data")
    storage_mod = types.ModuleType("torch_geometric.data.storage")

    class GlobalStorage:
        def __init__(self, _parent=None):
            self.__dict__["_mapping"] = {}
            self.__dict__["_parent"] = weakref.ref(_parent) if _parent is not None else None

        def __getstate__(self):
            out = self.__dict__.copy()
            if out.get("_parent") is not None:
                out["_parent"] = out["_parent"]()
            return out

        def __setstate__(self, mapping):
            self.__dict__.update(mapping)

    class DataEdgeAttr:
        pass

    class DataTensorAttr:
        pass

    class Data:
        def __init__(self, **kwargs):
            self.__dict__["_store"] = GlobalStorage(_parent=self)
            self.__dict__["_edge_attr_cls"] = DataEdgeAttr
            self.__dict__["_tensor_attr_cls"] = DataTensorAttr
            self._store._mapping.update(kwargs)

        def __getstate__(self):
            return self.__dict__.copy()

    for cls, mod in ((GlobalStorage, storage_mod), (DataEdgeAttr, data_mod),
                     (DataTensorAttr, data_mod), (Data, data_mod)):
        cls.__module__ = mod.__name__
        cls.__qualname__ = cls.__name__
        setattr(mod, cls.__name__, cls)
    mods = {"torch_geometric": root, "torch_geometric.data": data_pkg,
            "torch_geometric.data.data": data_mod, "torch_geometric.data.storage": storage_mod}
    sys.modules.update(mods)
    return Data, list(mods)


def _pack(n, e, T, seed):
    """A pack like gbuilder.py:115-131 emits (x [n, T, 6] with presence last).
    Pack 3 holds NaN / inf in some absent frames: the statistics must ignore
    them, as the reference's boolean indexing does (dataset.py:127-131)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, T, 6, generator=g)
    x[:, :, -1] = (torch.rand(n, T, generator=g) > 0.3).float()
    if seed == 3:
        absent = x[:, :, -1] < 0.5
        assert bool(absent.any())
        junk = torch.tensor([float("nan"), float("inf")])[torch.arange(int(absent.sum())) % 2]
        x[:, :, 0][absent] = junk
    return dict(x=x, xsttype=torch.randint(0, 256, (n,), generator=g),
                xdims=torch.rand(n, 2, generator=g) * 4,
                edge_index=torch.randint(0, n, (2, e), generator=g),
                edge_attr=torch.randn(e, 4, generator=g), y=torch.rand(5, generator=g))


@pytest.fixture
def pack_dir(tmp_path):
    Data, names = _install_fake_pyg()
    try:
        packs = [_pack(7 + i, 12 + 3 * i, 10, i) for i in range(4)]
        for i, p in enumerate(packs):
            torch.save(Data(**p), tmp_path / f"pack_{i}.pt")
        # a pickle naming an unrelated global must still be refused
        torch.save({"fn": json.dumps}, tmp_path / "evil.bin")
    finally:
        for k in names:
            sys.modules.pop(k, None)
    with open(tmp_path / "metadata.json", "w") as fh:
        json.dump(dict(n_samples=4, n_positive=1, n_edge_features=4, frames_num=10, m_radius=30.0,
                       active_labels=[0, 1, 2, 3, 4]), fh)
    return tmp_path, packs


def test_load_pack_without_pyg(pack_dir):
    from sldm_sage.dataset import PackGraph, load_pack
    d, packs = pack_dir
    assert "torch_geometric" not in sys.modules
    g = load_pack(d / "pack_2.pt")
    assert isinstance(g, PackGraph)
    assert sorted(g.keys()) == sorted(packs[2])
    for k, v in packs[2].items():
        assert torch.equal(getattr(g, k), v), k
    assert g.num_nodes == 9 and g.num_edges == 18
    with pytest.raises(Exception):
        load_pack(d / "evil.bin")


def test_pack_dataset_matches_mapgraph_semantics(pack_dir):
    """PackDataset.innerGet / computeMuSigma restate dataset.py:75-89 and
    :107-149 (per-vehicle loop over present frames, fp32 sums)."""
    from sldm_sage.dataset import PackDataset
    d, packs = pack_dir
    ds = PackDataset(d)
    assert len(ds) == 4 and ds.frames_num == 10
    # computeMuSigma, the reference's loop (dataset.py:121-147) written out
    nf = 5
    sx = torch.zeros(1, 1, nf)
    sx2 = torch.zeros(1, 1, nf)
    sd = torch.zeros(1, 2)
    sd2 = torch.zeros(1, 2)
    cnt = vcnt = 0
    for p in packs:
        for vi in range(p["x"].size(0)):
            gv = p["x"][vi:vi + 1]
            pm = gv[0, :, -1] > 0.5
            gv = gv[:, pm, :-1]
            sx += gv.sum(dim=1, keepdim=True)
            sx2 += (gv ** 2).sum(dim=1, keepdim=True)
            cnt += int(pm.sum())
        sd += p["xdims"].sum(0, keepdim=True)
        sd2 += (p["xdims"] ** 2).sum(0, keepdim=True)
        vcnt += p["xdims"].size(0)
    mu_x = sx / cnt
    sig_x = ((sx2 / cnt) - mu_x ** 2).sqrt().clamp(min=1e-8)
    mu_d = sd / vcnt
    sig_d = ((sd2 / vcnt) - mu_d ** 2).sqrt()
    tol = dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ds.mu["x"], mu_x, **tol)
    torch.testing.assert_close(ds.sigma["x"], sig_x, **tol)
    torch.testing.assert_close(ds.mu["xdims"], mu_d, **tol)
    torch.testing.assert_close(ds.sigma["xdims"], sig_d, **tol)
    g = ds[1]
    raw = packs[1]["x"]
    assert torch.equal(g.pos_raw, raw[:, :, :2])
    torch.testing.assert_close(g.x[:, :, :-1], (raw[:, :, :-1] - ds.mu["x"]) / ds.sigma["x"])
    assert torch.equal(g.x[:, :, -1], raw[:, :, -1])                  # presence untouched
    with ds.usingRawData:
        assert torch.equal(ds[1].x, raw)


def test_ingest_feeds_collate(pack_dir):
    """Loaded packs batch with sldm_sage.data.collate (PyG Batch semantics +
    the batch CSR), the path main.py:158-167 takes."""
    from sldm_sage.data import collate, host_csr
    from sldm_sage.dataset import PackDataset
    d, packs = pack_dir
    ds = PackDataset(d, normalizeZScore=False)
    b = collate([ds[i] for i in range(4)])
    assert b.num_graphs == 4 and b.num_nodes == sum(p["x"].size(0) for p in packs)
    offs = torch.tensor([0] + [p["x"].size(0) for p in packs]).cumsum(0)
    want = torch.cat([p["edge_index"] + offs[i] for i, p in enumerate(packs)], 1)
    assert torch.equal(b.edge_index, want)
    n, e, rp, col, trp, tcol = b._csr
    ref = host_csr(want, n)
    for a, r in zip((rp, col, trp, tcol), ref):
        assert (a == r).all()


def test_collate_csr_cache_follows_edge_index():
    """The per-graph host CSR is keyed on the edge_index tensor and
    its version, so an in-place rewire with the same edge count is seen."""
    from sldm_sage.data import collate, host_csr
    from sldm_sage.dataset import PackGraph
    p = PackGraph(**_pack(6, 10, 4, 3))
    collate([p])
    p.edge_index[0, 0] = (p.edge_index[0, 0] + 1) % 6         # in place, same E
    b = collate([p])
    ref = host_csr(p.edge_index, 6)
    assert all((a == r).all() for a, r in zip(b._csr[2:], ref))
    p.edge_index = p.edge_index.flip(1).contiguous()             # replaced, same E
    b = collate([p])
    ref = host_csr(p.edge_index, 6)
    assert all((a == r).all() for a, r in zip(b._csr[2:], ref))
