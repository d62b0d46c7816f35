"""End-to-end drop-in plumbing on CPU: the REFERENCE's own ``GruSage`` and
``train_model`` (/root/reference/src/models/grusage.py, src/utils.py) run with
this framework substituted at the PyG entry points --

  * ``src/models/blocks/sageblock.py``  -> the drop-in file
    (sldm-gnn_amd/dropin/..., placed ahead of the reference on ``sys.path``;
    the reference's ``src`` is a namespace package, so the overlay wins);
  * ``torch_geometric.nn.global_mean_pool / global_max_pool`` -> sldm_sage.pool;
  * ``torch_geometric.loader.DataLoader`` -> sldm_sage.data.GraphLoader;
  * ``MapGraph`` -> sldm_sage.dataset.PackDataset over pack_*.pt files written
    the way the reference's builder pickles them;

and nothing else changed: the vehicle SageBlock (grusage.py:109, :182), the
lane-map SageBlock inside MapEncoder (mapencoder.py:20-25, :37), the readout
(:185), ``train_model``'s batch loop (utils.py:218-233), ``saveSnapshot`` /
``state_dict_no_mapenc`` (utils.py:22-30, grusage.py:141), ``loadSnapshot`` +
strict ``load_state_dict`` (test.py:121-122) and ``grads()`` (grusage.py:194).

The reference tree exists only in the build container (it never travels to
the GPU box), so the module is skipped elsewhere; everything runs on CPU
tensors -- the reference's ``DEVICE = 'cpu'`` mode (main.py:58) -- through the
same dispatcher operators (torch.ops.sldm.sage_layer) as on the GPU.
torch_geometric and colorama are not installed here: the stand-in modules
below only carry the names the reference imports.
"""
from __future__ import annotations

import copy
import json
import os
import sys
import types

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DROPIN = os.path.join(ROOT, "sldm-gnn_amd", "dropin")

pytestmark = pytest.mark.skipif(
    not os.path.isfile(os.path.join(REF, "src", "models", "grusage.py")),
    reason="the reference tree exists only in the build container")

T, LABELS = 10, [0, 1]


@pytest.fixture
def ref(tmp_path):
    """Import the reference's model / training modules over the stand-ins;
    yields (GruSage, utils module, data dir); undone afterwards."""
    import sldm_sage
    from sldm_sage.data import GraphLoader
    from test_dataset import _install_fake_pyg, _pack

    saved_path = list(sys.path)
    added = []

    def module(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        added.append(name)
        return m

    class _NoColor:
        def __getattr__(self, _):
            return ""

    # the pack files, pickled with PyG-shaped stand-in classes (test_dataset.py)
    Data, names = _install_fake_pyg()
    try:
        gdir = tmp_path / ".graphs"
        gdir.mkdir()
        for i in range(6):
            p = _pack(6 + i, 14 + 2 * i, T, 20 + i)
            p["y"] = (torch.rand(len(LABELS), generator=torch.Generator().manual_seed(i)) > 0.5
                      ).float()
            torch.save(Data(**p), gdir / f"pack_{i}.pt")
    finally:
        for k in names:
            sys.modules.pop(k, None)
    with open(gdir / "metadata.json", "w") as fh:
        json.dump(dict(n_samples=6, n_positive=3, n_edge_features=4, frames_num=T,
                       m_radius=30.0, active_labels=LABELS), fh)

    tg = module("torch_geometric")
    tg.__path__ = []
    module("torch_geometric.nn", global_mean_pool=sldm_sage.global_mean_pool,
           global_max_pool=sldm_sage.global_max_pool, SAGEConv=sldm_sage.SageConv)
    module("torch_geometric.loader", DataLoader=GraphLoader)
    module("colorama", Fore=_NoColor(), Style=_NoColor(), Back=_NoColor())
    sys.path[:0] = [DROPIN, REF]
    try:
        import src.models.grusage as grusage
        import src.utils as utils
        import src.models.blocks.sageblock as blk_mod
        assert blk_mod.__file__.startswith(DROPIN), "the drop-in file must shadow the reference's"
        assert blk_mod.SageBlock is sldm_sage.SageBlock
        yield grusage.GruSage, utils, gdir
    finally:
        sys.path[:] = saved_path
        for k in [k for k in sys.modules if k == "src" or k.startswith("src.")] + added:
            sys.modules.pop(k, None)


def _map_tensors(seed=0, segs=12):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, segs, (30,), generator=g)
    dst = torch.randint(0, segs, (30,), generator=g)
    return dict(float_features=torch.randn(segs, 6, generator=g),
                bool_features=torch.rand(segs, 2, generator=g) > 0.5,
                lane_type_cats=torch.randint(0, 3, (segs,), generator=g),
                mgraph_edge_indexes=torch.stack([src, dst]),          # directed lane graph
                mseg_centroids=torch.randn(segs, 2, generator=g) * 3)


def _model(GruSage, dropout):
    torch.manual_seed(0)
    return GruSage(dynamic_features_num=6, frames_num=T, gru_hidden_size=16, gru_num_layers=1,
                   fc1dims=[24], sage_hidden_dims=[16, 16], fc2dims=[8], out_dim=len(LABELS),
                   num_st_types=256, emb_dim=4, dropout=dropout, negative_slope=0.1,
                   global_pooling="double", map_included=True, map_tensors=_map_tensors(),
                   mapenc_sage_hdims=[8, 8], mapenc_lane_embdim=2, map_attention_topk=3)


def test_grusage_step_matches_oracle_blocks(ref):
    """One train_model-style step (forward, BCE loss, backward; utils.py:219-225)
    of the reference's GruSage: with the drop-in SageBlock / pool / loader /
    dataset every parameter gradient equals that of the same model built on
    the oracle's SageBlock and pools (oracle/sage_ref.py, oracle/pool_ref.py)."""
    from oracle import pool_ref as R
    from oracle.sage_ref import RefSageBlock
    from sldm_sage.data import GraphLoader
    from sldm_sage.dataset import PackDataset
    GruSage, utils, gdir = ref
    ds = PackDataset(gdir, device="cpu", normalizeZScore=True)
    batch = next(iter(GraphLoader(ds, batch_size=4, shuffle=False)))
    assert batch.num_graphs == 4 and hasattr(batch, "pos_raw")

    model = _model(GruSage, dropout=None).train()
    twin = copy.deepcopy(model)

    def oracle_block(block):
        hd = [block.convs[0].in_channels] + [c.out_channels for c in block.convs]
        o = RefSageBlock(hd, None, 0.1)
        o.load_state_dict(block.state_dict())          # same keys, strict
        return o

    twin.sage = oracle_block(model.sage)
    twin.map_encoder.sage = oracle_block(model.map_encoder.sage)
    twin.global_pool = lambda x, b: torch.cat([R.global_mean_pool(x, b),
                                               R.global_max_pool(x, b)], dim=1)
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor(1.0))
    outs = []
    for m in (model, twin):
        logits = m(batch)
        y = batch.y.float().view(batch.num_graphs, len(LABELS))
        loss = crit(logits, y)
        loss.backward()
        outs.append((logits.detach(), loss.item()))
    torch.testing.assert_close(outs[0][0], outs[1][0], atol=1e-5, rtol=1e-5)
    got, want = dict(model.named_parameters()), dict(twin.named_parameters())
    assert set(got) == set(want)
    sage_keys = [k for k in got if k.startswith("sage.") or k.startswith("map_encoder.sage.")]
    assert len(sage_keys) == 2 * 2 * 5                      # 2 blocks x 2 layers x 5 tensors
    for k in got:
        assert got[k].grad is not None, k
        torch.testing.assert_close(got[k].grad, want[k].grad, atol=1e-5, rtol=1e-4,
                                   msg=lambda m, k=k: f"{k}: {m}")
    # grads() walks named_parameters of self.sage (grusage.py:204)
    tot, per = model.grads()
    tot_t, per_t = twin.grads()
    assert per["GraphSAGE Layers"] is not None
    assert abs(per["GraphSAGE Layers"] - per_t["GraphSAGE Layers"]) < 1e-5 * max(1.0, tot_t)


def test_train_model_runs_and_snapshot_round_trips(ref, tmp_path):
    """The reference's train_model (utils.py:176-308), one epoch, dropout 0.25:
    runs unchanged on the drop-ins, steps the SageBlock parameters, writes the
    best-validation snapshot (state_dict_no_mapenc + ip_dict), and the snapshot
    rebuilds the model the way test.py:121-122 does (strict load_state_dict)."""
    from sldm_sage.data import GraphLoader
    from sldm_sage.dataset import PackDataset
    GruSage, utils, gdir = ref
    ds = PackDataset(gdir, device="cpu", normalizeZScore=True)
    dl = GraphLoader(ds, batch_size=3, shuffle=True)
    model = _model(GruSage, dropout=0.25)
    before = {k: v.clone() for k, v in model.state_dict().items()}
    snap_path = tmp_path / "best_state.pth"
    (tr, _), (va, tot_va), _ = utils.train_model(
        model, dl, dl, epochs=1, lr=1e-2, device="cpu", active_labels=LABELS,
        neg_over_pos_ratio=1.0, best_state_path=snap_path, quiet=True)
    assert tr.shape == (len(LABELS), 1) and 0.0 <= float(tot_va[0, 0]) <= 1.0
    after = model.state_dict()
    moved = [k for k in before if k.startswith(("sage.", "map_encoder.sage."))
             and not torch.equal(before[k], after[k])]
    assert len(moved) == 20, moved                          # every SageBlock tensor stepped
    assert all(torch.isfinite(v).all() for v in after.values())
    if float(tot_va[0, 0]) > 0:                             # snapshot written on improvement
        snap = utils.loadSnapshot(snap_path)
        assert not any(k.startswith("map_encoder") for k in snap["state_dict"])
        assert any(k.startswith("sage.convs.0.lin_l") for k in snap["state_dict"])
        again = GruSage(**snap["ip_dict"])                  # map embeddings precomputed
        again.load_state_dict(snap["state_dict"])           # strict
        batch = next(iter(GraphLoader(ds, batch_size=6, shuffle=False)))
        model.eval(), again.eval()
        with torch.inference_mode():
            torch.testing.assert_close(again(batch), model(batch), atol=1e-5, rtol=1e-5)
