"""PyG-free collate: Batch.from_data_list semantics for
the reference's graph records and the batch CSR emitted at collate time.

CPU: attribute concatenation / offsets / batch / ptr against an independent
per-node loop; the batch CSR bit-equal to the C oracle's CSR of the batched
edge_index (tests/_helpers.ref_csr).  GPU: ``GraphBatch.to('cuda')``
registers that CSR for the moved edge_index -- bit-equal to the GPU builder's
-- and a SageBlock over the batch uses it.
"""
from __future__ import annotations

import types

import numpy as np
import pytest
import torch

from _helpers import ref_csr


def _graph(n, e, T=4, L=3, seed=0, kind="dict"):
    g = torch.Generator().manual_seed(seed)
    d = dict(x=torch.randn(n, T, 6, generator=g),
             xsttype=torch.randint(0, 10, (n,), generator=g),
             xdims=torch.randn(n, 2, generator=g),
             edge_index=torch.randint(0, max(n, 1), (2, e), generator=g) if n else
             torch.empty(2, 0, dtype=torch.long),
             edge_attr=torch.randn(e, 4, generator=g),
             y=torch.randint(0, 2, (L,), generator=g).float(),
             pos_raw=torch.randn(n, T, 2, generator=g),
             pid=seed)
    if kind == "object":
        return types.SimpleNamespace(**d)
    return d


def test_collate_matches_pyg_batch_semantics():
    from sldm_sage.data import collate
    graphs = [_graph(5, 12, seed=1), _graph(0, 0, seed=2), _graph(7, 20, seed=3, kind="object"),
              _graph(1, 1, seed=4)]
    b = collate(graphs)
    items = [g if isinstance(g, dict) else vars(g) for g in graphs]
    assert b.num_graphs == 4
    assert torch.equal(b.ptr, torch.tensor([0, 5, 5, 12, 13]))
    # per-node loop: node v of graph i is batch row ptr[i] + v
    rows = []
    for i, d in enumerate(items):
        for v in range(d["x"].size(0)):
            rows.append((i, v))
    for r, (i, v) in enumerate(rows):
        assert int(b.batch[r]) == i
        for k in ("x", "xsttype", "xdims", "pos_raw"):
            assert torch.equal(b[k][r], items[i][k][v])
    # edges: concatenated in graph order, node ids offset by ptr[i]
    e = 0
    for i, d in enumerate(items):
        for j in range(d["edge_index"].size(1)):
            assert torch.equal(b.edge_index[:, e], d["edge_index"][:, j] + int(b.ptr[i]))
            assert torch.equal(b.edge_attr[e], d["edge_attr"][j])
            e += 1
    assert e == b.num_edges
    assert torch.equal(b.y.view(b.num_graphs, 3), torch.stack([d["y"] for d in items]))
    assert torch.equal(b.pid, torch.tensor([1, 2, 3, 4]))


def test_batch_csr_equals_csr_of_batched_edges():
    from sldm_sage.data import collate
    graphs = [_graph(n, e, seed=s) for s, (n, e) in enumerate([(30, 90), (1, 0), (200, 1500),
                                                               (17, 0), (64, 300)])]
    b = collate(graphs)
    n, e, rp, col, trp, tcol = b._csr
    assert n == b.num_nodes and e == b.num_edges
    ref = ref_csr(b.edge_index, n)
    for got, exp in zip((rp, col, trp, tcol), ref):
        assert np.array_equal(got, exp)


def test_graph_csr_cached_on_graph_and_loader():
    from sldm_sage.data import GraphLoader, collate
    graphs = [_graph(10, 25, seed=s, kind="object") for s in range(6)]
    collate(graphs[:2])
    assert hasattr(graphs[0], "_sldm_csr")
    batches = list(GraphLoader(graphs, batch_size=4, shuffle=False))
    assert [bb.num_graphs for bb in batches] == [4, 2]
    assert torch.equal(batches[1].ptr, torch.tensor([0, 10, 20]))


def test_bad_node_id_raises():
    from sldm_sage.data import collate
    g = _graph(4, 5, seed=9)
    g["edge_index"][0, 2] = 4
    with pytest.raises(IndexError):
        collate([g])


@pytest.mark.gpu
def test_collate_csr_registered_on_device_and_used():
    from sldm_sage import SageBlock, graph_cache, ops
    from sldm_sage.data import collate
    from sldm_sage.graph import get_graph
    graphs = [_graph(n, e, seed=s) for s, (n, e) in enumerate([(40, 200), (3, 0), (300, 2500)])]
    b = collate(graphs).to("cuda")
    N = b.num_nodes
    g = get_graph(b.edge_index, N)
    rp, col, trp, tcol, _ = ops.csr_build(b.edge_index, N, True)
    for got, exp in zip((g.rowptr, g.col, g.t_rowptr, g.t_col), (rp, col, trp, tcol)):
        assert torch.equal(got, exp)
    assert get_graph(b.edge_index, N) is g          # served from the cache
    torch.manual_seed(0)
    blk = SageBlock([6, 16, 16], None, 0.1).cuda()
    x = b.x[:, -1, :].contiguous()
    out_a = blk(x, b.edge_index)
    graph_cache.clear()
    out_b = blk(x, b.edge_index)                    # GPU-built CSR
    assert torch.equal(out_a, out_b)


def _device_graphs(spec, seed=0):
    """Graphs on the GPU with awkward edge lists: duplicates, self loops,
    unsorted ids, a star (one row of high degree), an edge_index that is a
    column slice of a wider buffer (row stride > E), empty graphs."""
    out = []
    g = torch.Generator().manual_seed(seed)
    for i, (n, e, kind) in enumerate(spec):
        if kind == "star":
            src = torch.randint(0, n, (e,), generator=g)
            ei = torch.stack([src, torch.zeros(e, dtype=torch.long)])
        else:
            ei = torch.randint(0, max(n, 1), (2, e), generator=g) if n else \
                torch.empty(2, 0, dtype=torch.long)
        ei = ei.cuda()
        if kind == "strided":
            wide = torch.full((2, e + 7), -5, dtype=torch.long, device="cuda")
            wide[:, :e] = ei
            ei = wide[:, :e]
        out.append({"x": torch.randn(n, 8, generator=g).cuda(), "edge_index": ei})
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [
    [(250, 6000, ""), (300, 9000, ""), (0, 0, ""), (1, 3, ""), (40, 0, ""), (220, 5000, "strided")],
    [(n, 8 * n, "") for n in range(1, 60)],                 # > 48 graphs: two launches
    [(2000, 3000, "star"), (5, 40, ""), (16384, 20000, "")],  # high degree, max nodes
    # LDS variants of batch.hip by the launch's largest graph: edge pairs staged
    # (above: <= ~9.9k edges at 250 nodes), edge ids only (here), global (above)
    [(3000, 12000, ""), (100, 500, "strided"), (7, 0, "")],
])
def test_device_collate_fused_batch_matches_pyg_and_csr_build(spec):
    """The fused GPU batching kernel (batch.hip): edge_index / batch / ptr as
    Batch.from_data_list, and the batch CSR pair bit-equal to sldm_csr_build on
    the batched edge_index (row order = original edge order)."""
    from sldm_sage import graph_cache, ops
    from sldm_sage.data import collate
    graphs = _device_graphs(spec)
    b = collate(graphs)
    counts = [d["x"].size(0) for d in graphs]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    want_ei = torch.cat([d["edge_index"] + offs[i] for i, d in enumerate(graphs)], 1)
    assert torch.equal(b.edge_index, want_ei)
    assert torch.equal(b.ptr.cpu(), torch.tensor(offs))
    assert torch.equal(b.batch.cpu(), torch.repeat_interleave(torch.arange(len(graphs)),
                                                              torch.tensor(counts)))
    assert torch.equal(b.x, torch.cat([d["x"] for d in graphs]))
    g = b.sage_graph()
    assert g is not None and graph_cache.get(b.edge_index, b.num_nodes, True) is g
    rp, col, trp, tcol, _ = ops.csr_build(b.edge_index, b.num_nodes, True)
    for got, exp in zip((g.rowptr, g.col, g.t_rowptr, g.t_col), (rp, col, trp, tcol)):
        assert torch.equal(got, exp)


@pytest.mark.gpu
def test_device_collate_bad_id_raises_and_sageblock_uses_fused_csr():
    from sldm_sage import SageBlock, graph_cache
    from sldm_sage.data import collate
    graphs = _device_graphs([(30, 100, ""), (20, 50, "")], seed=3)
    bad = [dict(graphs[0]), dict(graphs[1])]
    bad[1]["edge_index"] = bad[1]["edge_index"].clone()
    bad[1]["edge_index"][1, 7] = 20                  # == N_g: outside its own graph
    with pytest.raises(IndexError):
        collate(bad)
    b = collate(graphs)
    torch.manual_seed(0)
    blk = SageBlock([8, 16, 16], 0.25, 0.1).cuda().train()
    x = b.x.detach().requires_grad_(True)
    torch.manual_seed(5)
    out_a = blk(x, b.edge_index)
    out_a.sum().backward()
    ga = x.grad.clone()
    graph_cache.clear()                              # rebuild with sldm_csr_build
    x.grad = None
    torch.manual_seed(5)
    out_b = blk(x, b.edge_index)
    out_b.sum().backward()
    assert torch.equal(out_a, out_b) and torch.equal(ga, x.grad)
