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
