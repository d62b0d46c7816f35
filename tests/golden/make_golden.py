"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Each .npz holds inputs (edge_index, x, upstream gradient gout, the SageBlock
state_dict as ``sd.<key>``, hdims, negative_slope) and the oracle's outputs
(out, dx, ``grad.<param>``), fp32, eval mode / dropout None.  The oracle is
oracle/sage_ref.py (plain-torch restatement of PyG 2.7.0 SAGEConv + the
reference SageBlock); parity is unpinned by reference outputs.
Seeds are fixed, so re-running reproduces the files bit for bit.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.sage_ref import RefSageBlock, random_graph, set_synthetic_params  # noqa: E402

CASES = {
    # name: (N, E, hdims, negative_slope, edge-set kind)
    "c1_16_16_16_leaky": (1000, 5000, [16, 16, 16], 0.1, "random"),
    "c1_16_32_32_relu": (1000, 5000, [16, 32, 32], None, "random"),
    "c1_16_16_16_relu": (1000, 5000, [16, 16, 16], None, "random"),
    "c1_16_32_32_leaky": (1000, 5000, [16, 32, 32], 0.1, "random"),
    "empty_graph": (64, 0, [16, 16, 16], 0.1, "random"),
    "isolated_dup_self": (200, 600, [16, 16, 16], 0.1, "dupself"),
    "hub_in_degree_10k": (2000, 12000, [16, 16], 0.1, "hub"),
}


def edges(kind: str, n: int, e: int):
    ei, x = random_graph(n, e, 1, seed=n + e)
    if kind == "dupself":
        ei[:, : e // 4] = ei[:, e // 4: e // 2]          # duplicate edges
        ei[1, e // 2: e // 2 + 50] = ei[0, e // 2: e // 2 + 50]   # self loops
        ei = ei[:, (ei[1] % 7) != 3]                      # leave nodes isolated
    elif kind == "hub":
        ei[1, :10_000] = 17                               # one node with in-degree 10k
    return ei


def main() -> None:
    for name, (n, e, hdims, ns, kind) in CASES.items():
        ei = edges(kind, n, e)
        gen = torch.Generator().manual_seed(7)
        x = torch.randn(n, hdims[0], generator=gen)
        gout = torch.randn(n, hdims[-1], generator=gen)
        ref = RefSageBlock(hdims, dropout=None, negative_slope=ns)
        set_synthetic_params(ref, seed=1)
        xr = x.clone().requires_grad_(True)
        out = ref(xr, ei)
        out.backward(gout)
        arrs = dict(edge_index=ei.numpy(), x=x.numpy(), gout=gout.numpy(),
                    out=out.detach().numpy(), dx=xr.grad.numpy(),
                    hdims=np.array(hdims, np.int64), has_slope=np.array(ns is not None),
                    negative_slope=np.array(ns if ns is not None else 0.0, np.float32))
        for k, v in ref.state_dict().items():
            arrs["sd." + k] = v.numpy()
        for k, p in ref.named_parameters():
            arrs["grad." + k] = p.grad.numpy()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrs)
        print(f"{path}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
