"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the reference's radius-edge construction,
/root/reference/src/gbuilder.py:85-111 (offline) and :241-268
(GraphOnlineCreator): for each ordered pair (i, j), i != j, the per-frame XY
distance as ``np.linalg.norm(xi - xj, axis=1)`` over torch float32 rows,
restricted to the frames where both presence flags exceed 0.5; an edge
(i, j) when any remain and their min <= radius, with
``[d.min(), d.max(), d.mean(), (d ** 2).mean()]`` as its attributes.  The
same numpy / torch float32 calls as the reference, so its bits.

Who may import this module: ``tests/`` only.  PARITY UNPINNED (the
reference ships no fixtures) -- this runs the reference's own
numpy operations on the test inputs.
"""
from __future__ import annotations

import numpy as np
import torch


def radius_edges(x: torch.Tensor, m_radius: float):
    """x: [V, T, 5] float32 CPU tensor ([X, Y, Speed, Angle, PresenceFlag])."""
    edge_index_list, edge_attr_list = [], []
    num_vehicles = x.shape[0]
    for i in range(num_vehicles):
        xi, pi = x[i, :, :2], x[i, :, 4]
        for j in range(num_vehicles):
            if i == j:
                continue
            xj, pj = x[j, :, :2], x[j, :, 4]
            dists = np.linalg.norm(xi - xj, axis=1)
            presence_mask = (pi > 0.5) & (pj > 0.5)
            dists = dists[presence_mask]
            if dists.size != 0 and dists.min() <= m_radius:
                edge_index_list.append([i, j])
                edge_attr_list.append([dists.min(), dists.max(), dists.mean(),
                                       (dists ** 2).mean()])
    ei = (torch.tensor(edge_index_list, dtype=torch.long).t().contiguous()
          if edge_index_list else torch.empty((2, 0), dtype=torch.long))
    ea = (torch.tensor(np.array(edge_attr_list, dtype=np.float32))
          if edge_attr_list else torch.empty((0, 4), dtype=torch.float))
    return ei, ea
