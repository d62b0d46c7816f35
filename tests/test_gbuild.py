"""Radius-edge construction: the GPU kernel against
the reference's numpy pair loop (oracle/gbuild_ref.py), bit for bit: same
edges in the same order, same float32 edge attributes.

Packs have T >= 2 frames: with T = 1 the reference indexes a numpy array with
a 1-element torch bool mask, which numpy reads as an integer index (mask
False keeps the frame, True raises IndexError); the kernel applies the mask.
"""
from __future__ import annotations

import pytest
import torch

from oracle.gbuild_ref import radius_edges as ref_radius_edges


def _pack(v, t, seed, grid=False, p_present=0.8):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(v, t, 5)
    if grid:   # integer positions: exact distances, some exactly at the radius
        x[:, :, :2] = torch.randint(-6, 7, (v, t, 2), generator=g).float()
    else:
        x[:, :, :2] = torch.randn(v, t, 2, generator=g) * 30
    x[:, :, 2:4] = torch.randn(v, t, 2, generator=g)
    x[:, :, 4] = (torch.rand(v, t, generator=g) < p_present).float()
    if v > 3:
        x[1, :, 4] = 0.0        # a vehicle never present
    return x


def test_oracle_known_answer():
    x = torch.zeros(3, 2, 5)
    x[1, :, 0] = torch.tensor([3.0, 10.0])
    x[1, :, 1] = torch.tensor([4.0, 0.0])
    x[2, :, 0] = 100.0
    x[:, :, 4] = 1.0
    x[0, 1, 4] = 0.0            # vehicle 0 absent in frame 1
    ei, ea = ref_radius_edges(x, 5.0)
    assert ei.tolist() == [[0, 1], [1, 0]]
    assert ea.tolist() == [[5.0, 5.0, 5.0, 25.0], [5.0, 5.0, 5.0, 25.0]]


@pytest.mark.gpu
@pytest.mark.parametrize("v,t", [(1, 10), (2, 2), (37, 7), (64, 100), (150, 100), (40, 129),
                                 (30, 256)])
@pytest.mark.parametrize("grid", [False, True])
def test_radius_edges_bit_exact(v, t, grid):
    from sldm_sage.gbuild import radius_edges_from_x
    x = _pack(v, t, seed=v * 1000 + t, grid=grid)
    radius = 5.0 if grid else 25.1
    ei_r, ea_r = ref_radius_edges(x, radius)
    ei_g, ea_g = radius_edges_from_x(x.cuda(), radius)
    assert torch.equal(ei_g.cpu(), ei_r)
    assert torch.equal(ea_g.cpu(), ea_r)


@pytest.mark.gpu
def test_radius_edges_strided_and_empty():
    from sldm_sage.gbuild import radius_edges
    x = _pack(20, 50, seed=3)
    xs = x.cuda()
    ei_g, ea_g = radius_edges(xs[:, :, 0:2], xs[:, :, 4], 1e-3)     # strided views
    ei_r, ea_r = ref_radius_edges(x, 1e-3)
    assert torch.equal(ei_g.cpu(), ei_r) and torch.equal(ea_g.cpu(), ea_r)
    e0, a0 = radius_edges(torch.zeros(0, 5, 2, device="cuda"), torch.zeros(0, 5, device="cuda"),
                          1.0)
    assert e0.shape == (2, 0) and a0.shape == (0, 4)
