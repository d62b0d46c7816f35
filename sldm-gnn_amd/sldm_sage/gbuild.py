"""Vehicle-graph edge construction on the GPU.

``radius_edges(pos, presence, radius)`` replaces the O(V^2 T) Python pair
loop of the reference's graph builders -- gbuilder.py:85-111 (offline,
build.py) and :241-268 (``GraphOnlineCreator``, run per pack on the online
path rcv.py:60, :77) -- with one kernel (radius.hip) that reproduces its
numpy float32 arithmetic bit for bit: same edges in the same order (i-major,
j ascending, no self loops) and the same ``edge_attr`` rows
[min, max, mean, mean of squares] of the per-frame distances over the frames
both vehicles are present in.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, ops


def radius_edges(pos: torch.Tensor, presence: torch.Tensor, radius: float):
    """pos [V, T, 2] (X, Y), presence [V, T] (flag > 0.5 = present), fp32 on the
    GPU -> (edge_index int64 [2, E], edge_attr fp32 [E, 4])."""
    dev = ops._require_gpu(pos, presence)
    if pos.dim() != 3 or pos.size(2) != 2 or presence.shape != pos.shape[:2]:
        raise ValueError(f"radius_edges: pos [V, T, 2] and presence [V, T] expected, got "
                         f"{tuple(pos.shape)} and {tuple(presence.shape)}")
    if pos.dtype != torch.float32 or presence.dtype != torch.float32:
        pos, presence = pos.float(), presence.float()
    V, T = presence.shape
    cap = max(V * (V - 1), 1)
    ei = torch.empty(2, cap, dtype=torch.int64, device=dev)
    attr = torch.empty(cap, 4, dtype=torch.float32, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws_bytes = lib.sldm_radius_edges_workspace_bytes(V)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    # the reference compares min(d) (float32) with a Python float: numpy 2
    # promotes the Python float to float32 first
    r32 = float(np.float32(radius))
    _lib.check(lib.sldm_radius_edges(
        pos.data_ptr(), pos.stride(0), pos.stride(1), pos.stride(2), presence.data_ptr(),
        presence.stride(0), presence.stride(1), V, T, r32, ei.data_ptr(), cap, attr.data_ptr(),
        count.data_ptr(), ws.data_ptr(), ws_bytes, ops._stream(dev)), "sldm_radius_edges")
    e = int(count.item())
    return ei[:, :e].contiguous(), attr[:e].contiguous()


def radius_edges_from_x(x: torch.Tensor, radius: float):
    """The builders' temporal features x [V, T, 5] ([X, Y, Speed, Angle,
    PresenceFlag], before the heading's sin/cos encoding, gbuilder.py:64-87)."""
    return radius_edges(x[:, :, 0:2], x[:, :, 4], radius)
