"""Graph-level readout: global mean / max / mean||max pooling over ``batch``.

Drop-in for the PyG 2.7.0 readouts GruSage uses (grusage.py:3 import,
:119-127 selection, :185 call):

    global_mean_pool(x, batch, size=None)   # utils.scatter(reduce='mean')
    global_max_pool(x, batch, size=None)    # utils.scatter(reduce='max')
    global_pool(mode)                       # the 'mean' | 'max' | 'double' callable

Same signatures and semantics: ``batch=None`` pools all rows into one
graph (max gradient to the first maximal row, as x.max(dim)); ``size``
defaults to ``batch.max() + 1``; empty graphs give 0; with a batch the max
gradient is split evenly among tied maxima with torch's amax-backward
divisor (pool.hip header).  Compute runs in libsldm_sage.so (pool.hip); the
segment CSR of a ``batch`` tensor is built once by the CSR kernel and cached
on the tensor object like a graph.
"""
from __future__ import annotations

import threading
import weakref

import torch

from . import _lib, ops

_MEAN, _MAX = 1, 2


class _Segments:
    __slots__ = ("num_segments", "rowptr", "member", "piece_ptr", "num_pieces", "seg_of")

    def __init__(self, batch: torch.Tensor, size: int):
        dev = batch.device
        n = batch.numel()
        b = batch.reshape(-1)
        ei = torch.stack([torch.arange(n, device=dev, dtype=torch.int64), b.to(torch.int64)])
        rowptr, member, _, _, bad = ops.csr_build(ei, max(n, size, 1), transpose=False)
        if n and int(bad.item()) != 0:
            raise IndexError(f"batch holds a graph id outside [0, {size})")
        self.num_segments = size
        self.rowptr = rowptr[: size + 1]
        self.member = member
        piece = _lib.load().sldm_segment_pool_piece_rows()
        lens = (self.rowptr[1:] - self.rowptr[:-1]).to(torch.int64)
        pieces = torch.div(lens + piece - 1, piece, rounding_mode="floor")
        self.piece_ptr = torch.zeros(size + 1, dtype=torch.int32, device=dev)
        if size:
            self.piece_ptr[1:] = torch.cumsum(pieces, 0).to(torch.int32)
        self.num_pieces = int(self.piece_ptr[-1].item()) if size else 0
        self.seg_of = b.to(torch.int64).contiguous()


class _SegmentCache:
    """batch tensor -> _Segments, keyed like the graph cache (object + version)."""

    def __init__(self, max_entries: int = 64):
        self._lock = threading.RLock()
        self._entries: dict[int, tuple] = {}
        self._max = max_entries

    def get(self, batch: torch.Tensor, size: int) -> _Segments:
        if batch.is_inference():
            return _Segments(batch, size)
        key, ver = id(batch), batch._version
        with self._lock:
            ent = self._entries.get(key)
        if ent is not None and ent[0]() is batch and ent[1] == ver and ent[2].num_segments == size:
            return ent[2]
        seg = _Segments(batch, size)
        try:
            ref = weakref.ref(batch, lambda _r, k=key: self._drop(k))
        except TypeError:
            return seg
        with self._lock:
            if len(self._entries) >= self._max:
                self._entries.pop(next(iter(self._entries)))
            self._entries[key] = (ref, ver, seg)
        return seg

    def _drop(self, key):
        with self._lock:
            self._entries.pop(key, None)

    def clear(self):
        with self._lock:
            self._entries.clear()


segment_cache = _SegmentCache()


def _segments(x: torch.Tensor, batch: torch.Tensor | None, size: int | None) -> _Segments:
    if batch is None:
        batch = _zeros_batch(x.size(0), x.device)
        size = 1 if size is None else size
    if size is None:
        size = int(batch.max().item()) + 1 if batch.numel() else 0
    return segment_cache.get(batch, int(size))


_ZEROS: dict = {}


def _zeros_batch(n: int, dev: torch.device) -> torch.Tensor:
    key = (n, str(dev))
    t = _ZEROS.get(key)
    if t is None:
        if len(_ZEROS) >= 16:
            _ZEROS.clear()
        t = _ZEROS[key] = torch.zeros(n, dtype=torch.int64, device=dev)
    return t


class _PoolFn(torch.autograd.Function):
    """``torch.ops.sldm.segment_pool`` / ``segment_pool_bwd`` (pool.hip)."""

    @staticmethod
    def forward(ctx, x, seg: _Segments, mode: int, first_arg: bool):
        from . import torch_ops
        x = x.contiguous()
        out, div, arg = torch_ops.load().segment_pool(x, seg.rowptr, seg.member, seg.piece_ptr,
                                                      seg.num_segments, seg.num_pieces, mode,
                                                      first_arg)
        ctx.seg, ctx.mode = seg, mode
        ctx.save_for_backward(x, out, div, arg)
        return out

    @staticmethod
    def backward(ctx, gout):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        x, out, div, arg = ctx.saved_tensors
        seg = ctx.seg
        dx = torch.ops.sldm.segment_pool_bwd(gout, x, out, div, arg, seg.seg_of, seg.rowptr,
                                             ctx.mode)
        return dx, None, None, None


def _pool(x: torch.Tensor, batch, size, mode: int) -> torch.Tensor:
    if x.dim() != 2:
        raise ValueError(f"pooling expects x [N, F], got {tuple(x.shape)}")
    if x.device.type == "cpu":
        # the reference's CPU mode (main.py:58): the host library
        from . import cpu
        first = batch is None
        if first:
            batch, size = torch.zeros(x.size(0), dtype=torch.int64), (1 if size is None else size)
        if size is None:
            size = int(batch.max().item()) + 1 if batch.numel() else 0
        if x.size(0) == 0 or x.size(1) == 0:
            return x.new_zeros(int(size), x.size(1) * (2 if mode == _MEAN | _MAX else 1))
        return cpu.PoolFn.apply(x, batch, int(size), mode, first)
    ops._require_gpu(x, batch)
    seg = _segments(x, batch, size)
    if x.size(0) == 0 or x.size(1) == 0:
        B, F = seg.num_segments, x.size(1)
        return x.new_zeros(B, F * (2 if mode == _MEAN | _MAX else 1))
    # batch=None: PyG reduces with x.max(dim) (gradient to the first maximal
    # row) instead of the scatter amax (gradient split over ties)
    return _PoolFn.apply(x, seg, mode, batch is None)


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """Per-graph mean of node rows (PyG 2.7.0 global_mean_pool)."""
    return _pool(x, batch, size, _MEAN)


def global_max_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """Per-graph column max of node rows (PyG 2.7.0 global_max_pool)."""
    return _pool(x, batch, size, _MAX)


def global_mean_max_pool(x: torch.Tensor, batch: torch.Tensor | None, size: int | None = None):
    """cat([mean, max], 1) in one pass over x (GruSage 'double', grusage.py:124)."""
    return _pool(x, batch, size, _MEAN | _MAX)


def global_pool(mode: str):
    """The readout callable GruSage selects (grusage.py:119-127)."""
    if mode == "mean":
        return global_mean_pool
    if mode == "max":
        return global_max_pool
    if mode == "double":
        return global_mean_max_pool
    raise ValueError(f"Unsupported global_pooling method: {mode}")
