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


def _pool_fwd(x: torch.Tensor, seg: _Segments, mode: int, first_arg: bool):
    dev = ops._require_gpu(x, seg.rowptr)
    B, F = seg.num_segments, x.size(1)
    dt = ops.dtype_code(x)
    lib = _lib.load()
    out = torch.empty(B, F * (2 if mode == _MEAN | _MAX else 1), dtype=x.dtype, device=dev)
    mean = out[:, :F] if mode & _MEAN else None
    mx = out[:, F * (1 if mode & _MEAN else 0):] if mode & _MAX else None
    div = (torch.empty(B, F, dtype=torch.float32, device=dev)
           if mode & _MAX and not first_arg else None)
    arg = torch.empty(B, F, dtype=torch.int32, device=dev) if mode & _MAX and first_arg else None
    ws_bytes = lib.sldm_segment_pool_workspace_bytes(seg.num_pieces, F)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with ops._Timed("pool_fwd", x.numel() * x.element_size()):
        _lib.check(lib.sldm_segment_pool(
            dt, x.data_ptr(), x.stride(0), seg.rowptr.data_ptr(), seg.member.data_ptr(), B,
            seg.piece_ptr.data_ptr(), seg.num_pieces, F, ops._ptr(mean),
            mean.stride(0) if mean is not None else 0, ops._ptr(mx),
            mx.stride(0) if mx is not None else 0, ops._ptr(div), ops._ptr(arg), ws.data_ptr(),
            ws_bytes, ops._stream(dev)), "sldm_segment_pool")
    return out, mx, div, arg


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seg: _Segments, mode: int, first_arg: bool):
        x = x.contiguous()
        out, mx, div, arg = _pool_fwd(x, seg, mode, first_arg)
        ctx.seg, ctx.mode = seg, mode
        if mode & _MAX:
            ctx.save_for_backward(x, mx, div, arg)
        else:
            ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, gout):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        seg, mode = ctx.seg, ctx.mode
        x = ctx.saved_tensors[0]
        mx, div, arg = ctx.saved_tensors[1:] if mode & _MAX else (None, None, None)
        F = x.size(1)
        g = gout.to(x.dtype)
        if g.stride(-1) != 1:
            g = g.contiguous()
        dmean = g[:, :F] if mode & _MEAN else None
        dmax = g[:, F * (1 if mode & _MEAN else 0):] if mode & _MAX else None
        dev = x.device
        dx = torch.empty_like(x)
        n = x.size(0)
        with ops._Timed("pool_bwd", 2 * x.numel() * x.element_size()):
            _lib.check(_lib.load().sldm_segment_pool_bwd(
                ops.dtype_code(x), x.data_ptr(), x.stride(0), seg.seg_of.data_ptr(),
                seg.rowptr.data_ptr(), n, F, ops._ptr(dmean),
                dmean.stride(0) if dmean is not None else 0, ops._ptr(mx),
                mx.stride(0) if mx is not None else 0, ops._ptr(dmax),
                dmax.stride(0) if dmax is not None else 0, ops._ptr(div), ops._ptr(arg),
                dx.data_ptr(), dx.stride(0), ops._stream(dev)), "sldm_segment_pool_bwd")
        return dx, None, None, None


def _pool(x: torch.Tensor, batch, size, mode: int) -> torch.Tensor:
    if x.dim() != 2:
        raise ValueError(f"pooling expects x [N, F], got {tuple(x.shape)}")
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
