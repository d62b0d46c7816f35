"""Tensor-level wrappers over the C ABI (device pointers + the current HIP stream).

Every op here launches a hand-written gfx950 kernel of libsldm_sage.so on
``torch.cuda.current_stream()``; outputs are allocated through the PyTorch
caching allocator.  CPU tensors are rejected: there is no CPU fallback.
"""
from __future__ import annotations

import torch

from . import _lib

_DTYPE_CODE = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}

# Optional per-kernel timing hook used by bench.py: a callable
# ``(name, start_event, end_event, units)`` or None.
_timing_hook = None


_timing_names = None


def set_timing_hook(hook, names=None) -> None:
    """Bracket launches with HIP events and hand them to ``hook`` (bench.py);
    ``names``: only these ops (None: all).  Diagnostic plumbing.  Launches
    made from Python here call ``hook(name, start_event, end_event, units)``;
    those made inside the ``torch.ops.sldm`` operators are recorded in C++ and
    reach ``hook.add_ms(name, ms, units)`` on :func:`flush_timing` (also
    called when the hook is removed)."""
    global _timing_hook, _timing_names
    from . import torch_ops
    if hook is None and _timing_hook is not None:
        flush_timing()
    _timing_hook = hook
    _timing_names = None if names is None else frozenset(names)
    torch_ops.timing_set(hook is not None, names)


def flush_timing() -> None:
    """Hand the launches recorded inside the C++ operators to the hook (waits
    for their end events)."""
    from . import torch_ops
    recs = torch_ops.timing_take()
    if _timing_hook is not None:
        for name, ms, units in recs:
            _timing_hook.add_ms(name, ms, units)


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DTYPE_CODE[t.dtype]
    except KeyError:
        raise TypeError(f"sldm_sage: unsupported dtype {t.dtype} (float32 or bfloat16)") from None


def _require_gpu(*ts: torch.Tensor) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "sldm_sage runs only on the GPU (HIP/gfx950); got a tensor on "
                f"'{t.device}'. There is no CPU fallback: move the inputs and the module "
                "to a ROCm device.")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"sldm_sage: tensors on different devices ({dev}, {t.device})")
    return dev


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(dev: torch.device) -> int:
    """The current HIP stream of ``dev`` as an integer handle (the raw query
    skips constructing a torch Stream object: a few µs per launch, which the
    small per-batch graphs notice)."""
    if _raw_stream is not None and dev.index is not None:
        return _raw_stream(dev.index)
    return torch.cuda.current_stream(dev).cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _f32(t: torch.Tensor | None) -> torch.Tensor | None:
    """An fp32 contiguous view of a small parameter (bias / gamma / beta) for
    its device pointer; the parameter itself when it already is one (the
    common case: no detach / copy per launch)."""
    if t is None or (t.dtype == torch.float32 and t.is_contiguous()):
        return t
    return t.detach().float().contiguous()


class _Timed:
    """Brackets one launch with HIP events when the timing hook is set."""

    __slots__ = ("name", "units", "start")

    def __init__(self, name: str, units: float):
        self.name, self.units, self.start = name, units, None

    def __enter__(self):
        if _timing_hook is not None and (_timing_names is None or self.name in _timing_names):
            self.start = torch.cuda.Event(enable_timing=True)
            self.start.record()
        return self

    def __exit__(self, *exc):
        if self.start is not None and exc[0] is None:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            _timing_hook(self.name, self.start, end, self.units)
        return False


# -------------------------------------------------- dropout under capture --
class dropout_seed_source:
    """While active, every dropout-keyed launch this thread makes through the
    library adds the int64 word of ``word`` (a 1-element device tensor), read
    on the device when the kernel runs, to its seed
    (``sldm_set_dropout_seed_source``): launches recorded into a HIP graph
    then draw a new mask on every replay that finds a new value there.
    ``None`` is a no-op."""

    __slots__ = ("word",)

    def __init__(self, word: torch.Tensor | None):
        if word is not None and (word.dtype != torch.int64 or word.numel() != 1
                                 or word.device.type != "cuda"):
            raise TypeError("dropout_seed_source: a 1-element int64 device tensor")
        self.word = word

    def __enter__(self):
        if self.word is not None:
            _lib.load().sldm_set_dropout_seed_source(self.word.data_ptr())
        return self

    def __exit__(self, *exc):
        if self.word is not None:
            _lib.load().sldm_set_dropout_seed_source(None)
        return False


_SEED_COUNTERS: dict[int, torch.Tensor] = {}
_SEED_STEP = 0x2545F4914F6CDD1D & (2**62 - 1)      # odd: the counter visits every value


def capture_seed_counter(device: torch.device, create: bool = True) -> torch.Tensor | None:
    """The device's dropout counter for HIP graph capture: one int64 word in
    [0, 2^62), advanced by a fixed odd step by every captured SageBlock call
    that drops (so each replay, and each call inside a replay, keys its masks
    anew).  Created -- outside any capture -- from the state of the device's
    default generator (torch.manual_seed governs it); ``create=False`` returns
    None when it does not exist yet."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _SEED_COUNTERS.get(idx)
    if t is None and create:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(
                "the dropout counter of HIP graph capture must exist before the capture "
                "begins: run one training call of the block eagerly first (the warm-up "
                "torch.cuda.graph asks for anyway) or call "
                "sldm_sage.ops.capture_seed_counter(device)")
        # keyed by the generator's seed and offset, without advancing it: an
        # eager call's masks do not depend on whether the counter exists yet
        from .sageblock import _splitmix64
        gen = torch.cuda.default_generators[idx]
        v = _splitmix64(gen.initial_seed() ^ _splitmix64(gen.get_offset() ^ 0x5EED)) & (2**62 - 1)
        t = torch.tensor([v], dtype=torch.int64, device=torch.device("cuda", idx))
        _SEED_COUNTERS[idx] = t
    return t


def next_capture_seed(device: torch.device) -> torch.Tensor:
    """Advance the device's counter and return a copy of its new value, both
    as launches on the current stream (recorded when it is capturing): the
    seed word of one SageBlock call."""
    c = capture_seed_counter(device)
    c.add_(_SEED_STEP).bitwise_and_(2**62 - 1)
    return c.clone()


# ------------------------------------------------------------------ graph --
def csr_build(edge_index: torch.Tensor, num_nodes: int, transpose: bool = True):
    """edge_index [2,E] (int64/int32, on the GPU) -> (rowptr, col, t_rowptr, t_col, bad).

    ``bad`` is a 1-element int32 device tensor, nonzero if an id was outside
    [0, num_nodes).  t_rowptr / t_col are None when ``transpose`` is False.
    """
    dev = _require_gpu(edge_index)
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
    if edge_index.dtype not in (torch.int64, torch.int32):
        raise TypeError(f"edge_index must be int64 or int32, got {edge_index.dtype}")
    ei = edge_index.contiguous()
    E = ei.size(1)
    N = int(num_nodes)
    lib = _lib.load()
    i32 = dict(dtype=torch.int32, device=dev)
    rowptr = torch.empty(N + 1, **i32)
    col = torch.empty(max(E, 1), **i32)[:E]
    t_rowptr = torch.empty(N + 1, **i32) if transpose else None
    t_col = torch.empty(max(E, 1), **i32)[:E] if transpose else None
    bad = torch.zeros(1, **i32)
    ws_bytes = lib.sldm_csr_workspace_bytes(E, N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with _Timed("csr_build", E):
        _lib.check(lib.sldm_csr_build(ei.data_ptr(), int(ei.dtype == torch.int64), E, N,
                                      rowptr.data_ptr(), col.data_ptr(), _ptr(t_rowptr),
                                      _ptr(t_col), bad.data_ptr(), ws.data_ptr(), ws_bytes,
                                      _stream(dev)),
                   "sldm_csr_build")
    return rowptr, col, t_rowptr, t_col, bad


def batch_graphs(edge_indices, num_nodes, transpose: bool = True):
    """PyG Batch.from_data_list for G device-resident edge_index tensors, fused
    with the batch CSR pair (``sldm_batch_graphs``, batch.hip).

    edge_indices: int64 [2, E_g] on one GPU (unit column stride); num_nodes:
    N_g per graph.  Returns (edge_index [2, E], batch [N], ptr [G+1], rowptr,
    col, t_rowptr, t_col, bad) -- ``bad`` as in :func:`csr_build`.
    """
    import ctypes
    dev = _require_gpu(*edge_indices)
    G = len(edge_indices)
    for ei in edge_indices:
        if ei.dtype != torch.int64 or ei.dim() != 2 or ei.size(0) != 2 or (
                ei.size(1) > 1 and ei.stride(1) != 1) or ei.device != dev:
            raise ValueError("batch_graphs: edge_index must be int64 [2, E] with unit column "
                             "stride on one device")
    ne = [int(ei.size(1)) for ei in edge_indices]
    nn = [int(n) for n in num_nodes]
    E, N = sum(ne), sum(nn)
    lib = _lib.load()
    out_ei = torch.empty(2, E, dtype=torch.int64, device=dev)
    bp = torch.empty(N + G + 1, dtype=torch.int64, device=dev)
    nt = 2 if transpose else 1
    buf = torch.empty(nt * (N + 1 + E) + 1, dtype=torch.int32, device=dev)
    rowptr, col = buf[:N + 1], buf[N + 1:N + 1 + E]
    t_rowptr = buf[N + 1 + E:2 * (N + 1) + E] if transpose else None
    t_col = buf[2 * (N + 1) + E:2 * (N + 1 + E)] if transpose else None
    bad = buf[-1:]
    ptrs = (ctypes.c_void_p * G)(*[ei.data_ptr() for ei in edge_indices])
    strides = (ctypes.c_int64 * G)(*[ei.stride(0) if ei.size(1) else 0 for ei in edge_indices])
    c_ne = (ctypes.c_int64 * G)(*ne)
    c_nn = (ctypes.c_int64 * G)(*nn)
    with _Timed("batch_graphs", E):
        _lib.check(lib.sldm_batch_graphs(G, ptrs, strides, c_ne, c_nn, out_ei.data_ptr(), E,
                                         bp.data_ptr(), bp[N:].data_ptr(), rowptr.data_ptr(),
                                         col.data_ptr(), _ptr(t_rowptr), _ptr(t_col),
                                         bad.data_ptr(), _stream(dev)),
                   "sldm_batch_graphs")
    return out_ei, bp[:N], bp[N:], rowptr, col, t_rowptr, t_col, bad


def degree_order(rowptr: torch.Tensor) -> torch.Tensor:
    """Rows by decreasing degree (stable): the longest-first gather schedule."""
    dev = _require_gpu(rowptr)
    n = rowptr.numel() - 1
    lib = _lib.load()
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
    ws_bytes = lib.sldm_degree_order_workspace_bytes(n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    _lib.check(lib.sldm_degree_order(rowptr.data_ptr(), n, order.data_ptr(), ws.data_ptr(),
                                     ws_bytes, _stream(dev)), "sldm_degree_order")
    return order


# ------------------------------------------------------------ aggregation --
def gather_rows(x: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor, num_rows: int,
                mean: bool, addend: torch.Tensor | None = None,
                out: torch.Tensor | None = None, name: str = "gather",
                order: torch.Tensor | None = None, edges: int | None = None,
                hub=None) -> torch.Tensor:
    """out[i] = (addend[i] +) sum_{k in row i} x[col[k]]  (/ max(1, deg_i) if mean).

    ``order`` (optional) lists the rows to compute, slot s -> row order[s]
    (``num_rows`` = len(order)): a schedule from :func:`degree_order`, or a
    row subset (then ``out`` holds all rows and ``edges`` is the subset's
    edge count, for the timing hook's byte accounting).  ``hub`` (a
    :class:`~sldm_sage.graph.HubPlan` of ``rowptr``): its high-degree rows
    are summed as split edge chunks (``sldm_gather_rows_split``); with a row
    subset in ``order`` the plan must list exactly the subset's hubs (rows
    above the plan's max_deg are never summed by a row slot)."""
    dev = _require_gpu(x, rowptr, col, addend, out, order)
    if x.dim() != 2 or x.stride(1) != 1:
        x = x.contiguous()
    F = x.size(1)
    if out is None:
        out = torch.empty(num_rows, F, dtype=x.dtype, device=dev)
    if addend is not None:
        if addend.dtype != out.dtype or addend.stride(-1) != 1:
            addend = addend.to(out.dtype).contiguous()
    if num_rows == 0 or F == 0:
        return out
    E = col.numel()
    s = x.element_size()
    bytes_alg = (E if edges is None else edges) * (4 + F * s) + (num_rows + 1) * 4 + num_rows * F * s * (2 if addend is not None else 1)
    if hub is not None:
        partials = torch.empty(hub.num_chunks, F, dtype=torch.float32, device=dev)
        with _Timed(name, bytes_alg):
            _lib.check(_lib.load().sldm_gather_rows_split(
                dtype_code(x), x.data_ptr(), x.stride(0), rowptr.data_ptr(),
                col.data_ptr() if E else rowptr.data_ptr(), _ptr(order), num_rows, F,
                int(bool(mean)),
                _ptr(addend), addend.stride(0) if addend is not None else 0,
                dtype_code(out), out.data_ptr(), out.stride(0), hub.hub_rows.data_ptr(),
                hub.chunk_ptr.data_ptr(), hub.num_hubs, hub.chunk_row.data_ptr(),
                hub.chunk_beg.data_ptr(), hub.num_chunks, hub.chunk_len, hub.max_deg,
                partials.data_ptr(), _stream(dev)), "sldm_gather_rows_split")
        return out
    with _Timed(name, bytes_alg):
        _lib.check(_lib.load().sldm_gather_rows(
            dtype_code(x), x.data_ptr(), x.stride(0), rowptr.data_ptr(),
            col.data_ptr() if E else rowptr.data_ptr(), _ptr(order), num_rows, F, int(bool(mean)),
            _ptr(addend), addend.stride(0) if addend is not None else 0,
            dtype_code(out), out.data_ptr(), out.stride(0), _stream(dev)), "sldm_gather_rows")
    return out


def scale_rows_by_inv_deg_(d: torch.Tensor, rowptr: torch.Tensor) -> torch.Tensor:
    dev = _require_gpu(d, rowptr)
    assert d.stride(1) == 1
    _lib.check(_lib.load().sldm_scale_rows_by_inv_deg(
        dtype_code(d), d.data_ptr(), d.stride(0), rowptr.data_ptr(), d.size(0), d.size(1),
        _stream(dev)), "sldm_scale_rows_by_inv_deg")
    return d


# ------------------------------------------------------------ dense (MFMA) --
def sage_dense_fwd(agg: torch.Tensor, x: torch.Tensor, wcat: torch.Tensor, bias, gamma, beta,
                   eps: float, slope: float, drop_p: float, seed: int, save: bool,
                   row_offset: int = 0, outs=None):
    """out = dropout(act(LN([agg|x]·wcat^T + bias))); returns (out, xhat|None, rstd|None).

    wcat is [F_out, 2 F_in] (= [W_l | W_r]) in x's dtype.  ``outs``: optional
    preallocated (out, xhat, rstd), contiguous (row slices of bigger tensors)."""
    dev = _require_gpu(agg, x, wcat, gamma, beta, bias)
    n, fi = x.shape
    fo = wcat.size(0)
    assert agg.shape == x.shape and agg.stride(1) == 1 and x.stride(1) == 1
    assert wcat.is_contiguous() and wcat.shape == (fo, 2 * fi) and wcat.dtype == x.dtype
    if outs is not None:
        out, xhat, rstd = outs
        assert out.is_contiguous() and out.shape == (n, fo) and out.dtype == x.dtype
        assert (xhat is not None) == save and (rstd is not None) == save
        assert not save or (xhat.is_contiguous() and rstd.is_contiguous())
    else:
        out = torch.empty(n, fo, dtype=x.dtype, device=dev)
        xhat = torch.empty(n, fo, dtype=x.dtype, device=dev) if save else None
        rstd = torch.empty(n, dtype=torch.float32, device=dev) if save else None
    bias_, gamma_, beta_ = _f32(bias), _f32(gamma), _f32(beta)
    s = x.element_size()
    with _Timed("dense_fwd", (2 * n * fi + n * fo * (2 if save else 1)) * s):
        _lib.check(_lib.load().sldm_sage_dense_fwd(
            dtype_code(x), agg.data_ptr(), agg.stride(0), fi, x.data_ptr(), x.stride(0), fi,
            wcat.data_ptr(), n, fo, _ptr(bias_), gamma_.data_ptr(), beta_.data_ptr(), float(eps),
            float(slope), float(drop_p), seed & (2**64 - 1), int(row_offset), out.data_ptr(), _ptr(xhat),
            _ptr(rstd), _stream(dev)), "sldm_sage_dense_fwd")
    return out, xhat, rstd


def gemm_nt_rowscale(a: torch.Tensor, b: torch.Tensor, rowptr: torch.Tensor | None,
                     scale_cols: int, split: bool = False):
    """C = a · b^T, columns < scale_cols divided by max(1, deg(row)).

    ``split``: return (C[:, :scale_cols], C[:, scale_cols:]) as two separate
    contiguous tensors (one launch) instead of one [n, nc] tensor."""
    dev = _require_gpu(a, b, rowptr)
    assert a.stride(1) == 1 and b.is_contiguous() and a.dtype == b.dtype
    n, k = a.shape
    nc = b.size(0)
    if split:
        if not 0 < scale_cols < nc or scale_cols % 4:
            raise ValueError("gemm_nt_rowscale(split=True) needs 0 < scale_cols < nc, "
                             "scale_cols % 4 == 0")
        out = torch.empty(n, scale_cols, dtype=a.dtype, device=dev)
        out2 = torch.empty(n, nc - scale_cols, dtype=a.dtype, device=dev)
    else:
        out = torch.empty(n, nc, dtype=a.dtype, device=dev)
        out2 = None
    with _Timed("dense_bwd_data", (n * k + n * nc) * a.element_size()):
        _lib.check(_lib.load().sldm_gemm_nt_rowscale(
            dtype_code(a), a.data_ptr(), a.stride(0), k, b.data_ptr(), b.stride(0), n, nc,
            _ptr(rowptr), scale_cols, out.data_ptr(), out.stride(0), _ptr(out2),
            out2.stride(0) if out2 is not None else 0, _stream(dev)),
            "sldm_gemm_nt_rowscale")
    return (out, out2) if split else out


def gemm_nt_rowscale_blocked_ok(a: torch.Tensor, nc: int, scale_cols: int, blk_cols: int) -> bool:
    """Whether :func:`gemm_nt_rowscale_blocked` takes this dtype / shape."""
    return (a.is_cuda and a.dtype in _DTYPE_CODE and a.stride(1) == 1 and a.stride(0) % 8 == 0
            and bool(_lib.load().sldm_gemm_nt_rowscale_blocked_ok(
                dtype_code(a), a.size(1), nc, scale_cols, blk_cols)))


def gemm_nt_rowscale_blocked(a: torch.Tensor, b: torch.Tensor, rowptr: torch.Tensor | None,
                             scale_cols: int, blk_cols: int, out2: torch.Tensor | None = None):
    """C = a · b^T as :func:`gemm_nt_rowscale` (split=True), the scaled half
    C[:, :scale_cols] / deg returned column-blocked: flat [scale_cols //
    blk_cols][n][blk_cols] -- what :func:`cols_pack` makes of it, written by
    the GEMM.  Returns (blocked, C[:, scale_cols:])."""
    dev = _require_gpu(a, b, rowptr, out2)
    assert a.stride(1) == 1 and b.is_contiguous() and a.dtype == b.dtype
    n, k = a.shape
    nc = b.size(0)
    out = torch.empty(n * scale_cols, dtype=a.dtype, device=dev)
    if out2 is None:
        out2 = torch.empty(n, nc - scale_cols, dtype=a.dtype, device=dev)
    assert out2.shape == (n, nc - scale_cols) and out2.stride(1) == 1 and out2.dtype == a.dtype
    with _Timed("dense_bwd_data", (n * k + n * nc) * a.element_size()):
        _lib.check(_lib.load().sldm_gemm_nt_rowscale_blocked(
            dtype_code(a), a.data_ptr(), a.stride(0), k, b.data_ptr(), b.stride(0), n, nc,
            _ptr(rowptr), scale_cols, out.data_ptr(), blk_cols, out2.data_ptr(), out2.stride(0),
            _stream(dev)), "sldm_gemm_nt_rowscale_blocked")
    return out, out2


def gemm_tn(a: torch.Tensor, b0: torch.Tensor, b1: torch.Tensor | None, split: bool = False):
    """fp32 [a.size(1), b0.size(1)+b1.size(1)] = a^T · [b0 | b1] (sum over rows).

    ``split``: return (a^T b0, a^T b1) as two contiguous tensors written by the
    same launch (``sldm_gemm_tn_split``), the layer's (dW_l, dW_r)."""
    dev = _require_gpu(a, b0, b1)
    assert a.stride(1) == 1 and b0.stride(1) == 1 and (b1 is None or b1.stride(1) == 1)
    rows, mo = a.shape
    n0 = b0.size(1)
    n1 = 0 if b1 is None else b1.size(1)
    if split and not (n0 and n1):
        raise ValueError("gemm_tn(split=True) needs two non-empty operands")
    lib = _lib.load()
    ws_bytes = lib.sldm_gemm_tn_workspace_bytes(rows, mo, n0 + n1)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with _Timed("dense_bwd_weight", rows * (mo + n0 + n1) * a.element_size()):
        if split:
            out0 = torch.empty(mo, n0, dtype=torch.float32, device=dev)
            out1 = torch.empty(mo, n1, dtype=torch.float32, device=dev)
            _lib.check(lib.sldm_gemm_tn_split(
                dtype_code(a), a.data_ptr(), a.stride(0), mo, b0.data_ptr(), b0.stride(0), n0,
                b1.data_ptr(), b1.stride(0), n1, rows, out0.data_ptr(), out1.data_ptr(),
                ws.data_ptr(), ws_bytes, _stream(dev)), "sldm_gemm_tn_split")
            return out0, out1
        out = torch.empty(mo, n0 + n1, dtype=torch.float32, device=dev)
        _lib.check(lib.sldm_gemm_tn(
            dtype_code(a), a.data_ptr(), a.stride(0), mo, b0.data_ptr(), b0.stride(0), n0,
            _ptr(b1), b1.stride(0) if b1 is not None else 0, n1, rows, out.data_ptr(),
            ws.data_ptr(), ws_bytes, _stream(dev)), "sldm_gemm_tn")
    return out


# ------------------------------------------------------------------- post --
def post_fwd(h: torch.Tensor, bias, gamma, beta, eps: float, slope: float, drop_p: float,
             seed: int, out_dtype: torch.dtype, save: bool, row_offset: int = 0):
    """bias + LayerNorm + (Leaky)ReLU + dropout; returns (out, xhat|None, rstd|None)."""
    dev = _require_gpu(h, gamma, beta, bias)
    N, F = h.shape
    if h.stride(1) != 1:
        h = h.contiguous()
    out = torch.empty(N, F, dtype=out_dtype, device=dev)
    xhat = torch.empty(N, F, dtype=out_dtype, device=dev) if save else None
    rstd = torch.empty(N, dtype=torch.float32, device=dev) if save else None
    bias_, gamma_, beta_ = _f32(bias), _f32(gamma), _f32(beta)
    with _Timed("post_fwd", N * F * (h.element_size() + out.element_size() * (2 if save else 1))):
        _lib.check(_lib.load().sldm_post_fwd(
            dtype_code(h), h.data_ptr(), h.stride(0), N, F, _ptr(bias_), gamma_.data_ptr(),
            beta_.data_ptr(), float(eps), float(slope), float(drop_p), seed & (2**64 - 1), int(row_offset),
            _DTYPE_CODE[out_dtype], out.data_ptr(), _ptr(xhat), _ptr(rstd), _stream(dev)),
            "sldm_post_fwd")
    return out, xhat, rstd


def gather_post_bwd(g: torch.Tensor, t_rowptr: torch.Tensor, t_col: torch.Tensor,
                    t_order: torch.Tensor | None, addend: torch.Tensor, xhat: torch.Tensor,
                    rstd: torch.Tensor, gamma, beta, slope: float, drop_p: float, seed: int,
                    row_offset: int = 0):
    """Fused layer boundary of the backward (gather_post.hip): the transpose
    gather of layer l (+ its root-path ``addend``) fed straight into layer
    l-1's LayerNorm/act/dropout backward.  Returns (dh, dgamma, dbeta, dbias)
    of layer l-1, as :func:`post_bwd` would from the gathered gradient."""
    dev = _require_gpu(g, t_rowptr, t_col, t_order, addend, xhat, rstd)
    N, F = xhat.shape
    assert g.dtype == xhat.dtype == addend.dtype and g.stride(1) == 1 and addend.stride(1) == 1
    assert xhat.is_contiguous() and g.size(1) == F and addend.shape == (N, F)
    lib = _lib.load()
    np_ = lib.sldm_gather_post_bwd_num_partials(N, F)
    dh = torch.empty(N, F, dtype=xhat.dtype, device=dev)
    partials = torch.empty(np_, 3 * F, dtype=torch.float32, device=dev)
    cols = torch.empty(3 * F, dtype=torch.float32, device=dev)
    gamma_, beta_ = _f32(gamma), _f32(beta)
    s = xhat.element_size()
    E = t_col.numel()
    with _Timed("gather_post_bwd", E * (4 + F * s) + (N + 1) * 4 + 3 * N * F * s + 4 * N):
        _lib.check(lib.sldm_gather_post_bwd(
            dtype_code(xhat), g.data_ptr(), g.stride(0), t_rowptr.data_ptr(),
            t_col.data_ptr() if E else t_rowptr.data_ptr(), _ptr(t_order), addend.data_ptr(),
            addend.stride(0), N, F, xhat.data_ptr(), rstd.data_ptr(), gamma_.data_ptr(),
            beta_.data_ptr(), float(slope), float(drop_p), seed & (2**64 - 1), int(row_offset),
            dh.data_ptr(), partials.data_ptr(), np_, _stream(dev)), "sldm_gather_post_bwd")
        _lib.check(lib.sldm_colsum(partials.data_ptr(), np_, 3 * F, cols.data_ptr(),
                                   _stream(dev)), "sldm_colsum")
    return dh, cols[:F], cols[F:2 * F], cols[2 * F:]


def cols_layout_ok(t: torch.Tensor, block_cols: int) -> bool:
    """Whether :func:`cols_pack` / :func:`cols_unpack` take this dtype / width."""
    return t.dtype in _DTYPE_CODE and (block_cols * t.element_size()) % 16 == 0


def cols_pack(rows: torch.Tensor, num_blocks: int, block_cols: int,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """rows [n, B*bc] -> flat [B][n][bc] (layout.hip)."""
    dev = _require_gpu(rows, out)
    n = rows.size(0)
    assert rows.size(1) == num_blocks * block_cols and rows.stride(1) == 1
    if out is None:
        out = torch.empty(num_blocks * n * block_cols, dtype=rows.dtype, device=dev)
    with _Timed("cols_pack", 2 * rows.numel() * rows.element_size()):
        _lib.check(_lib.load().sldm_cols_pack(dtype_code(rows), rows.data_ptr(), rows.stride(0),
                                              n, num_blocks, block_cols, out.data_ptr(),
                                              _stream(dev)), "sldm_cols_pack")
    return out


def cols_unpack(blocks: torch.Tensor, num_rows: int, num_blocks: int, block_cols: int,
                out: torch.Tensor, addend: torch.Tensor | None = None) -> torch.Tensor:
    """flat [B][n][bc] -> out [n, B*bc] (+ addend, one rounding) (layout.hip)."""
    dev = _require_gpu(blocks, out, addend)
    assert out.shape == (num_rows, num_blocks * block_cols) and out.stride(1) == 1
    if addend is not None:
        assert addend.shape == out.shape and addend.stride(1) == 1 and addend.dtype == out.dtype
    with _Timed("cols_unpack", (2 + (addend is not None)) * out.numel() * out.element_size()):
        _lib.check(_lib.load().sldm_cols_unpack(
            dtype_code(out), blocks.data_ptr(), num_rows, num_blocks, block_cols, _ptr(addend),
            addend.stride(0) if addend is not None else 0, out.data_ptr(), out.stride(0),
            _stream(dev)), "sldm_cols_unpack")
    return out


def post_bwd(dout: torch.Tensor, xhat: torch.Tensor, rstd: torch.Tensor, gamma, beta,
             slope: float, drop_p: float, seed: int, dh_dtype: torch.dtype,
             zout: torch.Tensor | None = None, row_offset: int = 0):
    """Returns (dh [N,F], dgamma [F], dbeta [F], dbias [F]) (the last three fp32).

    ``zout`` (the forward output) fixes the activation branch exactly."""
    dev = _require_gpu(dout, xhat, rstd, zout)
    N, F = xhat.shape
    if dout.dtype != xhat.dtype or dout.stride(1) != 1 or dout.stride(0) != F:
        dout = dout.to(xhat.dtype).contiguous()
    if zout is not None:
        assert zout.dtype == xhat.dtype and zout.is_contiguous() and zout.shape == xhat.shape
    lib = _lib.load()
    np_ = lib.sldm_post_num_partials(N, F)
    dh = torch.empty(N, F, dtype=dh_dtype, device=dev)
    partials = torch.empty(np_, 3 * F, dtype=torch.float32, device=dev)
    cols = torch.empty(3 * F, dtype=torch.float32, device=dev)
    gamma_, beta_ = _f32(gamma), _f32(beta)
    with _Timed("post_bwd", N * F * ((3 if zout is not None else 2) * xhat.element_size()
                                     + dh.element_size())):
        _lib.check(lib.sldm_post_bwd(
            dtype_code(xhat), dout.data_ptr(), xhat.data_ptr(), _ptr(zout), rstd.data_ptr(), N, F,
            gamma_.data_ptr(), beta_.data_ptr(), float(slope), float(drop_p),
            seed & (2**64 - 1), int(row_offset), _DTYPE_CODE[dh_dtype], dh.data_ptr(), partials.data_ptr(), np_,
            _stream(dev)), "sldm_post_bwd")
        _lib.check(lib.sldm_colsum(partials.data_ptr(), np_, 3 * F, cols.data_ptr(),
                                   _stream(dev)), "sldm_colsum")
    return dh, cols[:F], cols[F:2 * F], cols[2 * F:]
