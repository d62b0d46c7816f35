"""Drop-in ``SageBlock`` (and ``SageConv``) running on hand-written gfx950 kernels.

Mirrors /root/reference/src/models/blocks/sageblock.py:4-20 exactly at the API
level — constructor ``SageBlock(hdims, dropout=None, negative_slope=None)``,
``forward(x, edge_index)``, the module tree and therefore the state_dict keys

    convs.{i}.lin_l.weight [F_{i+1}, F_i]   convs.{i}.lin_l.bias [F_{i+1}]
    convs.{i}.lin_r.weight [F_{i+1}, F_i]   posts.{i}.0.weight / .bias [F_{i+1}]

(posts.{i}.1 is LeakyReLU/ReLU, posts.{i}.2 Dropout/Identity) — so GruSage
(grusage.py:108-110,182), MapEncoder (mapencoder.py:20-25,37), strict
``load_state_dict`` of old snapshots (test.py:122, rcv.py:63),
``state_dict_no_mapenc`` (grusage.py:141) and ``grads()`` (grusage.py:204)
work unchanged.

Each layer (PyG 2.7.0 SAGEConv(mean) + LayerNorm + act + Dropout) runs as
one autograd node over the C ABI:
  forward : gather-mean over CSR-by-dst -> [agg|x]·[W_l|W_r]^T -> bias+LN+act+dropout
  backward: LN/act/dropout bwd -> dh·[W_l|W_r] -> dW -> 1/deg prescale ->
            transpose gather + lin_r grad
Dropout masks come from a counter-based hash (not torch's RNG stream), so
parity runs use eval mode or dropout=None.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import dense, ops
from .graph import SageGraph, get_graph


def _act_slope(act: nn.Module) -> float:
    if isinstance(act, nn.LeakyReLU):
        return float(act.negative_slope)
    if isinstance(act, nn.ReLU):
        return 0.0
    raise TypeError(f"SageBlock post activation must be LeakyReLU or ReLU, got {type(act)}")


def _drop_p(drop: nn.Module) -> float:
    if isinstance(drop, nn.Identity):
        return 0.0
    if isinstance(drop, nn.Dropout):
        return float(drop.p) if drop.training else 0.0
    raise TypeError(f"SageBlock post dropout must be Dropout or Identity, got {type(drop)}")


def _splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


_SEED_LOCK = __import__("threading").Lock()


def _new_seed(device: torch.device | None = None) -> int:
    """Dropout key of one layer call, drawn the way nn.Dropout on a GPU
    draws its mask: from the device's default generator (its seed and philox
    offset, the offset advanced per call), so torch.manual_seed governs the
    masks and the caller's CPU RNG stream (DataLoader shuffling, CPU randn)
    is left untouched.  No device sync."""
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    gen = torch.cuda.default_generators[dev.index if dev.index is not None
                                        else torch.cuda.current_device()]
    with _SEED_LOCK:
        off = gen.get_offset()
        gen.set_offset(off + 4)
    return _splitmix64(gen.initial_seed() ^ _splitmix64(off)) & (2**62 - 1)


class _SageLayerFn(torch.autograd.Function):
    """One SageBlock layer: SAGEConv(mean) -> LayerNorm -> act -> dropout."""

    @staticmethod
    def forward(ctx, x, wl, bl, wr, gamma, beta, graph: SageGraph, slope: float, drop_p: float,
                seed: int, eps: float):
        n = x.size(0)
        agg = ops.gather_rows(x, graph.rowptr, graph.col, n, mean=True, name="gather_fwd",
                              order=graph.order, hub=graph.hub)
        needs_grad = any(ctx.needs_input_grad[:6])
        wcat = dense.weight_cat(wl, wr, x.dtype)
        out, xhat, rstd = dense.sage_layer_fwd(agg, x, wl, bl, wr, gamma, beta, eps, slope,
                                               drop_p, seed, save=needs_grad, wcat=wcat)
        if needs_grad:
            ctx.wcat = wcat
            # `out` is saved too (it is the next layer's input anyway): with
            # SLDM_ACT_BRANCH_FROM_OUTPUT=1 its sign picks the activation
            # branch in the backward (ops.branch_source).
            ctx.save_for_backward(x, agg, xhat, rstd, wl, wr, gamma, beta, out)
            ctx.graph = graph
            ctx.cfg = (slope, drop_p, seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, agg, xhat, rstd, wl, wr, gamma, beta, out = ctx.saved_tensors
        graph: SageGraph = ctx.graph
        slope, drop_p, seed = ctx.cfg
        dh, dgamma, dbeta, dbl = ops.post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed,
                                              dh_dtype=x.dtype, zout=ops.branch_source(out))
        dwl, dwr = dense.sage_linear_bwd_weight(dh, agg, x)
        dx = None
        if ctx.needs_input_grad[0]:
            if graph.t_rowptr is None:
                raise RuntimeError("SageGraph was built without its transpose; rebuild with "
                                   "transpose=True for backward")
            # [dAgg/deg | dx_root] in one MFMA pass, then the transpose gather
            # adds the root-path gradient as it sums over out-edges.
            g, dx_r = dense.sage_linear_bwd_data(dh, wl, wr, graph.rowptr, wcat=ctx.wcat)
            dx = ops.gather_rows(g, graph.t_rowptr, graph.t_col, x.size(0), mean=False,
                                 order=graph.t_order, hub=graph.t_hub,
                                 addend=dx_r, name="gather_bwd")
        return (dx, dwl.to(wl.dtype), dbl.to(wl.dtype), dwr.to(wr.dtype),
                dgamma.to(gamma.dtype), dbeta.to(beta.dtype), None, None, None, None, None)


# Training runs the stack as one autograd node with fused layer boundaries
# (_SageStackFn); False (or SLDM_FUSE_BOUNDARIES=0) selects one node per layer
# (_SageLayerFn) -- same results, for A/B comparisons and the tests.
FUSE_BOUNDARIES = __import__("os").environ.get("SLDM_FUSE_BOUNDARIES", "1") != "0"
# Opt-in (SLDM_OVERLAP_DW=1): weight gradients (dW = dh^T [agg | h]) on a side
# stream, concurrent with the same layer's dX GEMM and transpose gather.  At C4
# it measured 70.0-70.5 vs 70.5-71.2 ms/step in the same call, and one of two
# runs took 168 ms/step (the caching allocator holding the cross-stream blocks
# of 5-GB tensors) -- not worth the risk as the default.
OVERLAP_DW = __import__("os").environ.get("SLDM_OVERLAP_DW", "0") == "1"
_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device):
    st = _SIDE_STREAMS.get(dev.index)
    if st is None:
        st = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(dev)
    return st


class _SageStackFn(torch.autograd.Function):
    """All layers of a SageBlock as one autograd node, so the backward can fuse
    each layer boundary: the transpose gather of layer l and the LayerNorm /
    act / dropout backward of layer l-1 run as one kernel (gather_post.hip)
    and the input gradient of layer l never reaches HBM.  Forward and every
    per-layer operation are those of :class:`_SageLayerFn`; the results are
    bit-identical to it (dh from the fused kernel equals post_bwd of the
    gathered gradient; only the fp32 column sums of dgamma / dbeta / dbias are
    summed in a different row order)."""

    @staticmethod
    def forward(ctx, x, graph: SageGraph, cfgs, *params):
        n = x.size(0)
        saved, wcats = [], []
        h = x
        for i, (slope, drop_p, seed, eps) in enumerate(cfgs):
            wl, bl, wr, gamma, beta = params[5 * i: 5 * i + 5]
            agg = ops.gather_rows(h, graph.rowptr, graph.col, n, mean=True, name="gather_fwd",
                                  order=graph.order, hub=graph.hub)
            wcat = dense.weight_cat(wl, wr, h.dtype)
            out, xhat, rstd = dense.sage_layer_fwd(agg, h, wl, bl, wr, gamma, beta, eps, slope,
                                                   drop_p, seed, save=True, wcat=wcat)
            saved += [h, agg, xhat, rstd]
            wcats.append(wcat)
            h = out
        ctx.save_for_backward(*saved, *params)
        ctx.wcats = wcats
        ctx.graph, ctx.cfgs, ctx.nl = graph, cfgs, len(cfgs)
        return h

    @staticmethod
    def backward(ctx, dout):
        nl, graph, cfgs = ctx.nl, ctx.graph, ctx.cfgs
        st = ctx.saved_tensors
        acts, params = st[: 4 * nl], st[4 * nl:]
        if graph.t_rowptr is None:
            raise RuntimeError("SageGraph was built without its transpose; rebuild with "
                               "transpose=True for backward")
        grads = [None] * len(params)
        x_in = acts[0]
        top = nl - 1
        slope, drop_p, seed, _ = cfgs[top]
        wl, bl, wr, gamma, beta = params[5 * top: 5 * top + 5]
        dh, dgamma, dbeta, dbl = ops.post_bwd(dout, acts[4 * top + 2], acts[4 * top + 3], gamma,
                                              beta, slope, drop_p, seed, dh_dtype=x_in.dtype)
        dx = None
        main = torch.cuda.current_stream(dh.device)
        side = _side_stream(dh.device) if OVERLAP_DW else None
        side_out = []
        for i in range(top, -1, -1):
            h, agg = acts[4 * i], acts[4 * i + 1]
            wl, bl, wr, gamma, beta = params[5 * i: 5 * i + 5]
            if side is not None:
                # inputs produced on the main stream; the caching allocator must
                # not hand their blocks to main-stream allocations until the
                # side stream is done with them (record_stream)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    dwl, dwr = dense.sage_linear_bwd_weight(dh, agg, h)
                    dwl, dwr = dwl.to(wl.dtype), dwr.to(wr.dtype)
                for t in (dh, agg, h):
                    t.record_stream(side)
                side_out += [dwl, dwr]
            else:
                dwl, dwr = dense.sage_linear_bwd_weight(dh, agg, h)
                dwl, dwr = dwl.to(wl.dtype), dwr.to(wr.dtype)
            grads[5 * i: 5 * i + 5] = [dwl, dbl.to(wl.dtype), dwr, dgamma.to(gamma.dtype),
                                       dbeta.to(beta.dtype)]
            if i == 0 and not ctx.needs_input_grad[0]:
                break
            g, dx_r = dense.sage_linear_bwd_data(dh, wl, wr, graph.rowptr, wcat=ctx.wcats[i])
            if i == 0:
                dx = ops.gather_rows(g, graph.t_rowptr, graph.t_col, h.size(0), mean=False,
                                     order=graph.t_order, hub=graph.t_hub, addend=dx_r, name="gather_bwd")
                break
            # boundary: layer i's input gradient straight into layer i-1's post backward
            slope, drop_p, seed, _ = cfgs[i - 1]
            gamma_b, beta_b = params[5 * (i - 1) + 3], params[5 * (i - 1) + 4]
            if graph.t_hub is not None:
                # out-degree hubs: the split transpose gather, then the post
                # backward (the fused kernel sums each row in one row group)
                dxi = ops.gather_rows(g, graph.t_rowptr, graph.t_col, h.size(0), mean=False,
                                      hub=graph.t_hub, addend=dx_r, name="gather_bwd")
                dh, dgamma, dbeta, dbl = ops.post_bwd(
                    dxi, acts[4 * (i - 1) + 2], acts[4 * (i - 1) + 3], gamma_b, beta_b, slope,
                    drop_p, seed, dh_dtype=x_in.dtype)
                continue
            dh, dgamma, dbeta, dbl = ops.gather_post_bwd(
                g, graph.t_rowptr, graph.t_col, graph.t_order, dx_r, acts[4 * (i - 1) + 2],
                acts[4 * (i - 1) + 3], gamma_b, beta_b, slope, drop_p, seed)
        if side is not None:
            # the weight grads are consumed on the main stream after this returns
            main.wait_stream(side)
            for t in side_out:
                t.record_stream(main)
        return (dx, None, None, *grads)


class SageConv(nn.Module):
    """Parameter layout of PyG 2.7.0 ``SAGEConv(in, out)`` with default arguments
    (aggr='mean', root_weight=True, bias=True, normalize=False, project=False),
    as instantiated at sageblock.py:8: ``lin_l`` (with bias) on the mean
    aggregate, ``lin_r`` (no bias) on the root features."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin_l = nn.Linear(in_channels, out_channels, bias=True)
        self.lin_r = nn.Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self) -> None:
        self.lin_l.reset_parameters()
        self.lin_r.reset_parameters()

    def forward(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        """Stand-alone conv (no post stack): lin_l(mean_j x_j) + lin_r(x)."""
        graph = get_graph(edge_index, x.size(0), transpose=torch.is_grad_enabled())
        agg = _MeanAggFn.apply(x, graph)
        out = nn.functional.linear(agg.to(self.lin_l.weight.dtype), self.lin_l.weight,
                                   self.lin_l.bias)
        return out + nn.functional.linear(x.to(self.lin_r.weight.dtype), self.lin_r.weight)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, aggr=mean)"


class _MeanAggFn(torch.autograd.Function):
    """Mean neighbour aggregation alone (PyG propagate + MeanAggregation)."""

    @staticmethod
    def forward(ctx, x, graph: SageGraph):
        ctx.graph = graph
        ctx.n = x.size(0)
        return ops.gather_rows(x, graph.rowptr, graph.col, x.size(0), mean=True, order=graph.order, hub=graph.hub,
                               name="gather_fwd")

    @staticmethod
    def backward(ctx, g):
        graph = ctx.graph
        g = g.contiguous().clone()
        ops.scale_rows_by_inv_deg_(g, graph.rowptr)
        return ops.gather_rows(g, graph.t_rowptr, graph.t_col, ctx.n, mean=False, order=graph.t_order, hub=graph.t_hub,
                               name="gather_bwd"), None


def sage_aggregate(x: torch.Tensor, edge_index) -> torch.Tensor:
    """Mean aggregation over in-edges (differentiable)."""
    graph = get_graph(edge_index, x.size(0), transpose=torch.is_grad_enabled())
    return _MeanAggFn.apply(x, graph)


class SageBlock(nn.Module):
    """Drop-in for src/models/blocks/sageblock.py:4-20 (same signature, same
    state_dict).  ``edge_index`` may also be a prebuilt :class:`SageGraph`."""

    def __init__(self, hdims: list[int], dropout: float | None = None,
                 negative_slope: float | None = None):
        super().__init__()
        assert len(hdims) >= 1, "hdims must contain at least one element"
        self.convs = nn.ModuleList([SageConv(hdims[i], hdims[i + 1])
                                    for i in range(len(hdims) - 1)])
        self.posts = nn.ModuleList([
            nn.Sequential(
                nn.LayerNorm(hdims[i + 1]),
                nn.LeakyReLU(negative_slope=negative_slope) if negative_slope is not None else nn.ReLU(),
                nn.Dropout(p=dropout) if dropout is not None else nn.Identity(),
            ) for i in range(len(hdims) - 1)
        ])

    def forward(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        if len(self.convs) == 0:
            return x
        if x.dim() != 2:
            raise ValueError(f"SageBlock expects x [N, F], got {tuple(x.shape)}")
        if x.device.type == "cpu":
            return self._forward_cpu(x, edge_index)
        ops._require_gpu(x)
        grad = torch.is_grad_enabled() and (
            x.requires_grad or any(p.requires_grad for p in self.parameters()))
        graph = get_graph(edge_index, x.size(0), transpose=grad)
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        x = x.contiguous()
        layers = []
        for conv, post in zip(self.convs, self.posts):
            ln, act, drop = post[0], post[1], post[2]
            if not isinstance(ln, nn.LayerNorm) or ln.weight is None:
                raise TypeError("SageBlock post[0] must be an affine LayerNorm")
            p = _drop_p(drop)
            layers.append(((conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight, ln.weight,
                            ln.bias), (_act_slope(act), p, _new_seed(x.device) if p > 0 else 0,
                                       float(ln.eps))))
        if grad and FUSE_BOUNDARIES and ops.branch_source(x) is None:
            # training: one autograd node for the stack (fused layer boundaries)
            cfgs = tuple(c for _, c in layers)
            params = [t for w, _ in layers for t in w]
            return _SageStackFn.apply(x, graph, cfgs, *params)
        for (wl, bl, wr, gamma, beta), (slope, p, seed, eps) in layers:
            x = _SageLayerFn.apply(x, wl, bl, wr, gamma, beta, graph, slope, p, seed, eps)
        return x

    def _forward_cpu(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        """CPU tensors (the reference's DEVICE='cpu' mode): the host kernels of
        cpu.py, fp32 (the reference's dtype), one autograd node per layer."""
        from .cpu import _CpuLayerFn
        if x.dtype != torch.float32:
            raise TypeError(f"SageBlock on CPU computes in float32 (the reference's dtype), "
                            f"got {x.dtype}")
        if isinstance(edge_index, torch.Tensor) and edge_index.device.type != "cpu":
            raise RuntimeError("SageBlock: x is on the CPU but edge_index is on "
                               f"{edge_index.device}")
        grad = torch.is_grad_enabled() and (
            x.requires_grad or any(p.requires_grad for p in self.parameters()))
        graph = get_graph(edge_index, x.size(0), transpose=grad)
        x = x.contiguous()
        for conv, post in zip(self.convs, self.posts):
            ln, act, drop = post[0], post[1], post[2]
            p = _drop_p(drop)
            seed = _cpu_seed() if p > 0 else 0
            x = _CpuLayerFn.apply(x, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight,
                                  ln.weight, ln.bias, graph, _act_slope(act), p, seed,
                                  float(ln.eps))
        return x


def _cpu_seed() -> int:
    """Dropout key for a CPU-mode layer call, from torch's CPU generator (the
    generator nn.Dropout on CPU draws from), so torch.manual_seed governs it."""
    return int(torch.randint(0, 2**62, (1,)).item())
