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
one PyTorch custom operator (torch.ops.sldm.sage_layer; in training the whole
stack as sage_stack_fwd / sage_stack_bwd) over the C ABI:
  forward : gather-mean over CSR-by-dst -> [agg|x]·[W_l|W_r]^T -> bias+LN+act+dropout
  backward: LN/act/dropout bwd -> dh·[W_l|W_r] -> dW -> 1/deg prescale ->
            transpose gather + lin_r grad
Dropout masks come from a counter-based hash (not torch's RNG stream), so
parity runs use eval mode or dropout=None.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops, torch_ops
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


# Training runs the stack as one autograd node with fused layer boundaries
# (_SageStackFn); False (or SLDM_FUSE_BOUNDARIES=0) runs one differentiable
# operator per layer (torch.ops.sldm.sage_layer) -- same results, for A/B
# comparisons and the tests.
FUSE_BOUNDARIES = __import__("os").environ.get("SLDM_FUSE_BOUNDARIES", "1") != "0"


def sage_layer(x, graph: SageGraph, wl, bl, wr, gamma, beta, slope: float, drop_p: float,
               seed: int, eps: float) -> torch.Tensor:
    """One SageBlock layer, SAGEConv(mean) -> LayerNorm -> act -> dropout, as
    the dispatcher operator ``torch.ops.sldm.sage_layer`` (differentiable:
    its backward is registered with torch.library.register_autograd; ROCm and
    CPU tensors take their own kernels)."""
    sldm = torch_ops.load()
    gl, gm = graph.packed()
    save = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (x, wl, bl, wr, gamma, beta))
    return sldm.sage_layer(x, gl, gm, wl, bl, wr, gamma, beta, slope, drop_p, seed, eps, save)[0]


class _SageStackFn(torch.autograd.Function):
    """All layers of a SageBlock as one autograd node over two operators,
    ``torch.ops.sldm.sage_stack_fwd`` / ``sage_stack_bwd`` (one C++ call per
    direction), so the backward can fuse each layer boundary: the transpose
    gather of layer l and the LayerNorm / act / dropout backward of layer l-1
    run as one kernel (gather_post.hip) and the input gradient of layer l
    never reaches HBM.  Results are bit-identical to the per-layer operator
    (dh from the fused kernel equals post_bwd of the gathered gradient; only
    the fp32 column sums of dgamma / dbeta / dbias are summed in a different
    row order)."""

    @staticmethod
    def forward(ctx, x, graph: SageGraph, cfgs, seed_word, *params):
        sldm = torch_ops.load()
        gl, gm = graph.packed()
        slopes = [c[0] for c in cfgs]
        drops = [c[1] for c in cfgs]
        seeds = [c[2] for c in cfgs]
        eps = [c[3] for c in cfgs]
        with ops.dropout_seed_source(seed_word):
            res = sldm.sage_stack_fwd(x, gl, gm, params, slopes, drops, seeds, eps, True)
        ctx.save_for_backward(*res[1:], *params)
        ctx.graph, ctx.cfg, ctx.nl = graph, (slopes, drops, seeds), len(cfgs)
        ctx.seed_word = seed_word
        return res[0]

    @staticmethod
    def backward(ctx, dout):
        nl = ctx.nl
        st = ctx.saved_tensors
        saved, params = st[: 4 * nl], st[4 * nl:]
        slopes, drops, seeds = ctx.cfg
        gl, gm = ctx.graph.packed()
        need_dx = ctx.needs_input_grad[0]
        with ops.dropout_seed_source(ctx.seed_word):
            grads = torch.ops.sldm.sage_stack_bwd(dout, saved, gl, gm, params, slopes, drops,
                                                  seeds, need_dx, True)
        return (grads[0] if need_dx else None, None, None, None, *grads[1:])


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
        agg = sage_aggregate(x, edge_index)
        if x.device.type == "cuda":
            # the library's MFMA GEMMs, in x's storage dtype (fp32 or bf16) with fp32
            # accumulation, like the SageBlock's fused layers
            from .dense import SageLinearFn
            xs = x if x.dtype in (torch.float32, torch.bfloat16) else x.float()
            return SageLinearFn.apply(agg.to(xs.dtype), xs, self.lin_l.weight, self.lin_l.bias,
                                      self.lin_r.weight)
        out = nn.functional.linear(agg.to(self.lin_l.weight.dtype), self.lin_l.weight,
                                   self.lin_l.bias)
        return out + nn.functional.linear(x.to(self.lin_r.weight.dtype), self.lin_r.weight)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, aggr=mean)"


def sage_aggregate(x: torch.Tensor, edge_index) -> torch.Tensor:
    """Mean aggregation over in-edges (PyG propagate + MeanAggregation),
    differentiable: ``torch.ops.sldm.mean_aggregate``."""
    graph = get_graph(edge_index, x.size(0), transpose=torch.is_grad_enabled())
    gl, gm = graph.packed()
    if x.device.type == "cuda" and x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return torch_ops.load().mean_aggregate(x, gl, gm)


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
        drops = any(_drop_p(post[2]) > 0 for post in self.posts)
        # Recorded into a HIP graph, a host seed would freeze one mask into every
        # replay: the call's seed is then a device word (the device's capture
        # counter, advanced by a recorded launch) that the kernels add to the
        # layer index at run time.
        seed_word = None
        if drops and torch.cuda.is_current_stream_capturing():
            if not (grad and FUSE_BOUNDARIES):
                raise RuntimeError("SageBlock: dropout under HIP graph capture runs on the fused "
                                   "training stack only (grad enabled, SLDM_FUSE_BOUNDARIES on)")
            seed_word = ops.next_capture_seed(x.device)
        elif drops and grad:
            ops.capture_seed_counter(x.device)      # exists before any capture begins
        layers = []
        for conv, post in zip(self.convs, self.posts):
            ln, act, drop = post[0], post[1], post[2]
            if not isinstance(ln, nn.LayerNorm) or ln.weight is None:
                raise TypeError("SageBlock post[0] must be an affine LayerNorm")
            p = _drop_p(drop)
            seed = 0 if p <= 0 else (len(layers) if seed_word is not None
                                     else _new_seed(x.device))
            layers.append(((conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight, ln.weight,
                            ln.bias), (_act_slope(act), p, seed, float(ln.eps))))
        if grad and FUSE_BOUNDARIES:
            # training: one autograd node for the stack (fused layer boundaries)
            cfgs = tuple(c for _, c in layers)
            params = [t for w, _ in layers for t in w]
            return _SageStackFn.apply(x, graph, cfgs, seed_word, *params)
        for (wl, bl, wr, gamma, beta), (slope, p, seed, eps) in layers:
            x = sage_layer(x, graph, wl, bl, wr, gamma, beta, slope, p, seed, eps)
        return x

    def _forward_cpu(self, x: torch.Tensor, edge_index) -> torch.Tensor:
        """CPU tensors (the reference's DEVICE='cpu' mode): the same operator,
        dispatched to the host kernels of cpu.py; fp32 (the reference's
        dtype), one differentiable operator call per layer."""
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
            x = sage_layer(x, graph, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight,
                           ln.weight, ln.bias, _act_slope(act), p, seed, float(ln.eps))
        return x


def _cpu_seed() -> int:
    """Dropout key for a CPU-mode layer call, from torch's CPU generator (the
    generator nn.Dropout on CPU draws from), so torch.manual_seed governs it."""
    return int(torch.randint(0, 2**62, (1,)).item())
