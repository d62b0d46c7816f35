"""Drop-in ``GRU`` for the model's trajectory encoder.

GruSage builds ``torch.nn.GRU(input_size=dynamic_features_num,
hidden_size=gru_hidden_size, num_layers=gru_num_layers, batch_first=True)``
(/root/reference/src/models/grusage.py:66-71; main.py:22-54 sweeps a single
layer of 96 units over 6 features) and calls ``gru_out, hlast = self.gru(x)``
on ``x [N_vehicles, T=100, 6]`` (grusage.py:160-161).  torch runs that on
MIOpen at ~1 % of the fp32 MFMA peak (bench.py --config gru); this module
runs the recurrence on the hand-written gfx950 kernels of ``gru.hip``
(forward + backward through the C ABI), with nn.GRU's constructor, parameter
names (``weight_ih_l0`` ...), initialisation and ``forward(input, hx=None)``
contract, so GruSage's ``self.gru`` and its state_dict keys are unchanged.

Supported: one layer, unidirectional, fp32, ``1 <= input_size <= 16``,
``hidden_size`` a multiple of 16 up to 96, CUDA tensors.  Anything else
raises (no silent fallback to torch's GRU).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib
from .ops import _require_gpu, _stream


def supported(input_size: int, hidden_size: int, num_layers: int = 1,
              bidirectional: bool = False) -> bool:
    return (num_layers == 1 and not bidirectional and 1 <= input_size <= 16
            and 16 <= hidden_size <= 96 and hidden_size % 16 == 0)


def _ptr(t):
    return None if t is None else t.data_ptr()


class _GruFn(torch.autograd.Function):
    last_backward_had_dout: bool | None = None

    @staticmethod
    def forward(ctx, x, h0, w_ih, w_hh, b_ih, b_hh, batch_first: bool):
        dev = _require_gpu(x, h0, w_ih, w_hh, b_ih, b_hh)
        # an output nobody differentiates (GruSage reads only hlast,
        # grusage.py:160-161) reaches backward as None, not as an [N, T, H]
        # tensor of zeros the kernel would stream every step
        ctx.set_materialize_grads(False)
        for name, t in (("input", x), ("h0", h0), ("weight", w_ih), ("weight", w_hh),
                        ("bias", b_ih), ("bias", b_hh)):
            if t is not None and t.dtype != torch.float32:
                raise TypeError(f"sldm_sage.GRU: {name} must be float32, got {t.dtype}")
        if x.stride(-1) != 1:
            x = x.contiguous()
        if batch_first:
            N, T, I = x.shape
            ldxn, ldxt = x.stride(0), x.stride(1)
        else:
            T, N, I = x.shape
            ldxn, ldxt = x.stride(1), x.stride(0)
        H = w_hh.size(1)
        out = torch.empty((N, T, H) if batch_first else (T, N, H), dtype=torch.float32,
                          device=dev)
        ldon, ldot = (out.stride(0), out.stride(1)) if batch_first else (out.stride(1),
                                                                        out.stride(0))
        h_n = torch.empty(1, N, H, dtype=torch.float32, device=dev)
        lib = _lib.load()
        need = any(ctx.needs_input_grad[:6])      # (grad mode is off inside forward)
        gates = None
        if need:
            gates = torch.empty(lib.sldm_gru_workspace_bytes(N, T, H) // 4,
                                dtype=torch.float32, device=dev)
        h0c = h0.reshape(N, H).contiguous() if h0 is not None else None
        w_ih_c, w_hh_c = w_ih.contiguous(), w_hh.contiguous()
        b_ih_c = b_ih.contiguous() if b_ih is not None else None
        b_hh_c = b_hh.contiguous() if b_hh is not None else None
        _lib.check(lib.sldm_gru_fwd(x.data_ptr(), ldxn, ldxt, N, T, I, H, w_ih_c.data_ptr(),
                                    w_hh_c.data_ptr(), _ptr(b_ih_c), _ptr(b_hh_c), _ptr(h0c),
                                    out.data_ptr(), ldon, ldot, h_n.data_ptr(), _ptr(gates),
                                    _stream(dev)), "sldm_gru_fwd")
        if need:
            ctx.save_for_backward(x, h0c, w_ih_c, w_hh_c, out, gates)
            ctx.cfg = (batch_first, N, T, I, H, (ldxn, ldxt), (ldon, ldot),
                       b_ih is not None, b_hh is not None)
        return out, h_n

    @staticmethod
    def backward(ctx, dout, dh_n):
        x, h0c, w_ih, w_hh, out, gates = ctx.saved_tensors
        batch_first, N, T, I, H, (ldxn, ldxt), (ldon, ldot), has_bih, has_bhh = ctx.cfg
        dev = x.device
        lib = _lib.load()
        _GruFn.last_backward_had_dout = dout is not None     # observed by the tests
        if dout is not None:
            dout = dout if dout.stride(-1) == 1 else dout.contiguous()
            lddn, lddt = (dout.stride(0), dout.stride(1)) if batch_first else (dout.stride(1),
                                                                              dout.stride(0))
        else:
            lddn = lddt = 0
        dhn = dh_n.reshape(N, H).contiguous() if dh_n is not None else None
        need_dx = ctx.needs_input_grad[0]
        dx = torch.empty_like(x) if need_dx else None
        if need_dx:
            lddxn, lddxt = (dx.stride(0), dx.stride(1)) if batch_first else (dx.stride(1),
                                                                            dx.stride(0))
        else:
            lddxn = lddxt = 0
        dh0 = (torch.empty(1, N, H, dtype=torch.float32, device=dev)
               if ctx.needs_input_grad[1] else None)
        dw_ih = torch.empty_like(w_ih)
        dw_hh = torch.empty_like(w_hh)
        db_ih = torch.empty(3 * H, dtype=torch.float32, device=dev) if has_bih else None
        db_hh = torch.empty(3 * H, dtype=torch.float32, device=dev) if has_bhh else None
        ws_bytes = lib.sldm_gru_bwd_workspace_bytes(N, T, I, H, int(need_dx))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.check(lib.sldm_gru_bwd(
            x.data_ptr(), ldxn, ldxt, N, T, I, H, w_ih.data_ptr(), w_hh.data_ptr(), _ptr(h0c),
            out.data_ptr(), ldon, ldot, gates.data_ptr(), _ptr(dout), lddn, lddt, _ptr(dhn),
            _ptr(dx), lddxn, lddxt, _ptr(dh0), dw_ih.data_ptr(), dw_hh.data_ptr(), _ptr(db_ih),
            _ptr(db_hh), ws.data_ptr(), ws_bytes, _stream(dev)), "sldm_gru_bwd")
        return dx, dh0, dw_ih, dw_hh, db_ih, db_hh, None


class GRU(nn.Module):
    """``torch.nn.GRU`` (single layer, unidirectional, fp32) on gfx950 kernels."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1,
                 bias: bool = True, batch_first: bool = False, dropout: float = 0.0,
                 bidirectional: bool = False, device=None, dtype=None):
        super().__init__()
        if not supported(input_size, hidden_size, num_layers, bidirectional):
            raise ValueError(
                "sldm_sage.GRU supports one unidirectional layer with 1 <= input_size <= 16 "
                f"and hidden_size a multiple of 16 in [16, 96]; got input_size={input_size}, "
                f"hidden_size={hidden_size}, num_layers={num_layers}, "
                f"bidirectional={bidirectional}")
        if dtype is not None and dtype != torch.float32:
            raise TypeError("sldm_sage.GRU computes in float32")
        self.input_size, self.hidden_size = input_size, hidden_size
        self.num_layers, self.bias, self.batch_first = 1, bias, batch_first
        self.dropout, self.bidirectional = float(dropout), False
        fk = dict(device=device, dtype=torch.float32)
        self.weight_ih_l0 = nn.Parameter(torch.empty(3 * hidden_size, input_size, **fk))
        self.weight_hh_l0 = nn.Parameter(torch.empty(3 * hidden_size, hidden_size, **fk))
        if bias:
            self.bias_ih_l0 = nn.Parameter(torch.empty(3 * hidden_size, **fk))
            self.bias_hh_l0 = nn.Parameter(torch.empty(3 * hidden_size, **fk))
        else:
            self.register_parameter("bias_ih_l0", None)
            self.register_parameter("bias_hh_l0", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        """nn.GRU's initialisation: every parameter U(-1/sqrt(H), 1/sqrt(H))."""
        k = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -k, k)

    def forward(self, input: torch.Tensor, hx: torch.Tensor | None = None):
        unbatched = input.dim() == 2
        x = input.unsqueeze(0 if self.batch_first else 1) if unbatched else input
        if x.dim() != 3 or x.size(-1) != self.input_size:
            raise ValueError(f"GRU: expected input [.., .., {self.input_size}], "
                             f"got {tuple(input.shape)}")
        h0 = hx
        if hx is not None and unbatched:
            h0 = hx.unsqueeze(1)
        out, h_n = _GruFn.apply(x, h0, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0,
                                self.bias_hh_l0, self.batch_first)
        if unbatched:
            return out.squeeze(0 if self.batch_first else 1), h_n.squeeze(1)
        return out, h_n

    def extra_repr(self) -> str:
        s = f"{self.input_size}, {self.hidden_size}"
        if not self.bias:
            s += ", bias=False"
        if self.batch_first:
            s += ", batch_first=True"
        return s
