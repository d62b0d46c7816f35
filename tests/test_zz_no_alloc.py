"""The no-allocation entry point, sldm_gather_rows_split_static, through the
C ABI: its output must equal sldm_gather_rows_split's bit for bit (both sum
the same chunks in the same order; only where the fp32 chunk partials live
differs), on two calls in a row, the second with a smaller input -- the
static scratch keeps the first call's contents, which must not leak into the
second.  Sizes beyond the static scratch are rejected with a clear error.
"""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _powerlaw_graph(n, e, a=0.47, seed=7):
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(e, generator=g, dtype=torch.float64)
    b = 1.0 - a
    rank = ((1.0 + u * (n ** b - 1.0)) ** (1.0 / b)).floor().long().clamp(1, n) - 1
    dst = torch.randperm(n, generator=g)[rank]
    src = torch.randint(0, n, (e,), generator=g)
    return torch.stack([src, dst])


def _static_call(lib, x, g, hub, mean, addend, out):
    from sldm_sage import _lib, ops
    n, f = out.shape
    rc = lib.sldm_gather_rows_split_static(
        ops.dtype_code(x), x.data_ptr(), x.stride(0), g.rowptr.data_ptr(), g.col.data_ptr(), None,
        n, f, int(mean), None if addend is None else addend.data_ptr(),
        0 if addend is None else addend.stride(0), ops.dtype_code(out), out.data_ptr(),
        out.stride(0), hub.hub_rows.data_ptr(), hub.chunk_ptr.data_ptr(), hub.num_hubs,
        hub.chunk_row.data_ptr(), hub.chunk_beg.data_ptr(), hub.num_chunks, hub.chunk_len,
        hub.max_deg, torch.cuda.current_stream().cuda_stream)
    return rc, _lib


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_static_split_gather_equals_workspace_variant(dtype):
    from sldm_sage import _lib, build_graph, ops
    from sldm_sage.graph import hub_plan
    lib = _lib.load()
    torch.cuda.set_device(0)
    # first call large, second smaller (fewer rows, chunks and features)
    for n, e, f, thr, mean in [(20_000, 300_000, 256, 64, True), (3_000, 40_000, 64, 32, False)]:
        ei = _powerlaw_graph(n, e, seed=n)
        gen = torch.Generator().manual_seed(f)
        x = torch.randn(n, f, generator=gen).to(dtype).to(DEV)
        add = None if mean else torch.randn(n, f, generator=gen).to(dtype).to(DEV)
        g = build_graph(ei.to(DEV), n)
        hub = hub_plan(g.rowptr, thr)
        assert hub is not None and hub.num_chunks > hub.num_hubs > 0
        ref = ops.gather_rows(x, g.rowptr, g.col, n, mean=mean, addend=add, hub=hub)
        out = torch.full_like(ref, float("nan"))
        rc, _ = _static_call(lib, x, g, hub, mean, add, out)
        _lib.check(rc, "sldm_gather_rows_split_static")
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (n, f, dtype)


def test_static_split_gather_rejects_oversize():
    from sldm_sage import _lib, build_graph, ops
    from sldm_sage.graph import HubPlan, hub_plan
    lib = _lib.load()
    cap = lib.sldm_gather_rows_split_static_max_floats()
    assert cap == 4 << 20
    n, e, f = 3_000, 40_000, 64
    ei = _powerlaw_graph(n, e, seed=n)
    x = torch.randn(n, f).to(DEV)
    g = build_graph(ei.to(DEV), n)
    hub = hub_plan(g.rowptr, 32)
    big = HubPlan(hub.hub_rows, hub.chunk_ptr, hub.chunk_row, hub.chunk_beg, hub.num_hubs,
                  cap // f + 1, hub.chunk_len, hub.max_deg)
    out = torch.zeros(n, f, device=DEV)
    rc, _ = _static_call(lib, x, g, big, True, None, out)       # rejected before any launch
    assert rc == 1
    msg = lib.sldm_last_error().decode()
    assert "exceed the static scratch" in msg
    with pytest.raises(_lib.SldmError):
        _lib.check(rc, "sldm_gather_rows_split_static")
    assert ops.gather_rows(x, g.rowptr, g.col, n, mean=True, hub=hub).shape == (n, f)
