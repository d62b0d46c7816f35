"""CPU tests: the C-ABI library loads and exports every declared symbol, and the
Python module mirrors the reference's SageBlock API (no compute calls)."""
from __future__ import annotations

import os
import re

import pytest
import torch

from _helpers import ROOT


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "sldm_sage.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(sldm_[a-z0-9_]+)\s*\(", hdr)))


def test_library_loads_and_exports_header():
    import ctypes

    from sldm_sage import _lib
    lib = _lib.load()
    declared = _declared_symbols()
    assert len(declared) >= 9
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/sldm_sage.h but not exported"
        assert name in _lib.exported_symbols(), f"{name} has no ctypes signature"
    assert lib.sldm_abi_version() == _lib.ABI_VERSION
    assert isinstance(lib.sldm_last_error(), bytes)
    # host-only entry points (no device work)
    assert lib.sldm_csr_workspace_bytes(0, 10) > 0
    assert lib.sldm_post_num_partials(1000, 16) >= 1
    del ctypes


def test_error_reporting_without_gpu():
    """Argument validation fails before any device work and sets the message."""
    from sldm_sage import _lib
    lib = _lib.load()
    rc = lib.sldm_gather_rows(0, None, 16, None, None, None, 10, 16, 1, None, 0, 1, None, 16, None)
    assert rc != 0
    assert b"dtypes" in lib.sldm_last_error()
    with pytest.raises(_lib.SldmError):
        _lib.check(rc, "sldm_gather_rows")


def test_state_dict_layout_matches_reference():
    from oracle.sage_ref import RefSageBlock
    from sldm_sage import SageBlock
    for hd, p, ns in [([16, 32, 32], 0.25, 0.1), ([128, 96, 96], None, None), ([10, 8, 8], 0.1, 0.2),
                      ([8], None, None)]:
        a, b = SageBlock(hd, p, ns), RefSageBlock(hd, p, ns)
        sa = [(k, tuple(v.shape), v.dtype) for k, v in a.state_dict().items()]
        sb = [(k, tuple(v.shape), v.dtype) for k, v in b.state_dict().items()]
        assert sa == sb
        a.load_state_dict(b.state_dict(), strict=True)
        b.load_state_dict(a.state_dict(), strict=True)
        assert [n for n, _ in a.named_parameters()] == [n for n, _ in b.named_parameters()]
        # same submodule types at posts.{i}.{0,1,2}
        for pa, pb in zip(a.posts, b.posts):
            assert [type(m) for m in pa] == [type(m) for m in pb]


def test_gpu_ops_have_no_cpu_fallback(monkeypatch):
    """The GPU op layer rejects CPU tensors (no silent fallback); SageBlock sends
    CPU tensors explicitly to the native host library, and raises if that
    library is missing instead of falling back to torch."""
    from sldm_sage import SageBlock, cpu, ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gather_rows(torch.randn(3, 4), torch.zeros(4, dtype=torch.int32),
                        torch.zeros(0, dtype=torch.int32), 3, mean=True)
    monkeypatch.setattr(cpu, "CPU_LIB_PATH", "/nonexistent/libsldm_sage_cpu.so")
    monkeypatch.setattr(cpu, "_lib", None)
    blk = SageBlock([4, 4], None, 0.1)
    with pytest.raises(RuntimeError, match="libsldm_sage_cpu.so not found"):
        blk(torch.randn(3, 4), torch.tensor([[0, 1], [1, 2]]))


def test_identity_block_passthrough():
    from sldm_sage import SageBlock
    x = torch.randn(3, 4)
    assert SageBlock([4])(x, torch.empty(2, 0, dtype=torch.long)) is x


def test_dropin_module_importable():
    import importlib.util
    path = os.path.join(ROOT, "sldm-gnn_amd", "dropin", "src", "models", "blocks", "sageblock.py")
    spec = importlib.util.spec_from_file_location("dropin_sageblock", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from sldm_sage import SageBlock
    assert mod.SageBlock is SageBlock


def test_cpu_library_exports_header():
    """libsldm_sage_cpu.so (CPU-tensor path) exports every symbol its header declares."""
    from sldm_sage import cpu
    hdr = open(os.path.join(ROOT, "include", "sldm_sage_cpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = sorted(set(re.findall(r"\b(sldm_cpu_[a-z0-9_]+)\s*\(", hdr)))
    lib = cpu.load()
    assert len(declared) == 8
    for name in declared:
        assert hasattr(lib, name) and name in cpu.exported_symbols(), name
    assert lib.sldm_cpu_abi_version() == 2
