"""ctypes binding of libsldm_sage.so (the C ABI in include/sldm_sage.h).

The library is loaded after ``torch`` so that it binds to the HIP runtime
torch already loaded (both carry the soname libamdhip64.so.7).  There is no
fallback: if the library is missing or cannot be loaded, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SLDM_SAGE_LIB", os.path.join(_HERE, "libsldm_sage.so"))

ABI_VERSION = 9
F32, BF16 = 0, 1

_c_i64 = ctypes.c_int64
_c_i32p = ctypes.c_void_p
_vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/sldm_sage.h
_SIGNATURES = {
    "sldm_abi_version": (ctypes.c_int, []),
    "sldm_last_error": (ctypes.c_char_p, []),
    "sldm_set_dropout_seed_source": (None, [ctypes.c_void_p]),
    "sldm_csr_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "sldm_csr_build": (ctypes.c_int, [_vp, ctypes.c_int, _c_i64, _c_i64, _vp, _vp, _vp, _vp,
                                      _vp, _vp, ctypes.c_size_t, _vp]),
    "sldm_degree_order_workspace_bytes": (ctypes.c_size_t, [_c_i64]),
    "sldm_degree_order": (ctypes.c_int, [_vp, _c_i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "sldm_gather_rows": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _vp, _c_i64, _c_i64,
                                        ctypes.c_int, _vp, _c_i64, ctypes.c_int, _vp, _c_i64,
                                        _vp]),
    "sldm_gather_rows_split": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _vp, _c_i64,
                                              _c_i64, ctypes.c_int, _vp, _c_i64, ctypes.c_int,
                                              _vp, _c_i64, _vp, _vp, _c_i64, _vp, _vp, _c_i64,
                                              ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "sldm_gather_rows_split_static_max_floats": (ctypes.c_size_t, []),
    "sldm_gather_rows_split_static": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _vp,
                                                     _c_i64, _c_i64, ctypes.c_int, _vp, _c_i64,
                                                     ctypes.c_int, _vp, _c_i64, _vp, _vp, _c_i64,
                                                     _vp, _vp, _c_i64, ctypes.c_int32,
                                                     ctypes.c_int32, _vp]),
    "sldm_scale_rows_by_inv_deg": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _c_i64,
                                                  _c_i64, _vp]),
    "sldm_post_fwd": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp,
                                     ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_uint64, _c_i64, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "sldm_post_bwd": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp,
                                     ctypes.c_float, ctypes.c_float, ctypes.c_uint64, _c_i64,
                                     ctypes.c_int, _vp, _vp, ctypes.c_int, _vp]),
    "sldm_post_num_partials": (ctypes.c_int, [_c_i64, _c_i64]),
    "sldm_colsum": (ctypes.c_int, [_vp, ctypes.c_int, _c_i64, _vp, _vp]),
    "sldm_sage_dense_fwd": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _vp, _c_i64,
                                           _c_i64, _vp, _c_i64, _c_i64, _vp, _vp, _vp,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_uint64, _c_i64, _vp, _vp, _vp, _vp]),
    "sldm_gemm_nt_rowscale": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _vp, _c_i64,
                                             _c_i64, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp,
                                             _c_i64, _vp]),
    "sldm_gemm_nt_rowscale_blocked_ok": (ctypes.c_int, [ctypes.c_int, _c_i64, _c_i64, _c_i64,
                                                        _c_i64]),
    "sldm_gemm_nt_rowscale_blocked": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _vp,
                                                     _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp,
                                                     _c_i64, _vp, _c_i64, _vp]),
    "sldm_gemm_tn_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i64]),
    "sldm_gemm_tn": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64,
                                    _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, ctypes.c_size_t,
                                    _vp]),
    "sldm_gemm_tn_split": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _vp, _c_i64,
                                          _c_i64, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp,
                                          ctypes.c_size_t, _vp]),
    "sldm_gather_post_bwd_num_partials": (ctypes.c_int, [_c_i64, _c_i64]),
    "sldm_gather_post_bwd": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _vp, _vp, _c_i64,
                                            _c_i64, _c_i64, _vp, _vp, _vp, _vp, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_uint64, _c_i64, _vp, _vp,
                                            ctypes.c_int, _vp]),
    "sldm_cols_pack": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp,
                                      _vp]),
    "sldm_cols_unpack": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64,
                                        _vp, _c_i64, _vp]),
    "sldm_segment_pool_piece_rows": (ctypes.c_int, []),
    "sldm_segment_pool_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_i64]),
    "sldm_segment_pool": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _c_i64, _vp,
                                         _c_i64, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _vp,
                                         _vp, ctypes.c_size_t, _vp]),
    "sldm_segment_pool_bwd": (ctypes.c_int, [ctypes.c_int, _vp, _c_i64, _vp, _vp, _c_i64, _c_i64,
                                             _vp, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _vp,
                                             _vp, _c_i64, _vp]),
    "sldm_batch_graphs_max_nodes": (ctypes.c_int, []),
    "sldm_batch_graphs": (ctypes.c_int, [_c_i64, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp,
                                         _vp, _vp, _vp, _vp, _vp]),
    "sldm_radius_edges_workspace_bytes": (ctypes.c_size_t, [_c_i64]),
    "sldm_radius_edges": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _c_i64,
                                         _c_i64, _c_i64, ctypes.c_float, _vp, _c_i64, _vp, _vp,
                                         _vp, ctypes.c_size_t, _vp]),
    "sldm_gru_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i64]),
    "sldm_gru_fwd": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp]),
    "sldm_gru_bwd_workspace_bytes": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i64, _c_i64,
                                                       ctypes.c_int]),
    "sldm_gru_bwd": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _vp,
                                    _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_i64, _c_i64,
                                    _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                    ctypes.c_size_t, _vp]),
}

_lock = threading.Lock()
_lib = None
_load_error: str | None = None


class SldmError(RuntimeError):
    """A C-ABI call of libsldm_sage.so failed."""


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raise if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            _load_error = (f"libsldm_sage.so not found at {LIB_PATH}: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` or "
                           "`make -C sldm-gnn_amd/csrc`")
            raise SldmError(_load_error)
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.sldm_abi_version()
        if ver != ABI_VERSION:
            raise SldmError(f"libsldm_sage.so ABI {ver} != expected {ABI_VERSION}: rebuild")
        _lib = lib
        return lib


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sldm_last_error().decode(errors="replace")
        raise SldmError(f"{what} failed (status {rc}): {msg}")
