"""sldm_sage — MI355X-native (gfx950) SageBlock hot path of aledima00/sldm-gnn.

Drop-in for ``src/models/blocks/sageblock.py``:

    from sldm_sage import SageBlock

Compute runs in libsldm_sage.so (hand-written HIP kernels behind the C ABI in
include/sldm_sage.h); there is no CPU fallback.
"""
from .graph import SageGraph, build_graph, get_graph, graph_cache
from .gru import GRU
from .pool import global_max_pool, global_mean_max_pool, global_mean_pool, global_pool
from .sageblock import SageBlock, SageConv, sage_aggregate

__all__ = ["SageBlock", "SageConv", "SageGraph", "build_graph", "get_graph", "graph_cache",
           "sage_aggregate", "global_mean_pool", "global_max_pool", "global_mean_max_pool",
           "global_pool", "GRU"]
__version__ = "0.1.0"
