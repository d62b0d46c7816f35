"""Drop-in replacement for the reference's src/models/blocks/sageblock.py.

Copy this file over src/models/blocks/sageblock.py (or put it first on the
import path) with ``sldm-gnn_amd`` on PYTHONPATH; GruSage (grusage.py:7) and
MapEncoder (mapencoder.py:4) then build the MI355X-native SageBlock with the
same constructor, forward(x, edge_index) and state_dict keys.
"""
from sldm_sage import SageBlock  # noqa: F401

__all__ = ["SageBlock"]
