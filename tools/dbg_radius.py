"""Debug helper: GPU radius edges vs the oracle on one test pack (diagnostic)."""
import sys
sys.path[:0] = ['/root/repo', '/root/repo/sldm-gnn_amd', '/root/repo/tests']
import torch  # noqa: E402
from test_gbuild import _pack  # noqa: E402
from oracle.gbuild_ref import radius_edges as ref  # noqa: E402
from sldm_sage.gbuild import radius_edges_from_x  # noqa: E402
v, t, grid, r = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1", float(sys.argv[4])
x = _pack(v, t, seed=v * 1000 + t, grid=grid)
print(x)
ei_r, ea_r = ref(x, r)
ei_g, ea_g = radius_edges_from_x(x.cuda(), r)
print("ref", ei_r.tolist(), ea_r.tolist())
print("gpu", ei_g.cpu().tolist(), ea_g.cpu().tolist())
