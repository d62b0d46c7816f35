"""Timing of the halo partition's pieces at the C4 size on one GPU (no
process group: the exchanges are skipped).  Diagnostic.
Usage: partition_probe.py [world] [graph kind] [concurrent processes]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from sldm_sage import dist as D  # noqa: E402


def t(label, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    print(f"[{os.environ.get('PROBE_CHILD', 0)}] {label:40s} {time.perf_counter() - t0:8.3f} s", flush=True)
    return r


def fp64_index_add(ei, n):
    w = torch.full((n,), 17.0, dtype=torch.float64, device=ei.device)
    ones = torch.ones(ei.size(1), dtype=torch.float64, device=ei.device)
    w.index_add_(0, ei[1], ones)
    w.index_add_(0, ei[0], ones)
    return w


n, e, f, L, dtype, _ = bench.CONFIGS["c4"]
dev = torch.device("cuda", 0)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
kind = sys.argv[2] if len(sys.argv) > 2 else "local"
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1
if P > 1 and "PROBE_CHILD" not in os.environ:
    import subprocess
    procs = [subprocess.Popen([sys.executable, "-u", __file__, str(W), kind, str(P)],
                              env=dict(os.environ, PROBE_CHILD=str(i))) for i in range(P)]
    sys.exit(max(p.wait() for p in procs))
ei, x = t("make_graph " + kind, lambda: bench.make_graph(n, e, f, dtype, dev, kind=kind))
t("fp64 index_add_ (old row_bounds)", lambda: fp64_index_add(ei, n))
bounds = t("row_bounds cost", lambda: D.row_bounds(ei, n, W, "cost"))
r0, r1 = bounds[0], bounds[1]
src, dst = ei[0], ei[1]
ein = t("ein mask", lambda: ei[:, (dst >= r0) & (dst < r1)])
eout = t("eout mask", lambda: ei[:, (src >= r0) & (src < r1)])
uniq = t("unique ein src", lambda: torch.unique(ein[0]))
remote = uniq[(uniq < r0) | (uniq >= r1)]
owner = t("owner", lambda: D._owner(remote, bounds))
t("bincount", lambda: torch.bincount(owner, minlength=W)[:W].tolist())
pos = t("searchsorted remap", lambda: torch.searchsorted(remote, ein[0]))
fin = t("stack fin", lambda: torch.stack([ein[0].long(), (ein[1] - r0).long()]))
t("estimate remote_unique", lambda: D._remote_unique(ein[0], r0, r1))
