"""Does a source-sharing row schedule buy the forward gather cache hits on a
uniform random graph?  Rows are processed in the order of their smallest
source id, so rows that share that source run next to each other and its
second and later reads hit L2 / the memory-side cache.  Times the C4-shape
bf16 gather (10 M rows, 100 M edges, F = 256) in natural order, in that
order, and in a random order (the cost of scattered output rows alone).

  python tools/order_probe.py [--nodes N] [--edges E]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sldm-gnn_amd"))
from sldm_sage import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--feat", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, e, f = args.nodes, args.edges, args.feat
    g = torch.Generator(device=dev).manual_seed(0)
    ei = torch.randint(0, n, (2, e), generator=g, device=dev, dtype=torch.int64)
    rowptr, col, _, _, bad = ops.csr_build(ei, n, transpose=False)
    assert int(bad) == 0
    del ei
    x = torch.randn(n, f, device=dev).to(torch.bfloat16)
    out = torch.empty_like(x)
    print(f"N={n} E={e} F={f}", flush=True)

    t = timed(lambda: ops.gather_rows(x, rowptr, col, n, True, out=out))
    print(f"natural order            {t:8.3f} ms", flush=True)
    ref = out.clone()

    # smallest source id of every row (rows without edges last)
    deg = (rowptr[1:] - rowptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    smin = torch.full((n,), n, dtype=torch.int64, device=dev)
    smin.scatter_reduce_(0, rows, col.long(), reduce="amin")
    del rows
    order = torch.argsort(smin, stable=True).to(torch.int32)
    groups = int(torch.unique(smin).numel())
    print(f"distinct smallest sources {groups} ({groups / n:.3f} of rows)", flush=True)
    out.zero_()
    t = timed(lambda: ops.gather_rows(x, rowptr, col, n, True, out=out, order=order))
    print(f"smallest-source order    {t:8.3f} ms  equal={torch.equal(out, ref)}", flush=True)

    perm = torch.randperm(n, device=dev, generator=g).to(torch.int32)
    out.zero_()
    t = timed(lambda: ops.gather_rows(x, rowptr, col, n, True, out=out, order=perm))
    print(f"random order             {t:8.3f} ms  equal={torch.equal(out, ref)}", flush=True)


if __name__ == "__main__":
    main()
