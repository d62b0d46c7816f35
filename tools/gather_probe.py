"""Probe: forward-gather rate vs table size and row width (uniform random graph).

    python tools/gather_probe.py

For a fixed edge count, times ``ops.gather_rows`` (mean, bf16) over tables of
different row counts (F fixed) and of different row widths (N fixed), so the
effect of the table's footprint (TLB / Infinity-Cache reach) can be told
apart from the effect of the row size.  Diagnostic only; prints one line per
case with algorithmic GB/s.
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]

import torch  # noqa: E402

from kbench import timeit  # noqa: E402


def case(n, e, f, reps=5):
    from sldm_sage import build_graph, ops
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    ei = torch.stack([torch.randint(0, n, (e,), generator=g, device=dev),
                      torch.randint(0, n, (e,), generator=g, device=dev)])
    x = torch.randn(n, f, device=dev, generator=g).to(torch.bfloat16)
    gr = build_graph(ei, n, transpose=False)
    del ei
    out = torch.empty(n, f, dtype=torch.bfloat16, device=dev)
    ms = timeit(lambda: ops.gather_rows(x, gr.rowptr, gr.col, n, True, out=out), reps)
    b = e * (4 + f * 2) + (n + 1) * 4 + n * f * 2
    print(f"N={n:>10} F={f:>4} row={f*2:>5}B table={n*f*2/2**30:6.2f}GiB E={e} "
          f"{ms:8.3f} ms {b/ms/1e6:8.1f} GB/s", flush=True)
    del x, gr, out
    torch.cuda.empty_cache()


def main():
    e = 100_000_000
    for n in (250_000, 500_000, 1_250_000, 2_500_000, 5_000_000, 10_000_000, 20_000_000):
        case(n, e, 256)
    for f in (32, 64, 128, 512):
        case(10_000_000, e, f)


if __name__ == "__main__":
    main()
