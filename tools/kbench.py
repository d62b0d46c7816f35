"""Per-kernel micro-benchmark of the C-ABI ops at a chosen workload shape.

    python tools/kbench.py [--nodes 10000000] [--edges 100000000] [--feat 256] [--dtype bf16]

Times each op in isolation with HIP events (median of --reps after warm-up)
and prints algorithmic GB/s; variants isolate the cost of the fused parts
(dropout, saved xhat, column blocks).  Diagnostic only.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--feat", type=int, default=256)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from sldm_sage import build_graph, ops
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    s = 2 if dt == torch.bfloat16 else 4
    n, e, f = a.nodes, a.edges, a.feat
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    ei = torch.stack([torch.randint(0, n, (e,), generator=g, device=dev),
                      torch.randint(0, n, (e,), generator=g, device=dev)])
    x = torch.randn(n, f, device=dev, generator=g).to(dt)
    gr = build_graph(ei, n)
    agg = ops.gather_rows(x, gr.rowptr, gr.col, n, True)
    wcat = (torch.randn(f, 2 * f, device=dev) / (2 * f) ** 0.5).to(dt).contiguous()
    b = torch.zeros(f, device=dev)
    gam = torch.ones(f, device=dev)
    bet = torch.zeros(f, device=dev)
    dh = torch.randn(n, f, device=dev).to(dt)
    wt = wcat.t().contiguous()
    res = []

    def add(name, ms, nbytes, flops=0.0):
        res.append((name, ms, nbytes / ms / 1e6, flops / ms / 1e9))

    sel = a.only.split(",") if a.only else None

    def want(k):
        return sel is None or k in sel

    if want("gather"):
        add("gather_fwd", timeit(lambda: ops.gather_rows(x, gr.rowptr, gr.col, n, True), a.reps),
            e * (4 + f * s) + (n + 1) * 4 + n * f * s)
    fl = 2.0 * n * 2 * f * f
    if want("dense1"):
        # the default forward kernel only (library A/B)
        for p_ in (0.25, 0.0):
            ms = timeit(lambda: ops.sage_dense_fwd(agg, x, wcat, b, gam, bet, 1e-5, 0.1, p_, 7,
                                                   True), a.reps)
            add(f"dense_fwd p={p_} save=True", ms, 4 * n * f * s, fl)
    if want("dense"):
        for p_, save in [(0.25, True), (0.0, True), (0.0, False)]:
            ms = timeit(lambda: ops.sage_dense_fwd(agg, x, wcat, b, gam, bet, 1e-5, 0.1, p_, 7,
                                                   save), a.reps)
            add(f"dense_fwd p={p_} save={save}", ms, (2 * n * f + n * f * (2 if save else 1)) * s,
                fl)
    if want("nt"):
        add("gemm_nt_rowscale N=2f", timeit(lambda: ops.gemm_nt_rowscale(dh, wt, gr.rowptr, f),
                                            a.reps), (n * f + n * 2 * f) * s, fl)
        add("gemm_nt_rowscale N=2f split", timeit(
            lambda: ops.gemm_nt_rowscale(dh, wt, gr.rowptr, f, split=True), a.reps),
            (n * f + n * 2 * f) * s, fl)
        os.environ["SLDM_WS_GEMM"] = "0"
        add("gemm_nt_rowscale N=2f split stream", timeit(
            lambda: ops.gemm_nt_rowscale(dh, wt, gr.rowptr, f, split=True), a.reps),
            (n * f + n * 2 * f) * s, fl)
        os.environ.pop("SLDM_WS_GEMM")
        add("gemm_nt_rowscale N=f", timeit(lambda: ops.gemm_nt_rowscale(dh, wcat[:, :f].contiguous(),
                                                                         None, 0), a.reps),
            (n * f + n * f) * s, fl / 2)
    if want("tn"):
        add("gemm_tn", timeit(lambda: ops.gemm_tn(dh, agg, x), a.reps), 3 * n * f * s, fl)
        os.environ["SLDM_TN_DMA"] = "0"
        add("gemm_tn tiles", timeit(lambda: ops.gemm_tn(dh, agg, x), a.reps), 3 * n * f * s, fl)
        os.environ.pop("SLDM_TN_DMA")
    if want("mix"):
        # the traffic mixes of the dense kernels through torch's elementwise
        # kernels: the rate a plain streaming kernel reaches for them here
        c = torch.empty_like(dh)
        add("torch add 2R:1W [N,F]", timeit(lambda: torch.add(dh, x, out=c), a.reps), 3 * n * f * s)
        add("torch copy 1R:1W [N,F]", timeit(lambda: c.copy_(dh), a.reps), 2 * n * f * s)
        c2 = torch.empty(n, 2 * f, device=dev, dtype=dt)
        add("torch cat 2R:2W [N,2F]", timeit(lambda: torch.cat([dh, x], 1, out=c2), a.reps),
            4 * n * f * s)
        del c, c2
    if want("post"):
        out, xh, rs = ops.post_fwd(dh, None, gam, bet, 1e-5, 0.1, 0.0, 0, dt, True)
        for p_, zo in [(0.0, None), (0.25, None), (0.25, out)]:
            add(f"post_bwd p={p_} zout={zo is not None}",
                timeit(lambda: ops.post_bwd(dh, xh, rs, gam, bet, 0.1, p_, 3, dt, zout=zo),
                       a.reps), (3 + (zo is not None)) * n * f * s)
    if want("gpost"):
        # transpose gather + the LN backward of the layer below (the fused
        # layer boundary), and the plain transpose gather with an addend
        xh_, rs_ = dh, torch.rand(n, device=dev) + 0.5
        add("gather_post_bwd", timeit(lambda: ops.gather_post_bwd(
            agg, gr.t_rowptr, gr.t_col, None, x, xh_, rs_, gam, bet, 0.1, 0.25, 5), a.reps),
            e * (4 + f * s) + 4 * n * f * s)
        add("gather_bwd (sum + addend)", timeit(lambda: ops.gather_rows(
            agg, gr.t_rowptr, gr.t_col, n, False, addend=x, order=None), a.reps),
            e * (4 + f * s) + 2 * n * f * s)
    if want("concurrent"):
        # forward gather and dense forward on two streams at once (independent
        # data) vs one after the other: does overlapping them pay?
        agg2 = torch.empty_like(agg)
        s2 = torch.cuda.Stream()

        def serial():
            ops.gather_rows(x, gr.rowptr, gr.col, n, True, out=agg2)
            ops.sage_dense_fwd(agg, x, wcat, b, gam, bet, 1e-5, 0.1, 0.25, 7, True)

        def conc():
            cur = torch.cuda.current_stream()
            s2.wait_stream(cur)
            with torch.cuda.stream(s2):
                ops.sage_dense_fwd(agg, x, wcat, b, gam, bet, 1e-5, 0.1, 0.25, 7, True)
            ops.gather_rows(x, gr.rowptr, gr.col, n, True, out=agg2)
            cur.wait_stream(s2)

        add("gather_fwd + dense_fwd serial", timeit(serial, a.reps), 1, 0)
        add("gather_fwd || dense_fwd streams", timeit(conc, a.reps), 1, 0)
        tw = torch.empty(ops.gemm_tn(dh, agg, x).shape, device=dev)

        def serial_b():
            ops.gather_rows(x, gr.rowptr, gr.col, n, False, out=agg2)
            ops.gemm_tn(dh, agg, x)

        def conc_b():
            cur = torch.cuda.current_stream()
            s2.wait_stream(cur)
            with torch.cuda.stream(s2):
                ops.gemm_tn(dh, agg, x)
            ops.gather_rows(x, gr.rowptr, gr.col, n, False, out=agg2)
            cur.wait_stream(s2)

        add("gather_sum + gemm_tn serial", timeit(serial_b, a.reps), 1, 0)
        add("gather_sum || gemm_tn streams", timeit(conc_b, a.reps), 1, 0)
        del tw
    if want("torch"):
        add("torch.mm [agg|x]W^T", timeit(lambda: torch.mm(torch.cat([agg, x], 1), wcat.t()),
                                           a.reps), 3 * n * f * s, fl)
    for name, ms, gbs, tf in res:
        print(f"{name:32s} {ms:9.3f} ms {gbs:9.1f} GB/s {tf:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
