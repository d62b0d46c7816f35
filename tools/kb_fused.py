"""Kernel bench of the fused backward boundary vs gather + post (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402

from kbench import timeit  # noqa: E402


def main():
    from sldm_sage import build_graph, ops
    n, e, f = 10_000_000, 100_000_000, 256
    dev = "cuda"
    gen = torch.Generator(device=dev).manual_seed(0)
    ei = torch.stack([torch.randint(0, n, (e,), generator=gen, device=dev),
                      torch.randint(0, n, (e,), generator=gen, device=dev)])
    gr = build_graph(ei, n)
    del ei
    bf = torch.bfloat16
    g = torch.randn(n, f, device=dev, generator=gen).to(bf)
    add = torch.randn(n, f, device=dev, generator=gen).to(bf)
    xh = torch.randn(n, f, device=dev, generator=gen).to(bf)
    rs = torch.rand(n, device=dev) + 0.5
    gam, bet = torch.ones(f, device=dev), torch.zeros(f, device=dev)
    t_g = timeit(lambda: ops.gather_rows(g, gr.t_rowptr, gr.t_col, n, False, addend=add), 5)
    dx = ops.gather_rows(g, gr.t_rowptr, gr.t_col, n, False, addend=add)
    t_p = timeit(lambda: ops.post_bwd(dx, xh, rs, gam, bet, 0.1, 0.25, 3, bf), 5)
    t_f = timeit(lambda: ops.gather_post_bwd(g, gr.t_rowptr, gr.t_col, None, add, xh, rs, gam,
                                             bet, 0.1, 0.25, 3), 5)
    print(f"gather_bwd {t_g:.3f} ms + post_bwd {t_p:.3f} ms = {t_g + t_p:.3f} ms; "
          f"fused {t_f:.3f} ms")


if __name__ == "__main__":
    main()
