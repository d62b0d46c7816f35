"""Prints the planner's modelled per-layer times and choice for scaled-down C4
shapes (uniform and the locality variant) at W = 2, 4, 8 -- times x10 to C4
scale (diagnostic; one process, a gloo group of one for the max-reduce)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from sldm_sage.dist import choose_strategy, estimate_strategies
    n, e, f = 1_000_000, 10_000_000, 256
    g = torch.Generator().manual_seed(0)
    ei = torch.stack([torch.randint(0, n, (e,), generator=g),
                      torch.randint(0, n, (e,), generator=g)])
    dst = ei[1]
    blk = n // 8
    loc = (dst // blk) * blk + torch.randint(0, blk, (e,), generator=g)
    use = torch.rand(e, generator=g) < 0.9
    eil = torch.stack([torch.where(use, loc.clamp(max=n - 1), ei[0]), dst])
    for name, edges in (("uniform", ei), ("local", eil)):
        for w in (2, 4, 8):
            r = estimate_strategies(edges, n, w, 0, f, 2)
            best = choose_strategy(r)
            print(name, w, {k: round(v * 1e4, 2) for k, v in r.items() if k.endswith("_s")},
                  "->", best, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
