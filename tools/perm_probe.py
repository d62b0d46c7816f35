"""Probe: torch permute-copy rates of the feature-sliced layout switches (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]
import torch  # noqa: E402

from kbench import timeit  # noqa: E402

P, F = 1_250_000, 256
for W in (2, 4, 8):
    cs = F // W
    x = torch.randn(P, F, device="cuda").bfloat16()
    recv = torch.randn(W * P * cs, device="cuda").bfloat16()
    out = torch.empty(P, F, device="cuda", dtype=torch.bfloat16)
    a = torch.randn(P, F, device="cuda").bfloat16()
    t_pack = timeit(lambda: x.reshape(P, W, cs).transpose(0, 1).contiguous(), 5)
    t_unpack = timeit(lambda: out.view(P, W, cs).copy_(recv.view(W, P, cs).transpose(0, 1)), 5)
    t_add = timeit(lambda: a + out, 5)
    t_copy = timeit(lambda: x.clone(), 5)
    gb = P * F * 2 * 2 / 1e9
    print(f"W={W}: pack {t_pack:.3f} ms ({gb / t_pack:.2f} TB/s)  unpack {t_unpack:.3f} ms "
          f"({gb / t_unpack:.2f})  add {t_add:.3f} ms ({1.5 * gb / t_add:.2f})  clone {t_copy:.3f} "
          f"({gb / t_copy:.2f})", flush=True)
