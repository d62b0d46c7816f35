"""The distributed SageBlock's HIP backend on one GPU (world = 1 RCCL group):
the partitioned path must reproduce SageBlock exactly (same kernels, same CSR
order), including dropout masks (global-row keys)."""
from __future__ import annotations

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    if dist.is_initialized():
        yield
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("dropout", [None, 0.25])
def test_dist_world1_matches_sageblock(pg, dtype, dropout):
    from oracle.sage_ref import random_graph
    from sldm_sage import SageBlock
    from sldm_sage.dist import DistSageBlock, partition_graph
    n, e, hd = 3000, 20000, [32, 64, 64]
    ei, x = random_graph(n, e, hd[0], seed=2)
    ei, x = ei.cuda(), x.cuda().to(dtype)
    torch.manual_seed(0)
    blk = SageBlock(hd, dropout, 0.1).cuda().train()
    gout = torch.randn(n, hd[-1], device="cuda").to(dtype)

    torch.manual_seed(123)
    xa = x.clone().requires_grad_(True)
    out_a = blk(xa, ei)
    out_a.backward(gout)
    ga = {k: p.grad.clone() for k, p in blk.named_parameters()}
    blk.zero_grad(set_to_none=True)

    part = partition_graph(ei, n, 1, 0)
    model = DistSageBlock(blk, part)
    torch.manual_seed(123)                     # same dropout seeds
    xb = x.clone().requires_grad_(True)
    out_b = model(xb)
    out_b.backward(gout)
    assert torch.equal(out_a, out_b)
    assert torch.equal(xa.grad, xb.grad)
    for k, p in blk.named_parameters():
        torch.testing.assert_close(p.grad, ga[k], atol=1e-6, rtol=1e-6)
