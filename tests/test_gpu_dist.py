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
        # SageBlock's fused layer boundary sums the lower layers' LayerNorm /
        # bias column gradients in another row order (fp32 rounding only)
        torch.testing.assert_close(p.grad, ga[k], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_feature_sliced_world1_matches_sageblock(pg, dtype):
    """Feature slicing at W = 1 (chunked gathers, layout copies): forward bit-equal;
    input grad bit-equal in fp32 (bf16: the two-term add rounds once more)."""
    from oracle.sage_ref import random_graph
    from sldm_sage import SageBlock
    from sldm_sage.dist import DistSageBlock, partition_features
    n, e, hd = 3000, 20000, [32, 64, 64]
    ei, x = random_graph(n, e, hd[0], seed=5)
    ei, x = ei.cuda(), x.cuda().to(dtype)
    torch.manual_seed(0)
    blk = SageBlock(hd, 0.25, 0.1).cuda().train()
    gout = torch.randn(n, hd[-1], device="cuda").to(dtype)
    torch.manual_seed(7)
    xa = x.clone().requires_grad_(True)
    out_a = blk(xa, ei)
    out_a.backward(gout)
    ga = {k: p.grad.clone() for k, p in blk.named_parameters()}
    blk.zero_grad(set_to_none=True)

    part = partition_features(ei, n, 1, 0, chunks=3)
    model = DistSageBlock(blk, part)
    assert model.strategy == "feature"
    torch.manual_seed(7)
    xb = x.clone().requires_grad_(True)
    out_b = model(xb)
    out_b.backward(gout)
    assert torch.equal(out_a, out_b)
    if dtype == torch.float32:
        assert torch.equal(xa.grad, xb.grad)
    else:
        _close_in_range(xb.grad, xa.grad)
    for k, p in blk.named_parameters():
        _grad_close(p.grad, ga[k], dtype, k)


def _grad_close(a, b, dtype, what):
    """fp32: 1e-4.  bf16: the extra rounding of the input grad (above) feeds the
    lower layer's weight grads through LeakyReLU's kink and LayerNorm's
    backward, so they are compared by relative norm (bf16 bar, 3e-2)."""
    if dtype == torch.float32:
        torch.testing.assert_close(a, b, atol=2e-4, rtol=2e-4)
        return
    rel = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()
    assert rel <= 3e-2, f"{what}: relative norm error {rel:.3e}"


def _close_in_range(a, b, tol=1e-2):
    """north_star's bf16 bar (1e-2), relative to the tensor's range: the
    feature-sliced backward rounds dAgg to bf16 before adding the root-path
    grad (one bf16 ulp of either term, absolute)."""
    err = (a.float() - b.float()).abs().max().item()
    assert err <= tol * b.float().abs().max().item(), f"max err {err}"


def _mp_worker(rank, world, port, strategy, dtype_name, q):
    """One rank of a W-process run on the single GPU (gloo carries the
    collectives; every rank computes with the HIP kernels on cuda:0)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "sldm-gnn_amd")]
    import torch.distributed as dist
    try:
        from oracle.sage_ref import random_graph
        from sldm_sage import SageBlock
        from sldm_sage.dist import DistSageBlock, plan_partition
        dtype = getattr(torch, dtype_name)
        torch.cuda.set_device(0)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n, e, hd = 2001, 16000, [32, 48, 32]
        ei, x = random_graph(n, e, hd[0], seed=9)
        ei, x = ei.cuda(), x.cuda().to(dtype)
        torch.manual_seed(0)
        blk = SageBlock(hd, 0.25, 0.1).cuda().train()
        gout = torch.randn(n, hd[-1], device="cuda").to(dtype)
        torch.manual_seed(11)
        xa = x.clone().requires_grad_(True)
        out_a = blk(xa, ei)
        out_a.backward(gout)
        ga = {k: p.grad.clone() for k, p in blk.named_parameters()}
        blk.zero_grad(set_to_none=True)

        part, info = plan_partition(ei, n, world, rank, hd[0], x.element_size(),
                                    strategy=strategy, chunks=3)
        model = DistSageBlock(blk, part)
        r0, r1 = part.row_begin, part.row_end
        torch.manual_seed(11)
        xb = x[r0:r1].clone().requires_grad_(True)
        out_b = model(xb)
        out_b.backward(gout[r0:r1])
        torch.cuda.synchronize()
        assert torch.equal(out_b, out_a[r0:r1]), "forward rows differ"
        if dtype == torch.float32 or info["strategy"] in ("halo", "replicate"):
            assert torch.equal(xb.grad, xa.grad[r0:r1]), "input grad differs"
        else:
            _close_in_range(xb.grad, xa.grad[r0:r1])
        for k, p in blk.named_parameters():
            if info["strategy"] == "replicate":
                assert torch.equal(p.grad, ga[k]), k
            elif info["strategy"] == "halo":
                torch.testing.assert_close(p.grad, ga[k], atol=2e-4, rtol=2e-4)
            else:
                _grad_close(p.grad, ga[k], dtype, k)
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("strategy", ["halo", "feature", "replicate"])
@pytest.mark.parametrize("dtype_name", ["float32", "bfloat16"])
def test_two_ranks_one_gpu(strategy, dtype_name):
    """W = 2 processes sharing cuda:0 over gloo: the multi-rank protocol with
    the HIP kernels (RCCL needs one GPU per rank; the driver's 8-GPU bench
    covers RCCL itself)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, strategy, dtype_name, q))
             for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}:\n{msg}"
