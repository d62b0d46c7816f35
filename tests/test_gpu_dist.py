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
    """Feature slicing at W = 1 (chunked gathers, layout copies).  fp32 (with
    dropout): forward and input grad bit-equal to SageBlock.  bf16 (eval, no
    dropout): forward bit-equal to SageBlock; input and parameter grads
    element-wise within 1e-2 of the bf16-storage oracle in its
    ``round_sum_first`` form (the feature path rounds the gathered dAgg to
    bf16 before adding the root-path grad)."""
    from _helpers import assert_bf16_close, bf16_oracle, oracle_block
    from oracle.sage_ref import random_graph
    from sldm_sage import SageBlock
    from sldm_sage.dist import DistSageBlock, partition_features
    n, e, hd = 3000, 20000, [32, 64, 64]
    ei, x = random_graph(n, e, hd[0], seed=5)
    gout = torch.randn(n, hd[-1], generator=torch.Generator().manual_seed(6)).to(dtype)
    bf = dtype == torch.bfloat16
    ref = oracle_block(hd, 0.1)
    blk = SageBlock(hd, None if bf else 0.25, 0.1)
    blk.load_state_dict(ref.state_dict())
    blk = blk.cuda().train()
    eic, xc, gc = ei.cuda(), x.cuda().to(dtype), gout.cuda()
    torch.manual_seed(7)
    xa = xc.clone().requires_grad_(True)
    out_a = blk(xa, eic)
    out_a.backward(gc)
    ga = {k: p.grad.clone() for k, p in blk.named_parameters()}
    blk.zero_grad(set_to_none=True)

    part = partition_features(eic, n, 1, 0, chunks=3)
    model = DistSageBlock(blk, part)
    assert model.strategy == "feature"
    torch.manual_seed(7)
    xb = xc.clone().requires_grad_(True)
    out_b = model(xb)
    out_b.backward(gc)
    assert torch.equal(out_a, out_b)
    if not bf:
        assert torch.equal(xa.grad, xb.grad)
        for k, p in blk.named_parameters():
            torch.testing.assert_close(p.grad, ga[k], atol=2e-4, rtol=2e-4)
        return
    _, dx_r, gr = bf16_oracle(ref, x.to(dtype).float(), ei, gout.float(), 0.1,
                              round_sum_first=True)
    assert_bf16_close("dx", xb.grad, dx_r)
    for k, p in blk.named_parameters():
        assert_bf16_close(k, p.grad, gr[k])


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
        from _helpers import assert_bf16_close, bf16_oracle, oracle_block
        n, e, hd = 2001, 16000, [32, 48, 32]
        ei_cpu, x_cpu = random_graph(n, e, hd[0], seed=9)
        ei, x = ei_cpu.cuda(), x_cpu.cuda().to(dtype)
        # bf16 feature slicing runs in eval mode and is held to the
        # bf16-storage oracle (round_sum_first); everything else with dropout
        # against the single-GPU SageBlock
        bf_feat = dtype == torch.bfloat16 and strategy == "feature"
        torch.manual_seed(0)
        ref = oracle_block(hd, 0.1)
        blk = SageBlock(hd, None if bf_feat else 0.25, 0.1)
        if bf_feat:
            blk.load_state_dict(ref.state_dict())
        blk = blk.cuda().train()
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
        if bf_feat:
            _, dx_r, gr = bf16_oracle(ref, x_cpu.to(dtype).float(), ei_cpu, gout.float().cpu(),
                                      0.1, round_sum_first=True)
            assert_bf16_close("dx", xb.grad, dx_r[r0:r1])
            for k, p in blk.named_parameters():
                assert_bf16_close(k, p.grad, gr[k])
        else:
            assert torch.equal(xb.grad, xa.grad[r0:r1]), "input grad differs"
            for k, p in blk.named_parameters():
                if info["strategy"] == "replicate":
                    assert torch.equal(p.grad, ga[k]), k
                else:
                    torch.testing.assert_close(p.grad, ga[k], atol=2e-4, rtol=2e-4)
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
