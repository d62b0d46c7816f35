"""The partitioned SageBlock at the BASELINE configs' own sizes, W = 2 ranks
sharing cuda:0 over gloo (RCCL needs one GPU per rank), against the
single-GPU SageBlock on the same graph, weights, dropout seeds and upstream
gradient:

  * C5 (5M nodes / 80M edges, power-law in-degrees up to ~10^4, F = 256,
    2 layers) on the destination-row (halo) strategy with cost-balanced
    blocks; the top hub and a zero-in-degree node are checked by name;
  * C4 (10M nodes / 100M edges, uniform, F = 256, 2 layers) on the
    feature-sliced strategy.

Every own row of every rank is compared (a dense upstream gradient, training
mode with dropout 0.25: the masks' global row keys are part of the check):
fp32 -- forward rows and input-gradient rows BITWISE equal to one GPU (each
row is summed by one kernel in CSR order, hubs in the same chunks), parameter
gradients within 1e-4 of their range (the ranks' partial sums are added in
another order); bf16 -- forward bitwise, input gradients bitwise, parameter
gradients within 1e-2 of range.  bf16 feature slicing rounds the gathered
gradient to bf16 before the root-path add (one rounding more than
SageBlock), so its input gradient is compared bitwise with the SAME
feature-sliced path at W = 1 on the whole graph (whose rounding points
tests/test_gpu_dist.py pins to the bf16-storage oracle at small size), and
against SageBlock's only as a count: where the two terms cancel, half an ulp
of the larger term shows (measured at C4: 3.4e-6 of the elements beyond
1e-2 + 1e-2 |ref|, max |diff| 0.0625).
A small power-law case with a forced hub threshold runs the same worker.

The single-GPU SageBlock itself is pinned to the CPU oracle at these sizes by
tests/test_gpu_parity.py (k-hop property).
"""
from __future__ import annotations

import os
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, cfg, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "sldm-gnn_amd")]
    import torch.distributed as dist
    t0 = time.perf_counter()

    def log(msg):
        print(f"[fullsize r{rank}] {time.perf_counter() - t0:7.1f} s  {msg}", flush=True)

    try:
        import bench
        from _helpers import assert_bf16_close
        from sldm_sage import SageBlock
        from sldm_sage import graph as graph_mod
        from sldm_sage.dist import (DistSageBlock, FeaturePartition, GraphPartition,
                                    partition_features, plan_partition)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dtype = getattr(torch, cfg["dtype"])
        n, e, hd, strategy = cfg["n"], cfg["e"], cfg["hd"], cfg["strategy"]
        if cfg.get("hub_thr"):                       # small case: force the hub split
            graph_mod.HUB_MIN_EDGES = 0
            thr = cfg["hub_thr"]
            graph_mod.hub_threshold = lambda _n, _e: thr
        ei, x = bench.make_graph(n, e, hd[0], dtype, dev, seed=cfg.get("seed", 0),
                                 kind=cfg["kind"])
        gen = torch.Generator(device=dev).manual_seed(17)
        gout = torch.randn(n, hd[-1], generator=gen, device=dev).to(dtype)
        torch.manual_seed(0)
        blk = SageBlock(hd, 0.25, 0.1).to(dev).train()
        log(f"graph + inputs ready ({cfg['kind']}, {n} nodes, {e} edges, {cfg['dtype']})")

        part, info = plan_partition(ei, n, world, rank, hd[0], x.element_size(),
                                    strategy=strategy, chunks=4, balance="cost")
        assert info["strategy"] == strategy
        assert isinstance(part, FeaturePartition if strategy == "feature" else GraphPartition)
        r0, r1 = part.row_begin, part.row_end
        log(f"partition ready: rows [{r0}, {r1})")

        # the single-GPU reference, one rank at a time (its saved activations
        # are the memory peak); each rank keeps only its own rows of it
        deg = torch.bincount(ei[1], minlength=n)
        hub_row, zero_row = int(deg.argmax()), int((deg == 0).nonzero()[0])
        hub_deg = int(deg[hub_row])
        del deg
        ref = {}
        for turn in range(world):
            if turn == rank:
                torch.manual_seed(123)
                xa = x.clone().requires_grad_(True)
                out_a = blk(xa, ei)
                out_a.backward(gout)
                torch.cuda.synchronize()
                g = graph_mod.get_graph(ei, n)
                ref["hub_split"] = g.hub is not None
                ref["out"] = out_a.detach()[r0:r1].clone()
                ref["dx"] = xa.grad[r0:r1].clone()
                ref["grads"] = {k: p.grad.clone() for k, p in blk.named_parameters()}
                blk.zero_grad(set_to_none=True)
                if dtype == torch.bfloat16 and strategy == "feature":
                    # the feature-sliced arithmetic on one GPU (W = 1): the
                    # like-for-like reference of the bf16 input gradient
                    one = DistSageBlock(blk, partition_features(ei, n, 1, 0, chunks=4),
                                        broadcast_params=False)
                    torch.manual_seed(123)
                    x1 = x.clone().requires_grad_(True)
                    out_1 = one(x1)
                    out_1.backward(gout)
                    torch.cuda.synchronize()
                    assert torch.equal(out_1, out_a), "W = 1 feature slicing: forward differs"
                    ref["dx_feat1"] = x1.grad[r0:r1].clone()
                    blk.zero_grad(set_to_none=True)
                    del one, x1, out_1
                del xa, out_a, g
                graph_mod.graph_cache.clear()
                torch.cuda.empty_cache()
                log("single-GPU reference done")
            dist.barrier()
        if cfg["kind"] == "powerlaw":
            assert ref["hub_split"], "the single-GPU run did not take the hub split"
            if strategy == "halo":
                plans = [part.fwd.hub] + ([part.fwd_split.resident.hub, part.fwd_split.pending.hub]
                                          if part.fwd_split is not None else [])
                owned = r0 <= hub_row < r1
                assert owned == any(
                    p is not None and bool((p.hub_rows == hub_row - r0).any()) for p in plans)

        model = DistSageBlock(blk, part)
        torch.manual_seed(123)                      # the reference's dropout seeds
        xb = x[r0:r1].clone().requires_grad_(True)
        out_b = model(xb)
        out_b.backward(gout[r0:r1])
        torch.cuda.synchronize()
        log("partitioned step done")

        assert torch.equal(out_b, ref["out"]), "forward rows differ from the single-GPU run"
        bf16 = dtype == torch.bfloat16
        if bf16 and strategy == "feature":
            assert torch.equal(xb.grad, ref["dx_feat1"]), \
                "input-gradient rows differ from the W = 1 feature-sliced run"
            d = (xb.grad.float() - ref["dx"].float()).abs()
            beyond = int((d > 1e-2 + 1e-2 * ref["dx"].float().abs()).sum())
            log(f"dx vs SageBlock: {beyond} of {d.numel()} elements beyond 1e-2 + 1e-2|ref|, "
                f"max |diff| {float(d.max()):.4g}")
            assert beyond <= 2e-5 * d.numel() and float(d.max()) <= 0.25
            del d
        else:
            assert torch.equal(xb.grad, ref["dx"]), "input-gradient rows differ"
        for name, row in (("hub", hub_row), ("zero-in-degree", zero_row)):
            if cfg["kind"] == "powerlaw" and r0 <= row < r1:
                assert torch.equal(out_b[row - r0], ref["out"][row - r0]), name
                log(f"{name} row {row} (in-degree {hub_deg if name == 'hub' else 0}) checked")
        for k, p in blk.named_parameters():
            want = ref["grads"][k]
            if bf16:
                assert_bf16_close(k, p.grad, want, reduction=True)
            else:
                s = max(1.0, want.abs().max().item())
                torch.testing.assert_close(p.grad / s, want / s, atol=1e-4, rtol=1e-4,
                                           msg=lambda m: f"{k}: {m}")
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(cfg, world=2, timeout=800):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = [q.get(timeout=timeout) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, msg in results:
        assert msg == "ok", f"rank {rank}:\n{msg}"


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_small_powerlaw_halo_hub_split_two_ranks(dtype):
    """The worker on a small power-law graph with the hub threshold forced to
    48: both ranks split their own hubs into the single-GPU run's chunks."""
    _run(dict(kind="powerlaw", n=20_000, e=300_000, hd=[32, 32, 32], dtype=dtype,
              strategy="halo", hub_thr=48))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_small_f256_feature_two_ranks(dtype):
    """Feature slices at F = 256 on a small graph: in bf16 the backward's dX
    GEMM writes dAgg / deg in the all-to-all's send layout (no packing copy);
    same bitwise checks as the full-size case."""
    _run(dict(kind="uniform", n=30_000, e=200_000, hd=[256, 256, 256], dtype=dtype,
              strategy="feature"))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_full_size_c5_halo_two_ranks(dtype):
    """BASELINE configs[4] (C5, power-law) on cost-balanced destination-row
    blocks with the halo exchange."""
    _run(dict(kind="powerlaw", n=5_000_000, e=80_000_000, hd=[256, 256, 256], dtype=dtype,
              strategy="halo"))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_full_size_c4_feature_two_ranks(dtype):
    """BASELINE configs[3] (C4, uniform) on feature slices."""
    _run(dict(kind="uniform", n=10_000_000, e=100_000_000, hd=[256, 256, 256], dtype=dtype,
              strategy="feature"))
