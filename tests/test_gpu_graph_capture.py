"""The SageBlock operators under HIP graph capture (torch.cuda.graph): the
forward of an eval-mode block -- gathers and fused dense layers launched by
``torch.ops.sldm.sage_stack_fwd`` on the capturing stream, outputs from the
graph's private pool -- is captured once and replayed with new inputs; every
replay is compared with the eager result computed between the replays (eager
work and synchronisations in between, several replays).  A static graph's CSR
is built before the capture (the warm-up calls cache it); a per-batch graph's
build is recorded too, and a training step with dropout takes its seed from a
device word so that replays draw new masks."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("dtype,hd", [(torch.float32, [64, 64, 64]),
                                      (torch.bfloat16, [256, 256, 256]),
                                      (torch.float32, [256, 256])])
def test_sageblock_forward_replays_in_a_hip_graph(dtype, hd):
    from sldm_sage import SageBlock
    from oracle.sage_ref import random_graph
    n, e = 3000, 20000
    ei, x = random_graph(n, e, hd[0], seed=3)
    eid = ei.to(DEV)
    torch.manual_seed(0)
    blk = SageBlock(hd, None, 0.1).to(DEV).eval()
    static_x = x.to(DEV).to(dtype)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.no_grad(), torch.cuda.stream(side):
        for _ in range(3):                      # CSR build, library loads, allocator warm-up
            blk(static_x, eid)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(graph):
        static_out = blk(static_x, eid)
    gen = torch.Generator(device=DEV).manual_seed(11)
    for _ in range(4):
        new = torch.randn(n, hd[0], generator=gen, device=DEV).to(dtype)
        with torch.no_grad():
            eager = blk(new, eid)               # the program's own eager work between replays
        torch.cuda.synchronize()
        static_x.copy_(new)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(static_out, eager)


@pytest.mark.parametrize("dtype,hd", [(torch.float32, [16, 32, 32]),       # the lane-map block
                                      (torch.bfloat16, [256, 256, 256])])
def test_sageblock_training_step_replays_in_a_hip_graph(dtype, hd):
    """Forward + backward of a train-mode block without dropout on a static
    graph (the lane map's case, mapencoder.py:12, :37) captured as one HIP
    graph: outputs, the input gradient and every parameter gradient of each
    replay equal the eager step's on the same input."""
    from sldm_sage import SageBlock
    from oracle.sage_ref import random_graph
    n, e = 2500, 15000
    ei, x = random_graph(n, e, hd[0], seed=5)
    eid = ei.to(DEV)
    torch.manual_seed(1)
    blk = SageBlock(hd, None, 0.1).to(DEV).train()
    static_x = x.to(DEV).to(dtype).requires_grad_(True)
    static_g = torch.randn(n, hd[-1], device=DEV).to(dtype)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            blk.zero_grad(set_to_none=True)
            static_x.grad = None
            blk(static_x, eid).backward(static_g)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    blk.zero_grad(set_to_none=True)
    static_x.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_out = blk(static_x, eid)
        static_out.backward(static_g)
    static_grads = [p.grad for p in blk.parameters()]
    static_dx = static_x.grad
    gen = torch.Generator(device=DEV).manual_seed(13)
    twin = SageBlock(hd, None, 0.1).to(DEV).train()
    twin.load_state_dict(blk.state_dict())
    for _ in range(3):
        new = torch.randn(n, hd[0], generator=gen, device=DEV).to(dtype)
        newg = torch.randn(n, hd[-1], generator=gen, device=DEV).to(dtype)
        xe = new.clone().requires_grad_(True)
        twin.zero_grad(set_to_none=True)
        eager = twin(xe, eid)
        eager.backward(newg)
        torch.cuda.synchronize()
        with torch.no_grad():
            static_x.copy_(new)
            static_g.copy_(newg)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(static_out, eager.detach())
        assert torch.equal(static_dx, xe.grad)
        for got, p in zip(static_grads, twin.parameters()):
            assert torch.equal(got, p.grad)


def _padded_batch(n_real, e_real, n_pad, e_pad, feat, seed, dtype):
    """A batch's graph padded to the captured shapes: random edges among the
    first n_real nodes, the unused tail of edge_index filled with the padding
    edge (N, N) that the CSR build ignores, feature rows past n_real zero."""
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n_real, (2, e_real), generator=g)
    pad = torch.full((2, e_pad - e_real), n_pad, dtype=torch.int64)
    x = torch.zeros(n_pad, feat)
    x[:n_real] = torch.randn(n_real, feat, generator=g)
    return torch.cat([ei, pad], 1).to(DEV), x.to(DEV).to(dtype)


def test_per_batch_graph_forward_replays_in_a_hip_graph():
    """A per-batch graph (main.py:166: every pack has its own edge_index):
    the edge_index buffer is refilled between replays, so the CSR build is
    part of the captured graph; eval mode.  Each replay equals the eager call
    on a fresh copy of the same batch."""
    from sldm_sage import SageBlock
    n_pad, e_pad, hd = 1500, 9000, [64, 64, 64]
    torch.manual_seed(2)
    blk = SageBlock(hd, 0.25, 0.1).to(DEV).eval()
    static_ei, static_x = _padded_batch(1200, 7000, n_pad, e_pad, hd[0], 0, torch.float32)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.no_grad(), torch.cuda.stream(side):
        for _ in range(3):
            blk(static_x, static_ei.clone())
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(graph):
        static_out = blk(static_x, static_ei)
    for rep, (n_real, e_real) in enumerate([(1400, 8800), (900, 3000), (1499, 9000)]):
        ei, x = _padded_batch(n_real, e_real, n_pad, e_pad, hd[0], 10 + rep, torch.float32)
        with torch.no_grad():
            eager = blk(x, ei)
        torch.cuda.synchronize()
        static_ei.copy_(ei)
        static_x.copy_(x)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(static_out, eager)


@pytest.mark.parametrize("dtype,hd", [(torch.float32, [64, 64, 64]),        # tile kernels
                                      (torch.bfloat16, [256, 256, 256]),     # bf16 stream kernels
                                      (torch.float32, [256, 256]),           # fp32 stream kernels
                                      (torch.bfloat16, [128, 128, 128]),     # big-tile kernel
                                      (torch.float32, [16, 32, 32])])        # the lane-map block
def test_per_batch_training_step_with_dropout_replays_in_a_hip_graph(dtype, hd, monkeypatch):
    """The reference's training step on a pack (utils.py:218-227: train mode,
    dropout on, a new edge_index per batch) captured once at padded shapes:
    CSR build, forward and backward are all in the graph.  The dropout seed
    is the device's capture counter, advanced by a recorded launch, so every
    replay drops a new mask; with the counter's value as its host seed an
    eager call reproduces each replay bit for bit (outputs, input gradient,
    parameter gradients)."""
    import sldm_sage.sageblock as sb
    from sldm_sage import SageBlock, ops
    n_pad, e_pad = 1500, 9000
    torch.manual_seed(4)
    blk = SageBlock(hd, 0.25, 0.1).to(DEV).train()
    twin = SageBlock(hd, 0.25, 0.1).to(DEV).train()
    twin.load_state_dict(blk.state_dict())
    static_ei, x0 = _padded_batch(1200, 7000, n_pad, e_pad, hd[0], 0, dtype)
    static_x = x0.requires_grad_(True)
    static_g = torch.randn(n_pad, hd[-1], device=DEV).to(dtype)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            blk.zero_grad(set_to_none=True)
            static_x.grad = None
            blk(static_x, static_ei.clone()).backward(static_g)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    blk.zero_grad(set_to_none=True)
    static_x.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static_out = blk(static_x, static_ei)
        static_out.backward(static_g)
    static_grads = [p.grad for p in blk.parameters()]
    static_dx = static_x.grad
    masks = []
    for rep, (n_real, e_real) in enumerate([(1400, 8800), (900, 3000), (1400, 8800)]):
        ei, x = _padded_batch(n_real, e_real, n_pad, e_pad, hd[0], 20 + (rep % 2), dtype)
        g = torch.randn(n_pad, hd[-1], device=DEV).to(dtype)
        with torch.no_grad():
            static_ei.copy_(ei)
            static_x.copy_(x)
            static_g.copy_(g)
        graph.replay()
        torch.cuda.synchronize()
        word = int(ops.capture_seed_counter(DEV))       # this replay's seed word
        seeds = iter(word + layer for layer in range(len(hd) - 1))
        monkeypatch.setattr(sb, "_new_seed", lambda dev=None: next(seeds))
        xe = x.clone().requires_grad_(True)
        twin.zero_grad(set_to_none=True)
        eager = twin(xe, ei)
        eager.backward(g)
        torch.cuda.synchronize()
        assert torch.equal(static_out, eager.detach())
        assert torch.equal(static_dx, xe.grad)
        for got, p in zip(static_grads, twin.parameters()):
            assert torch.equal(got, p.grad)
        masks.append((static_out[:n_real] == 0).clone())
        frac = masks[-1].float().mean().item()
        assert 0.2 < frac < 0.3                          # p = 0.25 really drops
    # replays 0 and 2 ran the same batch: same inputs, different masks
    assert not torch.equal(masks[0], masks[2])
