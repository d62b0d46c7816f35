"""The SageBlock operators under HIP graph capture (torch.cuda.graph): the
forward of an eval-mode block -- gathers and fused dense layers launched by
``torch.ops.sldm.sage_stack_fwd`` on the capturing stream, outputs from the
graph's private pool -- is captured once and replayed with new inputs; every
replay is compared with the eager result computed between the replays (eager
work and synchronisations in between, several replays).  The graph's CSR is
built before the capture (its build clears counters and checks ids on the
host, which a capture cannot hold)."""
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
