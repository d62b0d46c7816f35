"""SageBlock fwd+bwd throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4] [--no-cpu-baseline]

One "step" = SageBlock.forward(x, edge_index) + backward of a fixed upstream
gradient over one synthetic graph, dropout 0.25 in training
mode, LeakyReLU(0.1) — the reference's training configuration (main.py:39-40).
``value`` = E·L / t_step (layer-edges per second, whole job).  Inputs are
resident in HBM before the timed region; the CSR is built on the first
(warm-up) call and cached on the edge_index tensor, as for any static graph
(``value_incl_csr_build`` re-times one step with the cache cleared).

N > 1 (torchrun, one rank per GPU, RCCL): the graph is partitioned across
ranks (sldm_sage.dist.plan_partition, ``--strategy``): destination rows with a
halo all-to-all-v per layer, or feature slices with balanced layout
all-to-alls, whichever has the lower modelled time for the graph at hand;
``scaling`` is "strong" (the graph is fixed).

The JSON line also carries ``roofline`` for the dominant kernel (the CSR
gather-mean: the SageBlock scatter-add), measured with HIP events around
every launch on the launch stream inside the timed region, and
``cpu_baseline``: the CPU oracle (oracle/sage_ref.py, the reference's ATen op
sequence) timed on this host on a bounded sample (rank 0, N=1 only), and
``step_roofline`` (N=1): T* = the algorithmic bytes of every timed kernel of a
step / 8 TB/s + the step's GEMM FLOP / the dense MFMA peak, as T*/t_step.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sldm-gnn_amd")]

import torch  # noqa: E402

CONFIGS = {
    # name: (N, E, F, L, dtype, description)
    "c1": (1_000, 5_000, 16, 2, torch.float32, "C1 1k nodes / 5k edges, F=16, 2 layers, fp32"),
    "c2": (100_000, 1_000_000, 128, 2, torch.float32,
           "C2 100k nodes / 1M edges, F=128, 2 layers, fp32"),
    "c3": (1_000_000, 10_000_000, 256, 3, torch.bfloat16,
           "C3 1M nodes / 10M edges, F=256, 3 layers, bf16"),
    "c4": (10_000_000, 100_000_000, 256, 2, torch.bfloat16,
           "C4 10M nodes / 100M edges, F=256, 2 layers, bf16"),
    "c5": (5_000_000, 80_000_000, 256, 2, torch.bfloat16,
           "C5 5M nodes / 80M edges power-law in-degree (max ~10k), F=256, 2 layers, bf16"),
}
ZIPF_A = 0.47   # dst rank ~ k^-a over N ranks: max in-degree ~ E*(2^(1-a)-1)/(N^(1-a)-1) ~ 10k at C5
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0   # measured float4-copy ceiling (MI355X_MICROARCH.md)
MFMA_PEAK_TFLOPS = {torch.bfloat16: 2500.0, torch.float32: 157.3}   # dense, same guide
BREAKDOWN_STEPS = 2      # untimed steps with every op bracketed (the "kernels" table)
PMC_SUMMARY = "r3_c4_pmc_traffic.json"   # latest committed PMC passes (tools/profile_round.sh)


class KernelTimer:
    """Per-kernel launch durations from HIP events on the launch stream:
    (start, end) event pairs from launches made in Python, read after a sync,
    and milliseconds from the events the torch.ops.sldm operators record
    around their launches in C++ (``add_ms``, via ops.flush_timing)."""

    def __init__(self):
        self.events: dict[str, list] = {}
        self.ms: dict[str, list] = {}

    def __call__(self, name, start, end, units):
        self.events.setdefault(name, []).append((start, end, units))

    def add_ms(self, name, ms, units):
        self.ms.setdefault(name, []).append((ms, units))

    def summary(self):
        from sldm_sage import ops
        ops.flush_timing()
        out = {}
        for name in sorted(set(self.events) | set(self.ms)):
            evs = self.events.get(name, [])
            pre = self.ms.get(name, [])
            ms = [s.elapsed_time(e) for s, e, _ in evs] + [m for m, _ in pre]
            units = [u for _, _, u in evs] + [u for _, u in pre]
            out[name] = dict(launches=len(ms), avg_ms=sum(ms) / len(ms),
                             avg_bytes=sum(units) / len(units))
        return out


def make_graph(n, e, f, dtype, device, seed=0, kind="uniform", p_local=0.9, blocks=8):
    """The synthetic benchmark graph: src, dst uniform in [0, N) (duplicates and
    self loops allowed).  kind="local" is the locality-structured variant: dst
    uniform, src drawn from dst's own block (N split into `blocks` contiguous
    ranges = the 8-GPU partition) with probability p_local, else uniform."""
    g = torch.Generator(device=device).manual_seed(seed)
    src = torch.randint(0, n, (e,), generator=g, device=device)
    dst = torch.randint(0, n, (e,), generator=g, device=device)
    if kind == "powerlaw":
        # C5: dst from a truncated power law over ranks, ids
        # permuted by a seeded randperm so hubs are scattered; src uniform.
        u = torch.rand(e, generator=g, device=device, dtype=torch.float64)
        b = 1.0 - ZIPF_A
        rank_ = ((1.0 + u * (n ** b - 1.0)) ** (1.0 / b)).floor().long() - 1
        perm = torch.randperm(n, generator=g, device=device)
        dst = perm[rank_.clamp_(0, n - 1)]
    if kind == "local":
        P = (n + blocks - 1) // blocks
        b0 = torch.div(dst, P, rounding_mode="floor") * P
        span = torch.clamp(n - b0, max=P)
        loc = b0 + (torch.rand(e, generator=g, device=device) * span).long().clamp(max=n - 1)
        keep = torch.rand(e, generator=g, device=device) < p_local
        src = torch.where(keep, loc, src)
    x = torch.randn(n, f, generator=g, device=device).to(dtype)
    return torch.stack([src, dst]), x


def available_cpus() -> dict:
    """CPUs this process may use: its affinity mask, capped by a cgroup v2
    CPU quota when one is set (a GPU box shares its host: nproc there counts
    the whole machine).  Also nproc and lscpu's model name and sockets."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    info = {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
            "usable": min(aff, quota) if quota else aff}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            k, _, v = ln.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip().lower().replace(" ", "_").replace("(s)", "s")] = v.strip()
    except (OSError, ValueError):
        pass
    return info


def cpu_baseline(cfg, threads, frac=10, budget_s=30.0):
    """The oracle (plain-torch restatement of PyG SAGEConv + SageBlock, fp32:
    the reference's ATen op sequence) on a bounded sample of the workload --
    the same F and L, nodes and edges / ``frac`` (E/10 when the
    full graph's [E, F] message tensors do not fit) -- on ``threads`` host
    threads, one warm-up step, then timed steps until ``budget_s``."""
    from oracle.sage_ref import RefSageBlock, random_graph, set_synthetic_params
    n, e, f, L, _, _ = cfg
    ns, es = max(n // frac, 1000), max(e // frac, 5000)
    torch.set_num_threads(threads)
    ei, x = random_graph(ns, es, f, seed=0)
    blk = RefSageBlock([f] * (L + 1), dropout=0.25, negative_slope=0.1)
    set_synthetic_params(blk, 1)
    blk.train()
    gout = torch.randn(ns, f, generator=torch.Generator().manual_seed(2))
    times = []
    t_end = time.perf_counter() + budget_s
    for it in range(12):
        xr = x.clone().requires_grad_(True)
        blk.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        blk(xr, ei).backward(gout)
        dt = time.perf_counter() - t0
        if it > 0:
            times.append(dt)
        if time.perf_counter() > t_end and len(times) >= 1:
            break
    t = statistics.median(times)
    # the framework's own host path on the same sample (SageBlock on CPU
    # tensors: libsldm_sage_cpu.so + BLAS), beside the reference's op sequence
    from sldm_sage import SageBlock
    ours = SageBlock([f] * (L + 1), dropout=0.25, negative_slope=0.1)
    ours.load_state_dict(blk.state_dict())
    ours.train()
    t_ours = []
    for it in range(4):
        xr = x.clone().requires_grad_(True)
        ours.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        ours(xr, ei).backward(gout)
        if it > 0:
            t_ours.append(time.perf_counter() - t0)
    to = statistics.median(t_ours)
    return dict(value=es * L / t, unit="edges/s", cores=threads, kind="port",
                sample=f"{ns} nodes / {es} edges (1/{frac} of the workload), F={f}, L={L}, fp32, "
                       f"median of {len(times)} fwd+bwd after 1 warm-up; oracle/sage_ref.py",
                ms_per_step=t * 1e3,
                sldm_cpu_path={"value": es * L / to, "ms_per_step": to * 1e3,
                               "note": "sldm_sage.SageBlock on CPU tensors (native host "
                                       "kernels + BLAS), same sample and threads, median of 3"})


def torch_ops_gpu_baseline(blk, ei, x, gout, warmup=1, steps=2):
    """The reference's GPU path on this GPU: PyG 2.7.0 ``SAGEConv(mean)`` +
    the SageBlock post stack (sageblock.py:16-20) as the ATen ops PyG issues --
    ``index_select`` of the [E, F] messages, ``scatter_add_`` of messages and
    of the fp32 count, ``clamp(min=1)``, division, ``lin_l`` + ``lin_r``,
    LayerNorm, LeakyReLU, Dropout -- with ``blk``'s weights, in x's dtype,
    fwd + bwd of the same upstream gradient.  A measurement baseline (the
    framework never runs it); None if it does not fit in memory."""
    import torch.nn.functional as Fn
    src, dst = ei[0], ei[1]
    n = x.size(0)
    cv = dict(device=x.device, dtype=x.dtype)
    layers = [tuple(t.detach().to(**cv).requires_grad_(True) for t in
                    (c.lin_l.weight, c.lin_l.bias, c.lin_r.weight, p[0].weight, p[0].bias))
              for c, p in zip(blk.convs, blk.posts)]

    def step():
        for t in (t for lay in layers for t in lay):
            t.grad = None                   # as a training loop's zero_grad(set_to_none)
        h = x.detach().requires_grad_(True)
        for wl, bl, wr, g, b in layers:
            xj = h.index_select(0, src)
            cnt = torch.zeros(n, dtype=h.dtype, device=h.device).scatter_add_(
                0, dst, torch.ones(dst.numel(), dtype=h.dtype, device=h.device)).clamp(min=1)
            agg = torch.zeros(n, h.size(1), dtype=h.dtype, device=h.device).scatter_add_(
                0, dst.view(-1, 1).expand_as(xj), xj) / cnt.view(-1, 1)
            o = Fn.linear(agg, wl, bl) + Fn.linear(h, wr)
            o = Fn.layer_norm(o, (o.size(1),), g, b, 1e-5)
            h = Fn.dropout(Fn.leaky_relu(o, 0.1), 0.25, training=True)
        h.backward(gout)

    try:
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps
    except torch.cuda.OutOfMemoryError:
        return None
    finally:
        torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# Real-workload lines
# ---------------------------------------------------------------------------
PACKS_PER_BATCH = 32          # main.py:22-26 batch_size
VEHICLES = (200, 300)         # vehicles per pack (rcv.py:14 caps packs at ~300)


def _synthetic_pack(gen, dev, v, feat, radius=30.0, strip=(600.0, 40.0)):
    """One pack as the SageBlock sees it: node features [v, feat] (the fc1 /
    map-context output, grusage.py:165-179) and the radius graph of
    gbuilder.py:85-111 (pairs within `radius` m, both directions, no self
    loops) over positions in a road strip."""
    pos = torch.rand(v, 2, generator=gen, device=dev) * torch.tensor(strip, device=dev)
    d = torch.cdist(pos, pos)
    adj = (d <= radius) & ~torch.eye(v, dtype=torch.bool, device=dev)
    ei = adj.nonzero().t().contiguous()          # i-major like gbuilder.py:92-109
    h = torch.randn(v, feat, generator=gen, device=dev)
    return {"x": h, "edge_index": ei}


def _time_steps(step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    gc.collect()
    gc.disable()        # as timeit does: no collector pauses inside the timed steps
    try:
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps
    finally:
        gc.enable()


def bench_vehicle(args, dev):
    """The vehicle SageBlock [128, 96, 96] (grusage.py:108-110 with the map
    context; main.py:39-46 dropout 0.25, slope 0.1) on collated batches of 32
    packs (main.py:166-167).  Packs are resident on the GPU (dataset.py:77
    loads with map_location=DEVICE); a step = PyG-free collate of 32 fresh
    pack records (sldm_sage.data.collate: feature concat + one fused kernel for
    the offset edge_index, batch / ptr and the batch CSR pair, with one host
    sync for the id check) + SageBlock forward + backward.  8 batches rotate."""
    from sldm_sage import SageBlock
    from sldm_sage.data import collate
    gen = torch.Generator(device=dev).manual_seed(0)
    hd = [128, 96, 96]
    pools = []
    for _ in range(8):
        vs = torch.randint(VEHICLES[0], VEHICLES[1] + 1, (PACKS_PER_BATCH,),
                           generator=torch.Generator().manual_seed(len(pools))).tolist()
        pools.append([_synthetic_pack(gen, dev, v, hd[0]) for v in vs])
    torch.manual_seed(0)
    blk = SageBlock(hd, dropout=0.25, negative_slope=0.1).to(dev).train()
    it = [0]
    edges = [sum(p["edge_index"].size(1) for p in pool) for pool in pools]
    nodes = [sum(p["x"].size(0) for p in pool) for pool in pools]

    def step():
        pool = pools[it[0] % len(pools)]
        it[0] += 1
        b = collate([dict(p) for p in pool])          # fresh records: no cached CSR
        blk.zero_grad(set_to_none=True)                # as a training loop does
        h = b.x.requires_grad_(True)
        out = blk(h, b.edge_index)
        out.backward(torch.ones_like(out))

    t = _time_steps(step, args.warmup, args.steps)
    # Like for like on collated batches: the SageBlock forward + backward alone
    # (batch CSR from collate) and the reference's ATen op sequence (what PyG
    # runs on the batch's edge_index) on the same batches.
    t_ref, t_own = [], []
    for pool in pools[:4]:
        b = collate([dict(p) for p in pool])
        gout = torch.ones(b.x.size(0), hd[-1], device=dev)

        def own(b=b, gout=gout):
            blk.zero_grad(set_to_none=True)
            blk(b.x.detach().requires_grad_(True), b.edge_index).backward(gout)

        t_own.append(_time_steps(own, 2, 10))
        tb = torch_ops_gpu_baseline(blk, b.edge_index, b.x, gout, warmup=2, steps=10)
        if tb:
            t_ref.append(tb)
    # The same training step (dropout on) as ONE captured HIP graph at padded
    # shapes: every batch is written into static buffers (feature rows past the
    # batch zero, the unused tail of edge_index filled with the padding edge
    # (N, N) that the CSR build ignores), and a replay runs the CSR build of that
    # edge_index, the forward and the backward; the dropout seed is a device
    # word advanced inside the graph.
    n_pad, e_pad = max(nodes), max(edges)
    padded = []
    for pool in pools[:4]:
        b = collate([dict(p) for p in pool])
        n, e = b.x.size(0), b.edge_index.size(1)
        xp = torch.zeros(n_pad, hd[0], device=dev)
        xp[:n] = b.x
        eip = torch.full((2, e_pad), n_pad, dtype=torch.int64, device=dev)
        eip[:, :e] = b.edge_index
        gp = torch.zeros(n_pad, hd[-1], device=dev)
        gp[:n] = 1.0
        padded.append((xp, eip, gp))
    sx = padded[0][0].clone().requires_grad_(True)
    sei, sg = padded[0][1].clone(), padded[0][2].clone()
    side_stream = torch.cuda.Stream()
    side_stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side_stream):
        for _ in range(3):
            blk.zero_grad(set_to_none=True)
            sx.grad = None
            blk(sx, sei.clone()).backward(sg)
    torch.cuda.current_stream().wait_stream(side_stream)
    torch.cuda.synchronize()
    blk.zero_grad(set_to_none=True)
    sx.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        blk(sx, sei).backward(sg)
    git = [0]

    def graph_step():
        xp, eip, gp = padded[git[0] % len(padded)]
        git[0] += 1
        with torch.no_grad():
            sx.copy_(xp)
            sei.copy_(eip)
            sg.copy_(gp)
        graph.replay()

    t_graph = _time_steps(graph_step, args.warmup, args.steps)
    e_avg, n_avg = sum(edges) / len(edges), sum(nodes) / len(nodes)
    return {"metric": "edges/sec SageBlock fwd+bwd (vehicle batches)", "value": round(
        e_avg * (len(hd) - 1) / t, 1), "unit": "edges/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic packs: 200-300 vehicles, 30 m radius graph in a 600x40 m strip",
        "config": {"workload": "vehicle SageBlock [128,96,96], 32 packs / batch incl. collate + "
                               "batch CSR", "nodes_per_batch": round(n_avg),
                   "edges_per_batch": round(e_avg), "dropout": 0.25, "negative_slope": 0.1},
        "graphs_per_s": round(PACKS_PER_BATCH / t, 1),
        "sageblock_only_ms": round(statistics.median(t_own) * 1e3, 3),
        "hip_graph": {"ms_per_step": round(t_graph * 1e3, 3),
                      "padded_nodes": n_pad, "padded_edges": e_pad,
                      "what": "three device copies of a padded batch into static buffers + one "
                              "replay of the captured training step (CSR build of the batch's "
                              "edge_index, forward, backward; dropout 0.25 keyed by a device "
                              "word the graph advances); compare with sageblock_only_ms, whose "
                              "CSR comes from collate"},
        "torch_ops_gpu_baseline": ({"ms_per_step": round(statistics.median(t_ref) * 1e3, 3),
                                    "speedup_vs_sageblock_only": round(
                                        statistics.median(t_ref) / statistics.median(t_own), 2),
                                    "note": "reference ATen op sequence on the same collated "
                                            "batches (collate not included; compare with "
                                            "sageblock_only_ms)"}
                                   if t_ref else None)}


def bench_map(args, dev):
    """The lane-map SageBlock [16, 32, 32] (mapencoder.py:18-25,37; main.py:50-52)
    over a static lane graph (CSR cached after the first call, as for the
    registered buffer at mapencoder.py:12): forward + backward per step.
    The lane graph is synthetic: S segments in chains of 20 (successor
    edges both ways) plus nearest-neighbour lane links (gbuilder.py:390-425
    builds the real one; no map file ships with the reference)."""
    from sldm_sage import SageBlock
    S = 4000
    gen = torch.Generator(device=dev).manual_seed(1)
    idx = torch.arange(S, device=dev)
    nxt = idx[(idx % 20) != 19]
    succ = torch.stack([nxt, nxt + 1])
    side = torch.stack([idx[:-20], idx[20:]])
    ei = torch.cat([succ, succ.flip(0), side, side.flip(0)], 1)
    x = torch.randn(S, 16, generator=gen, device=dev)
    torch.manual_seed(0)
    blk = SageBlock([16, 32, 32], dropout=0.25, negative_slope=0.1).to(dev).train()

    def step():
        blk.zero_grad(set_to_none=True)
        xr = x.detach().requires_grad_(True)
        out = blk(xr, ei)
        out.backward(torch.ones_like(out))

    t = _time_steps(step, args.warmup, args.steps)
    E = ei.size(1)

    # The same step as one captured HIP graph (static lane graph, fixed shapes):
    # the operators allocate from the graph's pool and sync nothing, so forward +
    # backward replay as a single launch; the dropout seed is a device word the
    # graph advances, so every replay drops a new mask.
    blk_g = blk
    sx = x.detach().clone().requires_grad_(True)
    sg = torch.ones(S, 32, device=dev)
    side_stream = torch.cuda.Stream()
    side_stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side_stream):
        for _ in range(3):
            blk_g.zero_grad(set_to_none=True)
            sx.grad = None
            blk_g(sx, ei).backward(sg)
    torch.cuda.current_stream().wait_stream(side_stream)
    torch.cuda.synchronize()
    blk_g.zero_grad(set_to_none=True)
    sx.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        blk_g(sx, ei).backward(sg)

    def eager_nodrop():
        blk_g.zero_grad(set_to_none=True)
        xr = x.detach().requires_grad_(True)
        blk_g(xr, ei).backward(sg)

    t_graph = _time_steps(graph.replay, args.warmup, args.steps)
    t_eager = _time_steps(eager_nodrop, args.warmup, args.steps)
    return {"metric": "edges/sec SageBlock fwd+bwd (lane map)", "value": round(E * 2 / t, 1),
            "hip_graph": {"ms_per_step": round(t_graph * 1e3, 3),
                          "eager_ms_per_step_same_block": round(t_eager * 1e3, 3),
                          "what": "forward + backward of the same block (dropout 0.25, a new "
                                  "mask per replay) captured once with torch.cuda.graph and "
                                  "replayed"},
            "unit": "edges/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic lane graph (chains of 20 segments + side links)",
            "config": {"workload": "map SageBlock [16,32,32], static graph, CSR cached",
                       "nodes": S, "edges": E}}


def bench_gru(args, dev):
    """The model's GRU (grusage.py:66-71,160-161): nn.GRU(6 -> 96, 1 layer,
    batch_first) over [N, T=100, 6], N = 32 packs x 300 vehicles, fp32,
    forward + backward of the last hidden state (MIOpen;
    measure before any hand kernel).  Roofline: the gate GEMMs' FLOP against
    the dense fp32 MFMA peak."""
    from sldm_sage import GRU
    N, T, I, H = PACKS_PER_BATCH * VEHICLES[1], 100, 6, 96
    gen = torch.Generator(device=dev).manual_seed(0)
    torch.manual_seed(0)
    ref = torch.nn.GRU(I, H, 1, batch_first=True).to(dev)
    ours = GRU(I, H, 1, batch_first=True).to(dev)
    ours.load_state_dict(ref.state_dict())
    x = torch.randn(N, T, I, generator=gen, device=dev)
    g = torch.randn(N, H, generator=gen, device=dev)

    def stepper(gru):
        def step():
            gru.zero_grad(set_to_none=True)
            _, hl = gru(x)
            hl[-1].backward(g)
        return step

    t = _time_steps(stepper(ours), args.warmup, args.steps)
    t_miopen = _time_steps(stepper(ref), min(args.warmup, 2), min(args.steps, 5))
    flop_fwd = 2.0 * N * T * 3 * (I * H + H * H)
    flop = 3 * flop_fwd                               # fwd + dX/dH + dW
    ach = flop / t / 1e12
    peak = MFMA_PEAK_TFLOPS[torch.float32]
    return {"metric": "GRU fwd+bwd sequences/s (vehicle batch)", "value": round(N / t, 1),
            "unit": "sequences/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic x~N(0,1)",
            "config": {"workload": f"GRU({I}->{H}) over [{N}, {T}, {I}], fwd + bwd of h_n "
                                   "(grusage.py:160-161), sldm_sage.GRU (gru.hip)"},
            "torch_miopen": {"ms_per_step": round(t_miopen * 1e3, 3),
                             "value": round(N / t_miopen, 1)},
            "roofline": {"bound": "mfma", "achieved": round(ach, 3), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(ach / peak, 5), "traffic": None,
                         "note": "gate GEMM FLOP (3 x fwd) / dense fp32 MFMA peak; the T = 100 "
                                 "recurrence serialises [N, 96] x [96, 288] steps"}}


SMALL_WORKLOADS = {"vehicle": bench_vehicle, "map": bench_map, "gru": bench_gru}


def _parallelism(strategy, world):
    if strategy == "replicate":
        return (f"replicated x{world} (the planner found no partition of this graph faster "
                "than one GPU doing all the work: every rank runs the whole block)")
    if strategy == "feature":
        return f"feature-sliced x{world} (all rows, F/{world} columns per rank), RCCL all-to-all"
    return f"dst-partition x{world}, RCCL halo all-to-all"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps (>= 20 after 3 warm-ups, median reported "
                         "as ms_per_step_median_rank0)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS) + sorted(SMALL_WORKLOADS),
                    help="a BASELINE graph config (c1-c5), or a real-workload line: vehicle / map "
                         "(per-batch small graphs, grusage.py:108 / mapencoder.py:18-25) or gru "
                         "(the model's GRU, grusage.py:160-161)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-torch-baseline", action="store_true",
                    help="skip timing the reference's ATen op sequence on the GPU")
    ap.add_argument("--torch-baseline", action="store_true",
                    help="time the reference's ATen op sequence on the GPU also on graphs of "
                         "5e7 edges or more (off by default there: its [E, F] message tensors "
                         "are 51 GB each at C4 and the leg once ended a box with a GPU memory "
                         "fault inside torch's own index_select / scatter_add_ kernels)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host threads of the CPU baseline (default: every usable CPU)")
    ap.add_argument("--cpu-frac", type=int, default=10,
                    help="CPU baseline sample: nodes and edges / this (default E/10)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="override the config's storage dtype (e.g. an fp32 C4 line)")
    ap.add_argument("--graph", default=None, choices=["uniform", "local", "powerlaw"],
                    help="uniform (headline), the locality-structured variant, or power-law "
                         "in-degrees (default for c5)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the partitioned (multi-GPU) path even on one GPU")
    ap.add_argument("--strategy", default="auto",
                    choices=["auto", "halo", "feature", "replicate"],
                    help="multi-GPU partition: destination rows + halo exchange, feature "
                         "slices + layout all-to-alls, or the lower modelled time (default)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one GPU per rank: the measured path) or gloo "
                         "(rehearsal of the N>1 flow with several ranks sharing the GPUs of "
                         "a smaller box; its times are not a measurement)")
    args = ap.parse_args()

    if args.graph is None:
        args.graph = "powerlaw" if args.config == "c5" else "uniform"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.force_dist
    t_start = time.perf_counter()

    def progress(msg):
        # rank 0's progress on stderr before every GPU phase (the JSON line
        # stays the only stdout line): names the phase a fault or hang is in
        if rank == 0:
            free, total = torch.cuda.mem_get_info()
            print(f"[bench] {time.perf_counter() - t_start:7.1f} s  {msg}  [gpu free "
                  f"{free / 2**30:.0f} of {total / 2**30:.0f} GiB, peak "
                  f"{torch.cuda.max_memory_allocated() / 2**30:.1f} GiB]", file=sys.stderr,
                  flush=True)
    if use_dist:
        import torch.distributed as dist
        # one GPU per rank (RCCL); a gloo rehearsal may put several ranks on one GPU
        local_rank %= torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_rank)
    if args.config in SMALL_WORKLOADS:
        if world > 1:
            raise SystemExit(f"--config {args.config} is a single-GPU workload line")
        print(json.dumps(SMALL_WORKLOADS[args.config](args, dev)), flush=True)
        return

    from sldm_sage import SageBlock, graph_cache, ops

    cfg = CONFIGS[args.config]
    if args.dtype is not None:
        want = torch.bfloat16 if args.dtype == "bf16" else torch.float32
        if want != cfg[4]:
            cfg = cfg[:4] + (want, cfg[5].replace("bf16" if want == torch.float32 else "fp32",
                                                   args.dtype))
    n, e, f, L, dtype, desc = cfg

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    link_bps = None
    if use_dist:
        # the node's achieved xGMI rate, measured once, prices the planner's
        # exchanges (RCCL only; gloo rehearsals keep the model constant)
        from sldm_sage.dist import measure_link_bps
        link_bps = measure_link_bps(dev)

    def run(kind, timed_kernels):
        """Build the workload on graph ``kind``, warm up, time args.steps steps
        (max over ranks).  Returns (elapsed_s, kernel summary, dist info, incl)."""
        ei, x = make_graph(n, e, f, dtype, dev, kind=kind)
        progress(f"graph {kind} built")
        torch.manual_seed(0)
        blk = SageBlock([f] * (L + 1), dropout=0.25, negative_slope=0.1).to(dev).train()
        gout = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(2)
                           ).to(dtype)
        dist_info = {}
        if use_dist:
            from sldm_sage.dist import DistSageBlock, plan_partition
            part, plan = plan_partition(ei, n, world, rank, f, x.element_size(),
                                        strategy=args.strategy, link_bps=link_bps)
            progress(f"partitioned: {plan['strategy']}")
            model = DistSageBlock(blk, part)
            x_in = x[part.row_begin:part.row_end].contiguous()
            g_in = gout[part.row_begin:part.row_end].contiguous()
            dist_info = {"strategy": plan["strategy"],
                         "exchange_bytes_per_layer_rank0":
                             part.exchange_bytes_per_layer(f, x.element_size())}
            if "halo_s" not in plan:       # forced strategy: still price every option
                from sldm_sage.dist import estimate_strategies
                plan.update(estimate_strategies(ei, n, world, rank, f, x.element_size(),
                                                link_bps=link_bps))
            dist_info["link_bps_measured"] = link_bps
            dist_info["link_bps_model"] = plan.get("link_bps")
            for k in ("halo_s", "feature_s", "replicate_s"):
                dist_info[f"model_{k[:-2]}_ms_per_layer"] = round(plan[k] * 1e3, 3)
            # the planner's prediction for this run (sldm_sage.dist cost model,
            # fwd + bwd per layer) beside the measured value
            t_pred = plan[f"{plan['strategy']}_s"] * L
            dist_info["model_prediction"] = {"ms_per_step": round(t_pred * 1e3, 3),
                                             "value": round(e * L / t_pred, 1)}
            if plan["strategy"] == "halo":
                hf, hb = part.halo_rows()
                cross = (float((part.fwd.col.long() >= part.num_rows).float().mean())
                         if part.fwd.num_edges else 0.0)

                def resident(split):
                    # fraction of own rows aggregated while the halo exchange is in flight
                    if split is None:
                        return 1.0
                    r, pnd = split.resident.rows.numel(), split.pending.rows.numel()
                    return round(r / max(r + pnd, 1), 4)

                dist_info.update({"halo_rows_fwd_rank0": hf, "halo_rows_bwd_rank0": hb,
                                  "cross_partition_edge_fraction_rank0": round(cross, 4),
                                  "overlap_resident_rows_fwd_rank0": resident(part.fwd_split),
                                  "overlap_resident_rows_bwd_rank0": resident(part.bwd_split)})
            elif plan["strategy"] == "feature":
                dist_info["chunks"] = part.num_chunks
            del ei, x, gout
            torch.cuda.empty_cache()

            def step():
                xr = x_in.detach().requires_grad_(True)
                out = model(xr)
                out.backward(g_in)
                return out
        else:
            def step():
                xr = x.detach().requires_grad_(True)
                out = blk(xr, ei)
                out.backward(gout)
                return out

        progress(f"warm-up: {args.warmup} steps")
        for _ in range(args.warmup):
            blk.zero_grad(set_to_none=True)
            step()
        barrier()
        progress("warm-up done")
        timer = KernelTimer()
        barrier()
        if timed_kernels:
            # inside the timed region only the roofline kernel is bracketed
            # with HIP events (per-op events on every launch cost the small
            # configurations up to 40 % of a step); the per-kernel table comes
            # from the untimed breakdown steps below
            ops.set_timing_hook(timer, names={"gather_fwd"})
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        gc.collect()
        gc.disable()        # as timeit does: no collector pauses inside the timed steps
        t0 = time.perf_counter()
        marks[0].record()
        for i in range(args.steps):
            blk.zero_grad(set_to_none=True)
            step()
            marks[i + 1].record()
        barrier()
        elapsed = time.perf_counter() - t0
        gc.enable()
        progress(f"timed steps done ({elapsed / args.steps * 1e3:.1f} ms/step)")
        step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
        ops.set_timing_hook(None)
        if world > 1:
            from sldm_sage.dist import all_reduce
            tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            elapsed = tt.item()

        kern_all = {}
        if timed_kernels:
            progress("per-kernel breakdown steps")
            # untimed breakdown: every op bracketed, BREAKDOWN_STEPS steps
            t_all = KernelTimer()
            ops.set_timing_hook(t_all)
            for _ in range(BREAKDOWN_STEPS):
                blk.zero_grad(set_to_none=True)
                step()
            ops.set_timing_hook(None)
            barrier()
            kern_all = t_all.summary()

        # CSR-build-inclusive step (N=1: static-graph cache cleared once)
        incl = None
        if world == 1 and not use_dist:
            progress("CSR-inclusive step")
            graph_cache.clear()
            barrier()
            t1 = time.perf_counter()
            blk.zero_grad(set_to_none=True)
            step()
            barrier()
            incl = e * L / (time.perf_counter() - t1)

        # Launch-bound sizes: the same training step (dropout on, a new mask per
        # replay) as one captured HIP graph; the CSR is the cached one.
        captured = None
        if world == 1 and not use_dist and e <= (1 << 20):
            progress("captured step")
            sx = x.detach().clone().requires_grad_(True)
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    blk.zero_grad(set_to_none=True)
                    sx.grad = None
                    blk(sx, ei).backward(gout)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            blk.zero_grad(set_to_none=True)
            sx.grad = None
            hip_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(hip_graph):
                blk(sx, ei).backward(gout)
            t_g = _time_steps(hip_graph.replay, args.warmup, args.steps)
            captured = {"ms_per_step": round(t_g * 1e3, 4), "value": round(e * L / t_g, 1),
                        "what": "forward + backward of the same block and graph captured once "
                                "with torch.cuda.graph and replayed (dropout keyed by a device "
                                "word the graph advances); not the headline value"}
        return elapsed, timer.summary(), dist_info, incl, step_ms, kern_all, captured

    elapsed, kern_timed, dist_info, incl, step_ms, kern, captured = run(args.graph, True)
    variant = None
    if world > 1 and args.graph == "uniform":
        # C4: also the locality-structured variant (block-community
        # graph, cut fraction stated) -- the regime where the exchange overlaps.
        torch.cuda.empty_cache()
        v_el, _, v_info, _, _, _, _ = run("local", False)
        variant = dict(graph="local", value=round(e * L * args.steps / v_el, 1),
                       ms_per_step=round(v_el / args.steps * 1e3, 3), **v_info)
        torch.cuda.empty_cache()

    ms = elapsed / args.steps * 1e3
    value = e * L * args.steps / elapsed
    g = kern_timed.get("gather_fwd")
    roof = None
    if g:
        achieved = g["avg_bytes"] / (g["avg_ms"] * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", PMC_SUMMARY)
        if (args.config == "c4" and args.graph == "uniform" and world == 1
                and dtype == torch.bfloat16 and os.path.exists(pmc)):
            # HBM bytes per launch of this kernel at this workload, from the
            # committed rocprofv3 PMC passes (2*FETCH_SIZE + WRITE_SIZE).
            with open(pmc) as fh:
                traffic = int(json.load(fh)["gather_fwd_c4"]["hbm_bytes_per_launch"])
        roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                    traffic_unit=(f"bytes/launch (PMC, profiles/{PMC_SUMMARY})"
                                  if traffic is not None else
                                  "no PMC pass committed for this workload"),
                    kernel="gather_rows_kernel (forward mean aggregation)",
                    avg_ms=round(g["avg_ms"], 4), launches=g["launches"],
                    bytes_per_launch=int(g["avg_bytes"]))
    # Full-step roofline: T* = (algorithmic bytes of every timed
    # kernel in a step) / HBM peak + (GEMM FLOP of a step) / dense MFMA peak,
    # reported as T*/t (N = 1; at N > 1 the per-rank work is not the whole graph).
    step_bytes = sum(v["avg_bytes"] * v["launches"] for v in kern.values()) / BREAKDOWN_STEPS
    step_roof = None
    if kern and not use_dist:
        flop = 3 * 2.0 * n * 2 * f * f * L        # fwd, dX, dW of [N,2F]x[2F,F] per layer
        # fp32 GEMMs run as six bf16 MFMA products per fp32 product (the default;
        # SLDM_FP32_GEMM=exact selects the fp32 MFMA): price what is issued
        split = dtype == torch.float32 and not os.environ.get("SLDM_FP32_GEMM", "").startswith("e")
        t_mfma = (6 * flop / (MFMA_PEAK_TFLOPS[torch.bfloat16] * 1e12) if split
                  else flop / (MFMA_PEAK_TFLOPS[dtype] * 1e12))
        t_star = step_bytes / (HBM_PEAK_GBS * 1e9) + t_mfma
        t_star_copy = step_bytes / (HBM_COPY_GBS * 1e9) + t_mfma
        step_roof = dict(bytes_per_step=int(step_bytes), flop_per_step=flop,
                         t_star_ms=round(t_star * 1e3, 3),
                         frac=round(t_star / (elapsed / args.steps), 4),
                         frac_vs_measured_copy=round(t_star_copy / (elapsed / args.steps), 4),
                         note="T* = bytes/8 TB/s + FLOP/dense MFMA peak"
                              + (" (fp32 as six bf16 MFMA products: 6 x FLOP at the bf16 peak)"
                                 if split else "")
                              + "; frac_vs_measured_copy prices bytes at the 6.29 TB/s copy "
                                "ceiling")
    kernels = {k: dict(avg_ms=round(v["avg_ms"], 4), launches=v["launches"],
                       gbs=round(v["avg_bytes"] / (v["avg_ms"] * 1e-3) / 1e9, 1))
               for k, v in kern.items()}
    torch_gpu = None
    if (world == 1 and not use_dist and not args.no_torch_baseline
            and (e < 50_000_000 or args.torch_baseline)):
        progress("ATen op-sequence baseline on the GPU")
        ei_b, x_b = make_graph(n, e, f, dtype, dev, kind=args.graph)
        torch.manual_seed(0)
        blk_b = SageBlock([f] * (L + 1), dropout=0.25, negative_slope=0.1)
        g_b = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(2)
                          ).to(dtype)
        t_b = torch_ops_gpu_baseline(blk_b, ei_b, x_b, g_b)
        del ei_b, x_b, g_b
        torch.cuda.empty_cache()
        torch_gpu = ({"value": round(e * L / t_b, 1), "ms_per_step": round(t_b * 1e3, 3),
                      "speedup": round(t_b / (elapsed / args.steps), 2),
                      "what": "the reference's ATen op sequence (PyG 2.7.0 SAGEConv(mean): "
                              "index_select + scatter_add_ + count + linear; LayerNorm, "
                              "LeakyReLU, Dropout) on this GPU, same graph / dtype / weights"}
                     if t_b else {"value": None, "note": "out of memory at this size"})
    if rank == 0:
        base = None
        if world == 1 and not args.no_cpu_baseline:
            progress("CPU baseline (host)")
            cpus = available_cpus()
            base = cpu_baseline(cfg, args.cpu_threads or cpus["usable"], frac=args.cpu_frac)
            base["host"] = cpus
        line = {
            "metric": "edges/sec SageBlock fwd+bwd",
            "value": round(value, 1),
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": {"uniform": "synthetic (uniform random src/dst",
                     "local": "synthetic (locality variant: src in dst's 1/8 block w.p. 0.9",
                     "powerlaw": f"synthetic (dst Zipf a={ZIPF_A} over permuted ids, src uniform"
                     }[args.graph] + ", x~N(0,1), random-init weights)",
            "config": {"workload": desc, "graph": args.graph, "nodes": n, "edges": e, "feat": f,
                       "layers": L, "dropout": 0.25, "negative_slope": 0.1,
                       "parallelism": (_parallelism(dist_info.get("strategy"), world)
                                       if use_dist else "single"), **dist_info},
            "graph_edges_per_s": round(e * args.steps / elapsed, 1),
            "ms_per_step_median_rank0": round(statistics.median(step_ms), 3),
            "value_incl_csr_build": round(incl, 1) if incl else None,
            "step_roofline": step_roof,
            "roofline": roof,
            "kernels": kernels,
            "kernels_from": (f"{BREAKDOWN_STEPS} untimed steps after the timed region, HIP events "
                             "around every launch (inside the timed region only the roofline "
                             "kernel's launches carry events)"),
            "cpu_baseline": base,
            "torch_ops_gpu_baseline": torch_gpu,
        }
        if variant is not None:
            line["locality_variant"] = variant
        if captured is not None:
            line["hip_graph"] = captured
        if use_dist and args.dist_backend != "nccl":
            line["rehearsal"] = (f"{args.dist_backend} backend, ranks sharing "
                                 f"{torch.cuda.device_count()} GPU(s): flow check, not a measurement")
        print(json.dumps(line), flush=True)
    if use_dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
