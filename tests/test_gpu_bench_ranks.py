"""Rehearsal of bench.py's N > 1 flow with several ranks on one GPU.

The driver runs ``python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N`` on a whole 8-GPU node over RCCL; this box has one GPU, and RCCL
needs one GPU per rank.  Here the same launcher starts 4 ranks that share
cuda:0 and carry the collectives over gloo (``--dist-backend gloo``): the
planner's max-reduce, the partition setup, DistSageBlock's exchanges, the
locality-variant second run, the max-over-ranks timing and rank 0's JSON line
all run as at N > 1.  The times are not a measurement (the line says so).

Opt-in (SLDM_REHEARSAL=1): with several ranks sharing one GPU, runs passed
(8 ranks, twice) but one 8-rank run ended in a HIP runtime abort of one rank
during a torch reduction and one 4-rank run hung (its peers waiting in gloo);
the cause is not determined, so the rehearsal stays out of the default GPU
suite.  The multi-rank protocol is covered by the CPU gloo tests
(tests/test_dist_cpu.py, W up to 8) and by tests/test_gpu_dist.py (2 ranks
on the GPU).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("SLDM_REHEARSAL") != "1",
                    reason="multi-rank-on-one-GPU rehearsal is opt-in (SLDM_REHEARSAL=1)")
@pytest.mark.parametrize("strategy", ["auto", "halo", "feature"])
def test_bench_multi_rank_gloo(strategy):
    world = 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", "c2",
           "--steps", "2", "--warmup", "1", "--dist-backend", "gloo", "--strategy", strategy]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    hsa = [ln for ln in r.stderr.splitlines() if "HSA_STATUS" in ln or "aborting" in ln]
    assert r.returncode == 0, "\n".join(hsa) + "\n" + r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["steps"] == 2 and line["value"] > 0
    assert "rehearsal" in line
    cfg = line["config"]
    if strategy != "auto":
        assert cfg["strategy"] == strategy
    assert cfg["strategy"] in ("halo", "feature", "replicate")
    assert cfg["parallelism"] != "single"
    lv = line["locality_variant"]
    assert lv["graph"] == "local" and lv["value"] > 0
