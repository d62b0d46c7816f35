"""Rehearsal of bench.py's N > 1 flow with several ranks on one GPU.

The driver runs ``python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N`` on a whole 8-GPU node over RCCL; this box has one GPU, and RCCL
needs one GPU per rank.  Here the same launcher starts 4 ranks that share
cuda:0 and carry the collectives over gloo (``--dist-backend gloo``): the
planner's max-reduce, the partition setup, DistSageBlock's exchanges, the
locality-variant second run, the max-over-ranks timing and rank 0's JSON line
all run as at N > 1.  The times are not a measurement (the line says so).

An earlier form of this flow once aborted in a rank (HIP runtime, during a
torch reduction, 8 ranks) and once hung in gloo (4 ranks).  What those runs
had in common was gloo's own CUDA path: device tensors handed to gloo collectives (its
internal streams and pinned staging, racing the kernels on the current
stream and the caching allocator), plus a halo-exchange skip decided per
rank.  sldm_sage.dist now stages every gloo collective on device tensors
through host memory explicitly (``.cpu()`` waits for the producing stream)
and decides the halo skip globally at partition time.  Each rank's full
stdout/stderr is kept (torchrun --log-dir) and reported on failure.
"""
import glob
import json
import os
import shutil
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_logs(log_dir):
    """Every rank's full stdout / stderr from torchrun's --log-dir tree."""
    out = []
    for dirpath, _, files in sorted(os.walk(log_dir)):
        for fn in sorted(files):
            p = os.path.join(dirpath, fn)
            with open(p, errors="replace") as fh:
                out.append(f"===== {os.path.relpath(p, log_dir)} =====\n{fh.read()}")
    return "\n".join(out)


def _rank0_stdout(log_dir):
    files = glob.glob(os.path.join(log_dir, "**", "0", "stdout.log"), recursive=True)
    assert len(files) == 1, _rank_logs(log_dir)
    with open(files[0]) as fh:
        return fh.read()


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["auto", "halo", "feature"])
def test_bench_multi_rank_gloo(strategy):
    world = 4
    log_dir = os.path.join(ROOT, "gpurun_out", f"rehearsal_{strategy}")
    shutil.rmtree(log_dir, ignore_errors=True)
    os.makedirs(log_dir, exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           f"--log-dir={log_dir}", "--redirects=3",
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", "c2",
           "--steps", "2", "--warmup", "1", "--dist-backend", "gloo", "--strategy", strategy]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (f"rc={r.returncode}\n--- launcher stdout\n{r.stdout}\n"
                               f"--- launcher stderr\n{r.stderr}\n{_rank_logs(log_dir)}")
    # rank 0's stdout is redirected into the log tree
    r = type(r)(r.args, r.returncode, _rank0_stdout(log_dir), r.stderr)
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
