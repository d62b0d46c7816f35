"""The C ABI driven by a non-Python host (sldm-gnn_amd/examples/abi_host.cpp,
built by __graft_entry__.build()): CSR build, mean gather and transpose
gather from plain C++ + the HIP runtime, checked bit for bit against the
program's own host restatement of the reference's order; then (up to 2^20
edges) the same launches recorded with hipStreamBeginCapture and replayed on
new edge lists padded with (N, N) edges, and a LayerNorm + dropout launch
recorded with a device seed word (sldm_set_dropout_seed_source).  Run as a
child process (never exec'd from this GPU-initialised process)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "sldm-gnn_amd", "examples", "abi_host")


@pytest.mark.gpu
@pytest.mark.parametrize("args", [[], ["1000", "0", "256"], ["3001", "50000", "96"],
                                  ["20000", "300000", "256"]])
def test_abi_host_program(args):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build()")
    r = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "DIFFERS" not in r.stdout, r.stdout
