"""The RCCL fallback of the data-parallel train step is captured into the train-step
hipGraph: one rank on the nccl backend, peer path off, graph vs eager
bit-identical (tests/rccl_capture_worker.py)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def test_rccl_chain_step_is_captured_and_equals_eager(device):
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='1',
               XA_PEER_ALLREDUCE='0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', f'--master-port={port}',
           str(ROOT / 'tests' / 'rccl_capture_worker.py')]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=str(ROOT))
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert 'RCCL CAPTURE OK 0' in out, out[-4000:]
    print([ln for ln in out.splitlines() if ln.startswith('RCCL step ms')])
