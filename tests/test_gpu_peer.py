"""Peer all-reduce (csrc/comm.hip) with W processes sharing the one test GPU: IPC block
exchange, rank-ordered sums bit-exact vs the gloo-gathered inputs, hipGraph replay,
and the bounded-wait timeout path (tests/peer_worker.py)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 4])
def test_peer_allreduce_processes_on_one_gpu(device, world):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={world}', '--master-addr=127.0.0.1',
           f'--master-port={_free_port()}', str(ROOT / 'tests' / 'peer_worker.py')]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110,
                         cwd=str(ROOT))
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    for r in range(world):
        assert f'PEER OK {r}' in out, out[-4000:]
