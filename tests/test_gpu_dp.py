"""Data-parallel paths with W processes sharing the one test GPU over a gloo group
(SURVEY.md 8e): the fused PPO step equals one process on the union of the shards, TD3 /
DDPG ranks with different done patterns run the same gradient steps (no collective
mismatch), and a stalled peer exchange falls back to the process group's all-reduce."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _run(worker, world, tag, extra_env=None, timeout=110):
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='1',
               **(extra_env or {}))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={world}', '--master-addr=127.0.0.1', f'--master-port={port}',
           str(ROOT / 'tests' / worker)]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout,
                         cwd=str(ROOT))
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    for line in out.splitlines():  # the workers' measured deviations (pytest -s shows them)
        if ' rel ' in line or 'flips' in line:
            print(line)
    for r in range(world):
        assert f'{tag} {r}' in out, out[-4000:]


@pytest.mark.parametrize('mode,world,shape', [('persistent', 2, None), ('chain', 2, None),
                                              ('persistent', 4, None),
                                              ('persistent', 2, 'headline')])
def test_ppo_data_parallel_equals_union(device, mode, world, shape):
    """xagents/ppo/agent.py:157-191 on the union of W shards vs the W-rank data-parallel
    step (advantage sums and gradients exchanged), tests/ppo_dp_worker.py: the persistent
    update exchanging inside its launch (W = 2 and 4), the per-minibatch chain, and the
    metric's per-rank shape (16 envs x 128 steps: the fixed-shape DP instantiation)."""
    env = {'XA_PPO_UPDATE': mode}
    if shape:
        env['XA_TEST_DP_SHAPE'] = shape
    _run('ppo_dp_worker.py', world, 'PPO DP OK', extra_env=env)


@pytest.mark.parametrize('world,bucket_mb,seed', [(2, None, 55), (2, None, 155), (2, None, 255),
                                                  (4, None, 55), (4, None, 155), (4, None, 255),
                                                  (2, '0', 55)])
def test_cnn_ppo_data_parallel_equals_union(device, world, bucket_mb, seed):
    """BASELINE configs[3]'s path: PPO with the CNN actor-critic on the layer executor,
    data parallel over W ranks (advantage statistics all-reduced once per train step, the
    77 MB gradient all-reduced per minibatch in buckets overlapping the conv backward),
    equal to the union of the shards (tests/cnn_ppo_dp_worker.py; xagents/ppo/agent.py:
    157-191): theta within 2e-5 of the update's norm of a float64 replay of the union train
    step that adopts the ranks' ReLU gates and clip-branch decisions (one bound, no flip
    escape), plus the f32 single-process union run (rollout equality; its theta deviation
    reported). Record seeds 55 / 155 / 255 at W = 2 and 4. bucket_mb '0': one bucket per
    layer (every layer's slice goes out as soon as it is final)."""
    env = {'XA_DP_SEED': str(seed)}
    if bucket_mb:
        env['XA_TEST_BUCKET_MB'] = bucket_mb
    _run('cnn_ppo_dp_worker.py', world, 'CNN DP OK', extra_env=env, timeout=200)


def test_ppo_data_parallel_xcd_local_equals_union(device):
    """The placement a rank that owns its GPU uses (XA_PPO_PLACE_LOCAL: the update's G
    workgroups elected on one XCD, hand-offs in that L2, cross-rank slices over the IPC
    exchange blocks), here with 2 ranks on the one test GPU: the worker's minibatches make
    G = 2, so both ranks' 8 x G launched workgroups are co-resident and neither election
    can strand the other's. Must equal the union step like the spread placement."""
    _run('ppo_dp_worker.py', 2, 'PPO DP OK',
         extra_env={'XA_PPO_UPDATE': 'persistent', 'XA_PPO_PLACE': 'local'})


def test_ppo_persistent_update_waits_for_late_ranks(device):
    """Launch skew between ranks (one process per GPU launches with its own host-side
    delay): rank 1 sleeps 0.5 s on the host before each of 3 train steps, so rank 0's
    persistent update spins inside its launch until rank 1's pushes arrive. Every step
    must complete without the timeout abort (status word 0), equal the union step, and
    leave both ranks with identical parameters."""
    _run('ppo_dp_worker.py', 2, 'PPO DP OK',
         extra_env={'XA_PPO_UPDATE': 'persistent', 'XA_TEST_SKEW_S': '0.5',
                    'XA_TEST_STEPS': '3'})


@pytest.mark.parametrize('path', ['fused', 'executor'])
def test_td3_data_parallel_done_patterns(device, path):
    """TD3 and DDPG at W = 2 (BASELINE configs[4]'s data-parallel step) on both gradient-step
    paths: DP gradients = the rank sum of local ones, vs float64 on the union batch, and
    different per-rank done patterns (ddpg/agent.py:157-166), tests/td3_dp_worker.py. The
    grid is the agent's default: ranks sharing the one test GPU each cap their persistent
    launches at 3/4 of their share of the CUs (DDPG._shared_blocks), so both
    ranks' launches are resident together."""
    _run('td3_dp_worker.py', 2, 'TD3 DP OK',
         extra_env={'XA_TEST_TD3_PATH': path}, timeout=200)


def test_peer_stall_falls_back_to_rccl(device):
    """A rank stalling past the peer-exchange timeout in the middle of training is detected
    by the periodic health check on every rank (tests/peer_stall_worker.py)."""
    _run('peer_stall_worker.py', 2, 'STALL OK',
         extra_env={'XA_PEER_TIMEOUT_S': '0.5', 'XA_PEER_CHECK_STEPS': '4',
                    'XA_PPO_UPDATE': 'chain'})
