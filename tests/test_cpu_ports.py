"""CPU tests of bench.py's CPU-port baselines (oracle/cpu_trpo.py, oracle/cpu_td3.py) and
of bench.py's FLOP constant: one short timed sample each, finite weights afterwards."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'oracle'))


def test_mlp_forward_flops_match_survey():
    import bench
    assert bench.mlp_fwd_flops() == 9088  # F = 9,088 FLOP per sample


def test_cpu_trpo_port_runs():
    import cpu_trpo
    from xagents_amd.envs import record_transitions
    rec = record_transitions(4, 256, (4,), np.float32, seed=1)
    np.random.seed(0)
    value, info = cpu_trpo.time_trpo(rec, seconds=0.0, threads=2, n_steps=32)
    assert value > 0 and info['train_steps'] == 1 and info['n_envs'] == 4


def test_cpu_td3_port_runs():
    import cpu_td3
    from xagents_amd.envs import record_transitions
    rec = record_transitions(8, 256, (24,), np.float32, seed=1, mean_episode=4)
    np.random.seed(0)
    agent = cpu_td3.CpuTD3(rec, threads=2)
    agent.fill(8)
    for _ in range(20):
        agent.train_step()
    assert agent.opts[1].t > 0  # some episodes ended and ran gradient steps
    assert all(torch.isfinite(p).all() for p in agent.actor + agent.critic1)


def test_cpu_acer_port_runs():
    import cpu_cnn
    from xagents_amd.envs import record_transitions
    rec = record_transitions(2, 16, (84, 84, 1), np.uint8, seed=1)
    np.random.seed(0)
    agent = cpu_cnn.CpuACER(rec, n_steps=2, threads=2, replay_ratio=1)
    before = [p.detach().clone() for p in agent.params]
    agent.train_step()
    agent.train_step()
    assert agent.steps == 2 * 2 * 2 and agent.t >= 2
    assert all(torch.isfinite(p).all() for p in agent.params)
    assert any(not torch.equal(a, b) for a, b in zip(before, agent.params))
