"""Data-parallel arithmetic of the update, world size 2 over gloo on the CPU.

Each rank holds half of a PPO minibatch. The multi-GPU path
all-reduces the advantage sums, normalises with the global mean / population std
(ppo/agent.py:180-183), scales each rank's loss by 1 / (local count * world) and
all-reduces the gradient. That must equal the single-process gradient of the union
minibatch. The float64 oracle stands in for the kernels; the host half of the
contract (PPO's launch arguments under an initialised process group) is checked on
an agent built on the CPU device (no kernel runs).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _shard_data(n=64, obs_dim=4, A=2, seed=7):
    rng = np.random.default_rng(seed)
    sys.path.insert(0, str(ROOT / 'oracle'))
    import oracle as O
    theta = rng.normal(0, 0.3, 4675)
    obs = rng.normal(0, 1, (n, obs_dim))
    act = rng.integers(0, A, n)
    ret = rng.normal(0, 1, n)
    oldv = rng.normal(0, 1, n)
    oldlp = O.log_softmax(O.forward_f64(theta, obs, obs_dim, A)[3])[np.arange(n), act]
    oldlp = oldlp + rng.normal(0, 0.05, n)
    return theta, obs, act, ret, oldv, oldlp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        sys.path.insert(0, str(ROOT / 'oracle'))
        import oracle as O
        theta, obs, act, ret, oldv, oldlp = _shard_data()
        n = obs.shape[0]
        sl = slice(rank * n // world, (rank + 1) * n // world)
        adv_raw = ret[sl] - oldv[sl]
        sums = torch.tensor([adv_raw.sum(), (adv_raw ** 2).sum()], dtype=torch.float64)
        dist.all_reduce(sums)
        count = n // world
        mean = sums[0].item() / (count * world)
        std = np.sqrt(max(sums[1].item() / (count * world) - mean * mean, 0.0))
        adv = (adv_raw - mean) / (std + 1e-8)
        _, g_local = O.ac_loss_grad_f64(theta, obs[sl], act[sl], ret[sl], oldv[sl], 2, 'ppo',
                                        old_logp=oldlp[sl], advantages=adv)
        # the oracle averages over the local count; the kernel's loss scale is
        # 1 / (count * world), i.e. the local mean divided by world
        g = torch.tensor(g_local / world, dtype=torch.float64)
        dist.all_reduce(g)
        # host contract of the fused PPO path under a process group
        from xagents_amd import PPO
        from xagents_amd.envs import ReplayVecEnv
        from xagents_amd.utils.common import create_model
        envs = ReplayVecEnv('CartPole-v1', 4, t_rec=64, seed=55 + rank, device='cpu')
        model = create_model(envs, 'ppo', 'model', seed=55, device='cpu')
        agent = PPO(envs, model, n_steps=8, seed=55, quiet=True, use_graph=False)
        args = [(a.loss_scale, a.adv_count) for a in agent._gargs_list]
        q.put((rank, g.numpy(), agent.world_size, agent.mini_batch_size, args,
               model.theta.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_world2_gradient_equals_union_gradient():
    sys.path.insert(0, str(ROOT / 'oracle'))
    import oracle as O
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    theta, obs, act, ret, oldv, oldlp = _shard_data()
    adv = O.normalize_advantages(ret, oldv)
    _, g_union = O.ac_loss_grad_f64(theta, obs, act, ret, oldv, 2, 'ppo', old_logp=oldlp,
                                    advantages=adv)
    for rank, g, ws, mb, args, theta_r in res:
        assert ws == world
        np.testing.assert_allclose(g, g_union, rtol=1e-10, atol=1e-14)
        # every minibatch launch scales by 1/(count*world) and normalises with the
        # global count
        assert all(ls == pytest.approx(1.0 / (mb * world)) and ac == mb * world
                   for ls, ac in args)
    # parameters were broadcast from rank 0
    np.testing.assert_array_equal(res[0][5], res[1][5])


def _plateau_worker(rank, world, port, q):
    """Two plateau reductions inside one DP sync window, then _dp_sync: every rank ends
    with lr0 * factor^2 (the reference compounds reductions, xagents/base.py:277-284) and
    rank 0's stop decision."""
    import time
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from xagents_amd import PPO
        from xagents_amd.envs import ReplayVecEnv
        from xagents_amd.utils.common import create_model
        envs = ReplayVecEnv('CartPole-v1', 4, t_rec=64, seed=55 + rank, device='cpu')
        model = create_model(envs, 'ppo', 'model', seed=55, device='cpu',
                             optimizer_kwargs=dict(learning_rate=1e-3))
        agent = PPO(envs, model, n_steps=8, seed=55, quiet=True, use_graph=False,
                    plateau_reduce_factor=0.5, plateau_reduce_patience=1,
                    divergence_monitoring_steps=1)
        agent.steps, agent.last_reset_time = 100, time.perf_counter()
        agent.total_rewards.extend([1.0, 2.0])
        agent.best_reward = 10.0
        agent.mean_reward = 1.5
        for _ in range(2):  # two plateaus before the sync
            agent.update_metrics()
            agent.mean_reward = 1.5
        lr_before = model.optimizer.learning_rate
        stop = agent._dp_sync(stop_local=rank == 0)
        q.put((rank, lr_before, model.optimizer.learning_rate, stop, agent.early_stop_count))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_plateau_reductions_compound_within_a_sync_window():
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_plateau_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lr_before, lr_after, stop, early in res:
        assert lr_before == pytest.approx(1e-3)  # applied only at the sync
        assert lr_after == pytest.approx(1e-3 * 0.25), lr_after
        assert stop is True  # rank 0's decision, on every rank
        assert early == 2
