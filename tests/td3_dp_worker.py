"""Worker for tests/test_gpu_dp.py::test_td3_data_parallel_*: W processes on ONE HIP device
with a gloo process group. Every rank owns its own 4 BipedalWalker-shaped replay envs
(seed 4 + rank, record length 23 + 6 rank, so episodes end at different steps on
different ranks) and ReplayBuffer2
rings. Checks:
  1. one gradient step: the data-parallel critic gradients are the SUM of the ranks' local
     gradients (Keras MSE summed over the union batch), and every rank ends with the same
     weights;
  2. train steps with DIFFERENT per-rank done patterns complete (every rank runs the
     gradient steps of the union of finished episodes, ddpg/agent.py:157-166) and keep the
     weights identical across ranks; the critic Adam step count is gradient_steps x the
     union's finished episodes.
Prints 'TD3 DP OK <rank>'."""
import random
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def make(kind, rank, data_parallel=True, gradient_steps=2):
    from xagents_amd import DDPG, TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n = 4
    # the replay record's last step is terminal: different lengths per rank give different
    # done patterns
    envs = create_envs('BipedalWalker-v3', n, device='cuda', seed=4 + rank, t_rec=23 + 6 * rank)
    kw = dict(seed=7, device='cuda', optimizer_kwargs=dict(learning_rate=1e-3))
    actor = create_model(envs, kind, 'actor_model', **kw)
    critic = create_model(envs, kind, 'critic_model', **kw)
    bufs = create_buffers(kind, 16 * n, 2 * n, n, initial_size=4 * n)
    cls = TD3 if kind == 'td3' else DDPG
    agent = cls(envs, actor, critic, bufs, gradient_steps=gradient_steps, seed=3, quiet=True)
    if not data_parallel:
        agent.distributed, agent.world_size = False, 1
        # the local reference runs the same layer-executor step as the data-parallel ranks
        # (a one-process agent would otherwise take the fused xa_td3_update / xa_td3_act,
        # whose sums run in another order)
        agent.__dict__['_fused'] = None
        agent.__dict__['_fused_act'] = None
    return agent


def gather(t):
    t = t.detach().cpu()
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return parts


def nets(agent):
    out = [agent.actor, agent.critic, agent.target_actor, agent.target_critic]
    if hasattr(agent, 'critic2'):
        out += [agent.critic2, agent.target_critic2]
    return out


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    for kind in ('td3', 'ddpg'):
        # 1. one gradient step: DP gradients vs the sum of local ones
        local = make(kind, rank, data_parallel=False)
        dp = make(kind, rank)
        for ag in (local, dp):
            np.random.seed(50 + rank)
            random.seed(50 + rank)
            ag.fill_buffers()
        for ag in (local, dp):
            np.random.seed(60 + rank)
            random.seed(60 + rank)
            ag.update_weights(1)
        torch.cuda.synchronize()
        # (the actor gradient runs through the critic AFTER its step, which differs
        # between the data-parallel and the local agent, so only the critics compare)
        grads = [('g_critic', local.g_critic, dp.g_critic)]
        if kind == 'td3':
            grads.append(('g_critic2', local.g_critic2, dp.g_critic2))
        for name, lg, dg in grads:
            want = torch.stack(gather(lg)).double().sum(0).float()
            torch.testing.assert_close(dg.cpu(), want, rtol=1e-5, atol=1e-7, msg=name)
        for m in nets(dp):
            parts = gather(m.theta)
            for p in parts[1:]:
                assert torch.equal(p, parts[0]), f'{kind}: ranks disagree after a gradient step'
        # 2. train steps with different per-rank done patterns
        np.random.seed(70 + rank)
        random.seed(70 + rank)
        dp.total_rewards.clear()
        dp.games = 0
        it0 = int(dp.critic.optimizer.iterations.item())
        for _ in range(60):
            dp.train_step()
        dp._drain_episode_stats()
        torch.cuda.synchronize()
        games = gather(torch.tensor([dp.games]))
        assert len({int(g) for g in games}) > 1 or world == 1, 'done patterns did not differ'
        it = int(dp.critic.optimizer.iterations.item()) - it0
        assert it == 2 * int(sum(int(g) for g in games)) and it > 0, (it, games)
        for m in nets(dp):
            parts = gather(m.theta)
            for p in parts[1:]:
                assert torch.equal(p, parts[0]), f'{kind}: ranks disagree after train steps'
        its = gather(dp.critic.optimizer.iterations)
        assert all(torch.equal(i, its[0]) for i in its)
    print(f'TD3 DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
