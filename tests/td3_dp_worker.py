"""Worker for tests/test_gpu_dp.py::test_td3_data_parallel_*: W processes on ONE HIP device
with a gloo process group. Every rank owns its own 4 BipedalWalker-shaped replay envs
(seed 4 + rank, record length 23 + 6 rank, so episodes end at different steps on
different ranks) and ReplayBuffer2 rings. XA_TEST_TD3_PATH picks the gradient step:
'fused' (xa_td3_update in its data-parallel stages: critics' gradients -> all-reduce ->
critics' Adam + actor gradient -> all-reduce -> actor Adam) or 'executor' (the layer
executor's launches). Checks:
  1. one gradient step: the data-parallel critic gradients are the SUM of the ranks' local
     gradients (same path, one process each; Keras MSE summed over the union batch), every
     rank ends with the same weights;
  2. the oracle leg: the data-parallel raw gradients of both critics and of the actor
     (through the updated critic 1) against the float64 restatement (oracle/nets_f64.py)
     on the UNION of the ranks' sampled batches, at 1e-4 relative
     (xagents/ddpg/agent.py:87-127, td3/agent.py:66-110 on one process holding every env);
  3. train steps with DIFFERENT per-rank done patterns complete (every rank runs the
     gradient steps of the union of finished episodes, ddpg/agent.py:157-166) and keep the
     weights identical across ranks; the critic Adam step count is gradient_steps x the
     union's finished episodes.
Prints 'TD3 DP OK <rank>'."""
import os
import random
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'oracle'))
FUSED = os.environ.get('XA_TEST_TD3_PATH', 'fused') == 'fused'


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
    if FUSED:
        assert agent._fused_args() is not None and agent._fused_act_args() is not None
    else:
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


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def _rel(got, want):
    return float(np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30))


def oracle_leg(kind, dp, before):
    """The DP step's raw gradients vs float64 on the union of the ranks' batches."""
    import nets_f64 as O
    twin = kind == 'td3'
    th = dict(zip(('actor', 'critic', 'target_actor', 'target_critic', 'critic2',
                   'target_critic2'), before))
    cat = lambda t: torch.cat(gather(t)).double().numpy()  # noqa: E731
    s, a, r, d, s2 = (cat(x) for x in (dp.s, dp.a, dp.r, dp.d, dp.s2))
    fw = lambda m, w, x: O.forward(m.layers, w, x, m.input_shape)  # noqa: E731
    out = lambda m, res: res[1][m.outputs[0]]  # noqa: E731
    ta = out(dp.target_actor, fw(dp.target_actor, th['target_actor'], s2))
    if twin:
        ta = np.clip(ta + cat(dp.noise), -1, 1)
    s2a2 = np.concatenate([s2, ta], 1)
    tcs = [('target_critic', dp.target_critic)] + ([('target_critic2', dp.target_critic2)]
                                                    if twin else [])
    tvs = [out(m, fw(m, th[k], s2a2)) for k, m in tcs]
    tv = np.minimum(*tvs) if twin else tvs[0]
    y = r[:, None] + (1 - d[:, None]) * np.float64(np.float32(dp.gamma)) * tv
    sa = np.concatenate([s, a], 1)
    crit = [('critic', dp.critic, dp.g_critic)] + ([('critic2', dp.critic2, dp.g_critic2)]
                                                   if twin else [])
    for k, m, gd in crit:
        x64, o = fw(m, th[k], sa)
        g = O.backward(m.layers, th[k], x64, o, {m.outputs[0]: 2 * (o[m.outputs[0]] - y)})
        e = _rel(_np(gd), g)
        assert e < 1e-4, f'{kind}: DP {k} gradient vs f64 on the union batch {e:.2e}'
    # the actor: each rank's loss is its local -mean Q (1 / B per row), the all-reduced
    # gradient their sum, through the UPDATED critic 1 (identical on every rank)
    B = dp.batch_size
    act = dp.actor
    xa, oa = fw(act, th['actor'], s)
    spa = np.concatenate([s, oa[act.outputs[0]]], 1)
    c1 = _np(dp.critic.theta)
    xc, oc = fw(dp.critic, c1, spa)
    _, dx = O.backward(dp.critic.layers, c1, xc, oc,
                       {dp.critic.outputs[0]: -np.ones((len(s), 1)) / B}, want_input_grad=True)
    ga = O.backward(act.layers, th['actor'], xa, oa, {act.outputs[0]: dx[:, s.shape[1]:]})
    e = _rel(_np(dp.g_actor), ga)
    assert e < 1e-4, f'{kind}: DP actor gradient vs f64 on the union batch {e:.2e}'


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
        before = [_np(m.theta) for m in nets(dp)]
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
        # 2. the oracle leg on the union batch
        oracle_leg(kind, dp, before)
        # 3. train steps with different per-rank done patterns
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
        if FUSED:
            assert int(dp._fused_status.item()) == 0
    print(f'TD3 DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
