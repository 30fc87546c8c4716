"""GPU tests of the BipedalWalker-v3 device stand-in (csrc/walker.hip; SURVEY.md 8(f)
rank 4): the kernel against its C restatement (oracle/xa_oracle.c xo_walker_step) bit for
bit over long random-action runs with falls and resets; TD3 / DDPG and Gaussian PPO train
on it through the agents' own env-step paths; play() scores a game the oracle replays.
gym's Box2D BipedalWalker is absent, so the dynamics themselves are parity-unpinned."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step_dev(env_state, episode, actions, seed, act_ld=4, reset=False):
    from xagents_amd._lib import XaWalkerStepArgs, call, stream
    n = env_state.shape[0]
    a = XaWalkerStepArgs()
    a.n_envs, a.state, a.episode = n, env_state.data_ptr(), episode.data_ptr()
    a.seed, a.reset_only = seed, int(reset)
    post = torch.empty(n, 24, device=env_state.device)
    a.out_post = post.data_ptr()
    out = None
    if not reset:
        out = (torch.empty(n, 24, device=env_state.device),
               torch.empty(n, device=env_state.device), torch.empty(n, device=env_state.device))
        a.actions, a.act_ld = actions.data_ptr(), act_ld
        a.out_obs, a.out_rew, a.out_done = (t.data_ptr() for t in out)
    call('xa_walker_step', ctypes.byref(a), stream())
    return post, out


def test_walker_kernel_bit_exact_vs_oracle(device):
    import oracle
    n, steps, seed, ld = 37, 700, 123456789, 6
    rng = np.random.default_rng(0)
    st = torch.zeros(n, 18, device=device)
    ep = torch.zeros(n, dtype=torch.int32, device=device)
    hs, he = np.zeros((n, 18), np.float32), np.zeros(n, np.int32)
    post, _ = _step_dev(st, ep, None, seed, reset=True)
    _, hpost, _, _ = oracle.walker_step(hs, he, None, seed, reset_only=True)
    assert np.array_equal(post.cpu().numpy(), hpost)
    dones = 0
    for t in range(steps):
        # rows of 6 floats, 4 used (a strided action buffer); some beyond [-1, 1]
        act = rng.uniform(-1.3, 1.3, (n, ld)).astype(np.float32)
        post, (obs, rew, done) = _step_dev(st, ep, torch.from_numpy(act).to(device), seed, ld)
        hobs, hpost, hrew, hdone = oracle.walker_step(hs, he, act[:, :4], seed)
        assert np.array_equal(obs.cpu().numpy(), hobs), f'obs differ at step {t}'
        assert np.array_equal(post.cpu().numpy(), hpost), f'post obs differ at step {t}'
        assert np.array_equal(rew.cpu().numpy(), hrew), f'rewards differ at step {t}'
        assert np.array_equal(done.cpu().numpy(), hdone), f'dones differ at step {t}'
        dones += int(hdone.sum())
    assert np.array_equal(st.cpu().numpy(), hs) and np.array_equal(ep.cpu().numpy(), he)
    assert dones > 0  # falls (reward -100) and resets were exercised
    assert np.all(np.isfinite(hs))


@pytest.mark.parametrize('kind', ['td3', 'ddpg'])
def test_td3_ddpg_train_on_walker_dynamics(device, kind):
    import oracle
    from xagents_amd import DDPG, TD3
    from xagents_amd.envs import WalkerVecEnv, create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n = 8
    envs = create_envs('BipedalWalker-v3', n, mode='dynamics', device=device, seed=4)
    assert isinstance(envs, WalkerVecEnv)
    kw = dict(seed=7, device=device)
    actor = create_model(envs, kind, 'actor_model', **kw)
    critic = create_model(envs, kind, 'critic_model', **kw)
    bufs = create_buffers(kind, 64 * n, 2 * n, n, initial_size=8 * n)
    agent = (TD3 if kind == 'td3' else DDPG)(envs, actor, critic, bufs, seed=3, quiet=True,
                                             gradient_steps=1)
    agent.fill_buffers()
    for _ in range(40):
        agent.train_step()
    torch.cuda.synchronize()
    for m in (agent.actor, agent.critic):
        assert torch.isfinite(m.theta).all()
    assert agent.steps == 40 * n
    # the ring holds walker transitions: stored states are walker observations
    ring_obs = agent.replay.states[:, :8].reshape(-1, 24).cpu().numpy()
    assert np.all(np.isfinite(ring_obs)) and np.any(ring_obs[:, 14:] > 0)
    # play(): the actor's noise-free actions replayed through the oracle give the same score
    recorded = []
    f = agent._play_actions

    def rec():
        a = f()
        recorded.append(a.clone())
        return a
    agent._play_actions = rec
    he = envs.episode.cpu().numpy().astype(np.int32)  # play's reset keeps the counters
    total = agent.play(max_steps=300)
    hs = np.zeros((n, 18), np.float32)
    oracle.walker_step(hs, he, None, envs.walker_seed, reset_only=True)
    ref, steps = 0.0, 0
    for a in recorded:  # the reference's play loop (xagents/base.py:625-653) on env 0
        if steps >= 300:
            break
        _, _, r, d = oracle.walker_step(hs, he, a.cpu().numpy(), envs.walker_seed)
        ref += float(r[0])
        if d[0]:
            break
        steps += 1
    assert total == pytest.approx(ref, rel=0, abs=1e-3)


def test_ppo_gaussian_rollout_steps_walker_with_its_actions(device):
    """Gaussian PPO on the dynamics env (executor path): every rollout step hands its
    sampled actions (env-major rows, stride T x 4) to the walker; the recorded observations
    equal the oracle stepped with those actions."""
    import oracle
    from xagents_amd import PPO
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_model
    n, T = 6, 16
    envs = create_envs('BipedalWalker-v3', n, mode='dynamics', device=device, seed=9)
    model = create_model(envs, 'ppo', 'model', seed=3, device=device)
    agent = PPO(envs, model, n_steps=T, seed=8, quiet=True, ppo_epochs=1, mini_batches=2)
    assert agent.executor_path and agent.gaussian
    hs = agent.envs.walker_state.cpu().numpy().copy()
    he = agent.envs.episode.cpu().numpy().copy()
    agent._executor_rollout()
    torch.cuda.synchronize()
    acts = agent.b_act.cpu().numpy()          # [N, T, 4]
    obs = agent.obs_buf.cpu().numpy()         # [T + 1, N, 24]: step t's policy input
    rew = agent.b_rew.cpu().numpy()
    for t in range(T):
        o, _, r, _ = oracle.walker_step(hs, he, acts[:, t], envs.walker_seed)
        assert np.array_equal(obs[t + 1], o), f'step {t}'
        assert np.array_equal(rew[:, t], r), f'step {t}'
    agent.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(model.theta).all()
