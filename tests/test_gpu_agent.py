"""GPU tests of the fused PPO / A2C train step through the agent surface."""
import numpy as np
import oracle
import pytest
import torch

pytestmark = pytest.mark.gpu


def make_agent(cls='ppo', n_envs=16, n_steps=32, seed=7, use_graph=True, t_rec=200, **kw):
    from xagents_amd import A2C, PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model

    envs = ReplayVecEnv('CartPole-v1', n_envs, t_rec=t_rec, seed=seed, device='cuda')
    model = create_model(envs, cls, 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=seed, device='cuda')
    agent_cls = PPO if cls == 'ppo' else A2C
    return agent_cls(envs, model, n_steps=n_steps, seed=seed, quiet=True, use_graph=use_graph,
                     **kw)


def test_graph_replay_equals_eager(device):
    a = make_agent(use_graph=True)
    b = make_agent(use_graph=False)
    for _ in range(4):
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert a._graph is not None
    np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())
    np.testing.assert_array_equal(a.b_act.cpu().numpy(), b.b_act.cpu().numpy())
    assert a.steps == b.steps == 4 * 16 * 32


@pytest.mark.parametrize('env', ['replay', 'dynamics'])
def test_multi_step_graph_equals_single_steps(device, monkeypatch, env):
    """fused_train_steps with XA_GRAPH_STEPS = 8 (eight train steps per hipGraph replay, and
    graphs of 4 and 2 for what is left; the episode statistics of each step in its own host
    slot, folded in groups) against single-step replays: parameters, Adam state, rollout
    buffers and the episode bookkeeping (total_rewards, games, the last dones) identical
    after 11 steps (groups of 8 and 2 + one single step), on the replay env and on the
    CartPole-dynamics env (both with episode ends inside the window)."""
    from xagents_amd import PPO
    from xagents_amd.envs import CartPoleVecEnv, ReplayVecEnv
    from xagents_amd.utils.common import create_model

    def make(steps_per_graph):
        monkeypatch.setenv('XA_GRAPH_STEPS', str(steps_per_graph))
        if env == 'replay':
            envs = ReplayVecEnv('CartPole-v1', 16, t_rec=100, seed=5, device='cuda')
        else:
            envs = CartPoleVecEnv(16, seed=5, device='cuda')
        model = create_model(envs, 'ppo', 'model', seed=5, device='cuda')
        agent = PPO(envs, model, n_steps=32, seed=5, quiet=True)
        agent.train_step()  # eager step + capture (with this XA_GRAPH_STEPS)
        return agent

    a, b = make(8), make(1)
    assert a.update_mode == 'persistent' and a._graph_S == 8 and len(a._graph) == 6
    assert a._graph_sizes == [8, 4, 2]
    assert b._graph_S == 1 and len(b._graph) == 3
    a.fused_train_steps(11)
    for _ in range(11):
        b.fused_train_step()
    for x in (a, b):
        x._drain_episode_stats()
    torch.cuda.synchronize()
    assert a.steps == b.steps == 12 * 16 * 32
    for name in ('theta', ):
        np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())
    np.testing.assert_array_equal(a.model.optimizer.m.cpu().numpy(),
                                  b.model.optimizer.m.cpu().numpy())
    assert int(a.model.optimizer.iterations.item()) == int(b.model.optimizer.iterations.item())
    for buf in ('b_act', 'b_logp', 'b_ret', 'b_done'):
        np.testing.assert_array_equal(getattr(a, buf).cpu().numpy(), getattr(b, buf).cpu().numpy())
    assert a.games == b.games > 0
    assert list(a.total_rewards) == list(b.total_rewards)
    assert a.dones == b.dones


def test_replan_to_chain_keeps_episode_stats(device, monkeypatch):
    """a re-plan from the persistent update (statistics stored by the update
    launch) to the per-minibatch chain mid-run (what a peer timeout triggers) must fold
    every step once. Agent a runs with the in-launch statistics, agent b with the copy-launch
    path (XA_STATS_IN_UPDATE=0); both re-plan to the chain after 3 steps, so their parameters
    and rollouts stay identical and so must the folded episode statistics."""
    def make(in_update):
        monkeypatch.setenv('XA_STATS_IN_UPDATE', '1' if in_update else '0')
        return make_agent(n_envs=16, n_steps=32, seed=11, t_rec=60)

    a, b = make(True), make(False)
    assert a._stats_fused and not b._stats_fused
    for x in (a, b):
        for _ in range(3):
            x.train_step()
    monkeypatch.setenv('XA_PPO_UPDATE', 'chain')
    for x in (a, b):
        x._setup_update()
        x._graph = None
        assert x.update_mode == 'chain' and not x._stats_fused
        for _ in range(3):
            x.train_step()
        x._drain_episode_stats()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())
    assert a.games == b.games > 0
    assert list(a.total_rewards) == list(b.total_rewards)
    assert a.done_envs == b.done_envs


def test_ppo_train_step_vs_oracle_pipeline(device):
    """One full train step: rollout buffers bit-exact vs the C oracle (same Philox
    stream), then 4 epochs x 4 minibatches against the float64 restatement of the
    reference update (same Feistel minibatch order)."""
    agent = make_agent(n_envs=16, n_steps=64, seed=3, use_graph=False)
    env = agent.envs
    theta0 = agent.model.theta.cpu().numpy().copy()
    host_env = dict(kind=0, state=env.state.cpu().numpy().copy(), done=np.zeros(16, np.float32),
                    cursor=np.zeros(16, np.int32), ep_return=np.zeros(16, np.float32),
                    rep_obs=env.rep_obs.cpu().numpy(), rep_state=env.rep_state.cpu().numpy(),
                    rep_rew=env.rep_rew.cpu().numpy(), rep_done=env.rep_done.cpu().numpy())
    agent.train_step()
    torch.cuda.synchronize()
    ref = oracle.mlp_rollout(theta0, 2, host_env, 64, seed=agent.rng_seed, ctr=0, return_kind=1,
                             gamma=0.99, gamma_lam=float(np.float32(0.99 * 0.95)))
    for k, buf in (('obs', agent.b_obs), ('act', agent.b_act), ('logp', agent.b_logp),
                   ('val', agent.b_val), ('rew', agent.b_rew), ('done', agent.b_done),
                   ('ret', agent.b_ret), ('next_val', agent.next_val)):
        np.testing.assert_array_equal(buf.cpu().numpy(), ref[k], err_msg=k)
    B, MB = agent.batch_size, agent.mini_batch_size
    obs = ref['obs'].reshape(B, 4)
    act, logp_old = ref['act'].reshape(B), ref['logp'].reshape(B)
    val, ret = ref['val'].reshape(B), ref['ret'].reshape(B)
    th = theta0.astype(np.float64)
    m = np.zeros_like(th)
    v = np.zeros_like(th)
    t = 0
    for e in range(agent.ppo_epochs):
        perm = oracle.shuffle_perm(B, e, agent.shuffle.seed, 0)
        for mb in range(agent.n_mb):
            idx = perm[mb * MB:(mb + 1) * MB]
            adv = oracle.normalize_advantages(ret[idx], val[idx])
            _, g = oracle.ac_loss_grad_f64(th, obs[idx], act[idx], ret[idx], val[idx], 2, 'ppo',
                                           logp_old[idx], adv)
            g, _ = oracle.clip_by_global_norm_f64(g, 0.5)
            t += 1
            th, m, v = oracle.keras_adam_f64(th, m, v, g, t, 7e-4, 0.9, 0.999, 1e-7)
    got = agent.model.theta.cpu().numpy().astype(np.float64)
    rel = np.linalg.norm(got - th) / np.linalg.norm(th - theta0)
    assert rel < 2e-3, f'parameter trajectory deviates: {rel:.2e}'
    assert int(agent.model.optimizer.iterations.cpu()[0]) == 16


def test_a2c_train_step_runs_and_matches_oracle_returns(device):
    agent = make_agent('a2c', n_envs=8, n_steps=5, seed=4, use_graph=True)
    for _ in range(3):
        agent.train_step()
    torch.cuda.synchronize()
    ret = oracle.nstep(agent.b_rew.cpu().numpy(), agent.b_done.cpu().numpy(),
                       agent.next_val.cpu().numpy(), 0.99)
    np.testing.assert_array_equal(agent.b_ret.cpu().numpy(), ret)
    assert np.isfinite(agent.model.theta.cpu().numpy()).all()


def test_config2_full_size_properties(device):
    """BASELINE config 2 shape (256 envs x 128 steps, 4x4 minibatches of 8192):
    size-independent properties on the full-size path."""
    agent = make_agent(n_envs=256, n_steps=128, seed=55, t_rec=4096)
    for _ in range(3):
        agent.train_step()
    torch.cuda.synchronize()
    theta = agent.model.theta.cpu().numpy()
    assert np.isfinite(theta).all()
    # fused GAE == standalone GAE kernel == oracle on the same buffers
    from xagents_amd import kernels

    ret2 = kernels.gae(agent.b_rew, agent.b_val, agent.b_done, agent.next_val, 0.99, 0.95)
    np.testing.assert_array_equal(ret2.cpu().numpy(), agent.b_ret.cpu().numpy())
    acts = agent.b_act.cpu().numpy()
    assert set(np.unique(acts)) <= {0, 1}
    assert int(agent.model.optimizer.iterations.cpu()[0]) == 3 * 16
    agent.init_training(None, 10 ** 9, None)
    agent.check_episodes()
    assert agent.games > 0 and len(agent.total_rewards) > 0


def test_fit_loop_and_episode_bookkeeping(device):
    agent = make_agent(n_envs=8, n_steps=16, seed=9)
    agent.fit(max_steps=8 * 16 * 5)
    assert agent.steps == 8 * 16 * 5
    done = agent.b_done.cpu().numpy()
    assert agent.games >= int(done[:, 1:].sum())
