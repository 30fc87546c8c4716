"""GPU tests of DDPG / TD3 (xagents/ddpg/agent.py, xagents/td3/agent.py): one gradient
step (twin critics with target smoothing, delayed actor update through critic1, Polyak
sync) against the float64 restatement, fed with the batch and the noise the device drew;
and the done-triggered training loop."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _agent(device, kind, n=4, gradient_steps=1, tau=0.05):
    from xagents_amd import DDPG, TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('BipedalWalker-v3', n, device=device, seed=4, t_rec=64)
    kw = dict(seed=7, device=device, optimizer_kwargs=dict(learning_rate=1e-3))
    actor = create_model(envs, kind, 'actor_model', **kw)
    critic = create_model(envs, kind, 'critic_model', **kw)
    bufs = create_buffers(kind, 8 * n, 2 * n, n, initial_size=4 * n)
    cls = TD3 if kind == 'td3' else DDPG
    return cls(envs, actor, critic, bufs, gradient_steps=gradient_steps, tau=tau, seed=3,
               quiet=True, gamma=0.99)


def _adam(th, m, v, g, t, lr=1e-3):
    sys.path.insert(0, str(ROOT / 'oracle'))
    import oracle as OR
    return OR.keras_adam_f64(th, m, v, g, t, lr, 0.9, 0.999, 1e-7)[0]


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def _step_close(got, th0, ref, lr=1e-3, tol=2e-2):
    step_got, step_ref = got - th0, ref - th0
    err = np.abs(step_got - step_ref).max() / lr
    assert err < tol, f'update mismatch {err:.3g} (units of lr)'


def _rel(got, want):
    return float(np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30))


@pytest.mark.parametrize('fused', [True, False], ids=['fused', 'executor'])
@pytest.mark.parametrize('kind,n', [('td3', 4), ('ddpg', 4), ('td3', 32), ('td3', 50)])
def test_one_gradient_step_vs_f64(device, kind, n, fused):
    """n = 4: batch 8 (one ragged row tile); n = 32: batch 64 (C5's); n = 50: batch 100 --
    four 32-row tiles (the last ragged), two 64-row weight-gradient k blocks, three column
    tiles per weight-gradient job. The raw gradients g_critic / g_critic2 / g_actor at 1e-4
    relative (magnitude: a first Adam step from zero moments is ~ lr sign(g), so the step
    check alone would pass a gradient off by a factor), then the applied step and the
    Polyak targets."""
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    agent = _agent(device, kind, n=n)
    assert agent.batch_size == 2 * n
    if fused:
        assert agent._fused_args() is not None
    else:
        agent.__dict__['_fused'] = agent.__dict__['_fused_act'] = None
    agent.fill_buffers()
    twin = kind == 'td3'
    nets = [agent.actor, agent.critic] + ([agent.critic2] if twin else [])
    tnets = [agent.target_actor, agent.target_critic] + ([agent.target_critic2] if twin else [])
    th0 = [_np(m.theta) for m in nets]
    tt0 = [_np(m.theta) for m in tnets]
    agent.update_weights(1)
    torch.cuda.synchronize()
    s, a, r, d, s2 = (_np(x) for x in (agent.s, agent.a, agent.r, agent.d, agent.s2))
    B = s.shape[0]
    fw = lambda m, th, x: O.forward(m.layers, th, x, m.input_shape)  # noqa: E731
    out = lambda m, res: res[1][m.outputs[0]]  # noqa: E731
    ta = out(agent.target_actor, fw(agent.target_actor, tt0[0], s2))
    if twin:
        noise = _np(agent.noise)
        assert np.all(np.abs(noise) <= 0.5 + 1e-7) and noise.std() > 0.01
        ta = np.clip(ta + noise, -1, 1)
    s2a2 = np.concatenate([s2, ta], 1)
    tvs = [out(agent.target_critic, fw(agent.target_critic, tt, s2a2)) for tt in tt0[1:]]
    tv = np.minimum(*tvs) if twin else tvs[0]
    y = r[:, None] + (1 - d[:, None]) * 0.99 * tv
    sa = np.concatenate([s, a], 1)
    new = [None] * len(nets)
    g_dev = [None, agent.g_critic] + ([agent.g_critic2] if twin else [])
    for ci in range(1, len(nets)):
        c = nets[ci]
        x64, o = fw(c, th0[ci], sa)
        v = o[c.outputs[0]]
        g = O.backward(c.layers, th0[ci], x64, o, {c.outputs[0]: 2 * (v - y)})
        e = _rel(_np(g_dev[ci]), g)
        assert e < 1e-4, f'critic {ci}: raw gradient {e:.2e}'
        new[ci] = _adam(th0[ci], 0, 0, g, 1)
    # actor step through the UPDATED critic1 (the reference updates critics first)
    act = agent.actor
    xa, oa = fw(act, th0[0], s)
    pa = oa[act.outputs[0]]
    spa = np.concatenate([s, pa], 1)
    xc, oc = fw(agent.critic, new[1], spa)
    _, dx = O.backward(agent.critic.layers, new[1], xc, oc,
                       {agent.critic.outputs[0]: -np.ones((B, 1)) / B}, want_input_grad=True)
    ga = O.backward(act.layers, th0[0], xa, oa, {act.outputs[0]: dx[:, s.shape[1]:]})
    new[0] = _adam(th0[0], 0, 0, ga, 1)
    # the raw actor gradient through the device's own updated critic 1 (an element whose
    # critic gradient is ~0 takes an Adam step that f32 and f64 may round apart)
    c1 = _np(agent.critic.theta)
    xc, oc = fw(agent.critic, c1, spa)
    _, dx = O.backward(agent.critic.layers, c1, xc, oc,
                       {agent.critic.outputs[0]: -np.ones((B, 1)) / B}, want_input_grad=True)
    ga = O.backward(act.layers, th0[0], xa, oa, {act.outputs[0]: dx[:, s.shape[1]:]})
    e = _rel(_np(agent.g_actor), ga)
    assert e < 1e-4, f'actor: raw gradient {e:.2e}'
    for m, th_ref, t0 in zip(nets, new, th0):
        _step_close(_np(m.theta), t0, th_ref)
    for tm, t0, th_ref in zip(tnets, tt0, new):
        np.testing.assert_allclose(_np(tm.theta), 0.95 * t0 + 0.05 * th_ref, rtol=0,
                                   atol=2e-6 * max(1, np.abs(t0).max()))


def test_td3_train_loop_runs_gradient_steps_on_done(device):
    agent = _agent(device, 'td3', n=4, gradient_steps=1)
    agent.fit(max_steps=4 * 80)
    torch.cuda.synchronize()
    # every done env triggered one gradient step (critic Adam step each time)
    it = int(agent.critic.optimizer.iterations.item())
    assert it == agent.games and it > 0
    # gradient_steps=1: every update_weights call runs gradient step 0, which also
    # updates the actor (0 % policy_delay == 0)
    assert int(agent.actor.optimizer.iterations.item()) == it
    assert int(agent.critic2.optimizer.iterations.item()) == it


@pytest.mark.parametrize('kind', ['td3', 'ddpg'])
def test_captured_gradient_steps_match_eager(device, kind):
    """update_weights replays captured hipGraphs after one eager pass per phase: the
    parameters after 5 gradient steps are bit-identical to all-eager launches (same host
    RNG draws for the sample indices, same device noise counter)."""
    import random
    out = []
    for use_graph in (False, True):
        np.random.seed(0)
        random.seed(0)
        agent = _agent(device, kind)
        agent.use_graph = use_graph
        agent.fill_buffers()
        agent.update_weights(5)
        torch.cuda.synchronize()
        nets = [agent.actor, agent.critic, agent.target_actor, agent.target_critic]
        if kind == 'td3':
            nets += [agent.critic2, agent.target_critic2]
        out.append([_np(m.theta) for m in nets])
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('kind', ['td3', 'ddpg'])
def test_captured_env_phase_matches_eager(device, kind):
    """train_step's env phase (actor forward [+ noise] + ring append) replayed as a hipGraph
    stores the same transitions, episode statistics and weights as eager launches."""
    import random
    out = []
    for use_graph in (False, True):
        np.random.seed(0)
        random.seed(0)
        agent = _agent(device, kind, n=4, gradient_steps=1)
        agent.use_graph = use_graph
        agent.fill_buffers()
        for _ in range(70):
            agent.train_step()
        agent._drain_episode_stats()
        torch.cuda.synchronize()
        r = agent.replay
        out.append(([_np(x) for x in (r.states, r.actions, r.rewards, r.dones, r.new_states,
                                      agent.actor.theta, agent.critic.theta)],
                    (agent.games, list(agent.total_rewards), agent.steps)))
    for a, b in zip(out[0][0], out[1][0]):
        np.testing.assert_array_equal(a, b)
    assert out[0][1] == out[1][1]
    assert out[1][1][0] > 0  # some episodes finished (gradient steps ran)


@pytest.mark.parametrize('kind', ['td3', 'ddpg'])
def test_fused_step_actions_vs_f64(device, kind):
    """get_step_actions in one launch (xa_td3_act): clip(tanh(actor(s)) + noise, -1, 1)
    against the float64 actor forward with the noise the launch drew; the draw is bit-equal
    to xa_noisy_actions' at the same counter, and the counter advances by one per call.
    40 envs: a full and a ragged 32-row tile."""
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    from xagents_amd._lib import call, stream
    agent = _agent(device, kind, n=40)
    fa = agent._fused_act_args()
    assert fa is not None
    torch.manual_seed(0)
    agent.envs.state.copy_(torch.randn_like(agent.envs.state))
    c0 = int(agent.rng_counter.item())
    noise = torch.zeros_like(agent.step_actions)
    fa.noise_out = noise.data_ptr()
    try:
        out = agent.get_step_actions().clone()
    finally:
        fa.noise_out = None
    torch.cuda.synchronize()
    nz = _np(noise)
    if kind == 'td3':
        # TD3 acts with the actor's output, no exploration noise (td3/agent.py:57-64)
        assert int(agent.rng_counter.item()) == c0
        assert not nz.any()
    else:
        assert int(agent.rng_counter.item()) == c0 + 1
        assert nz.std() > 0.01
    act = agent.actor
    _, o = O.forward(act.layers, _np(act.theta), _np(agent.envs.state), act.input_shape)
    ref = np.clip(o[act.outputs[0]] + nz, -1, 1)
    np.testing.assert_allclose(_np(out), ref, rtol=0, atol=1e-5)
    if kind == 'td3':
        return
    # xa_noisy_actions' draw at the same counter (zero input, unbounded clip)
    ctr = agent.rng_counter.clone().fill_(c0)
    zero = torch.zeros_like(agent.step_actions)
    n2 = torch.zeros_like(zero)
    o2 = torch.zeros_like(zero)
    rows, cols = zero.shape
    call('xa_noisy_actions', zero.data_ptr(), cols, rows, cols,
         float(np.float32(agent.step_noise_coef)), float('inf'), float('-inf'), float('inf'),
         ctr.data_ptr(), agent.rng_seed, o2.data_ptr(), cols, n2.data_ptr(), stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(n2), nz)


def test_fused_grid_size_is_bit_neutral_and_status_clean(device):
    """The fused step's result does not depend on its grid: 40 chained gradient steps at
    batch 8 on 256 workgroups (most blocks hold no job in most phases, so they would have
    arrived at no barrier before every block had to arrive at a launch's first one, ADVICE
    r04) and on 32 give bit-identical weights, moments and step counters, and the status
    word stays 0 (no barrier timed out)."""
    import random
    out = []
    for G in (256, 32):
        np.random.seed(0)
        random.seed(0)
        agent = _agent(device, 'td3')
        a = agent._fused_args()
        assert a is not None
        a.n_blocks = G
        agent.fill_buffers()
        agent.update_weights(40)
        torch.cuda.synchronize()
        assert int(agent._fused_status.item()) == 0
        assert int(agent.critic.optimizer.iterations.item()) == 40
        assert int(agent.actor.optimizer.iterations.item()) == 20
        nets = [agent.actor, agent.critic, agent.critic2, agent.target_actor,
                agent.target_critic, agent.target_critic2]
        out.append([_np(x) for m in nets for x in (m.theta,) + (
            (m.optimizer.m, m.optimizer.v) if getattr(m, 'optimizer', None) is not None else ())])
    for x, y in zip(*out):
        np.testing.assert_array_equal(x, y)
