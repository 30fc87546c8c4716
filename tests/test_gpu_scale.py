"""Scale-sensitive parity of the off-policy and CNN heads (SURVEY.md 8a A12 CNN, A21, A22,
A25, A26): the RAW gradients before Adam and the per-sample loss outputs of xa_dqn_td_grad
(plain / double), xa_critic_td_grad (twin / single), xa_mse_grad and xa_ac_head_grad
against the float64 restatement (oracle/nets_f64.py), then 3 chained steps whose Adam
moments are non-zero, so a gradient off by any factor (e.g. a dropped 1 / A) fails.
Tolerances: 1e-5 relative on the heads, 1e-4 through the layer executor."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))
pytestmark = pytest.mark.gpu

LR, B1, B2, EPS = 1e-3, 0.9, 0.999, 1e-7


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def _rel(got, want):
    want = np.asarray(want, np.float64)
    return float(np.linalg.norm(np.asarray(got, np.float64) - want) /
                 max(np.linalg.norm(want), 1e-30))


def _adam(th, m, v, g, t):
    import oracle as OR
    return OR.keras_adam_f64(th, m, v, g, t, LR, B1, B2, EPS)


def _opt_state(model):
    opt = model.optimizer
    return _np(model.theta), _np(opt.m), _np(opt.v), int(opt.iterations.item())


def _check_adam(model, before, g64, step_tol=1e-3):
    """The device step from `before` = (theta, m, v, t) against f64 Keras Adam with the f64
    gradient: moments (scale-sensitive once m, v are non-zero) and the parameter step."""
    th0, m0, v0, t0 = before
    th1, m1, v1 = _adam(th0, m0, v0, g64, t0 + 1)
    th, m, v, t = _opt_state(model)
    assert t == t0 + 1
    assert _rel(m, m1) < 1e-4, f'Adam m: {_rel(m, m1):.2e}'
    assert _rel(v, v1) < 2e-4, f'Adam v: {_rel(v, v1):.2e}'
    if t0 > 0:  # past the first step the update is no longer ~ lr * sign(g)
        assert _rel(th - th0, th1 - th0) < step_tol, f'step: {_rel(th - th0, th1 - th0):.2e}'


# ---------------------------------------------------------------------------------------
# DQN / double DQN (dqn/agent.py:118-171)
# ---------------------------------------------------------------------------------------
def _dqn(device, double, huber=None):
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=3)
    model = create_model(envs, 'dqn', 'model', seed=9, device=device,
                         optimizer_kwargs=dict(learning_rate=LR))
    bufs = create_buffers('dqn', 40, 4, 2, initial_size=20)
    np.random.seed(1)
    random.seed(1)
    agent = DQN(envs, model, bufs, double=double, seed=2, quiet=True, epsilon_start=0.0,
                epsilon_end=0.0, gamma=0.99, huber_delta=huber)
    # the dense layer's Adam runs inside its weight-gradient GEMM: ask it for the raw
    # gradient too, so the whole gradient is checked
    agent.write_raw_grad = True
    agent.fill_buffers()
    agent.target_model.theta.mul_(0.97)  # the target differs, so double DQN matters
    return agent


def _dqn_f64(agent, th, tt, huber=None):
    import nets_f64 as O
    model = agent.model
    B = agent.batch_size
    s, s2 = agent.xb[:B].cpu().numpy(), agent.xb[B:].cpu().numpy()
    a = agent.b_act.cpu().numpy()
    r = _np(agent.b_rew)
    d = agent.b_done.cpu().numpy()
    L, shape, out = model.layers, model.input_shape, model.outputs[0]
    x64, outs = O.forward(L, th, s, shape)
    q = outs[out]
    qt = O.forward(L, tt, s2, shape)[1][out]
    if agent.double:
        an = O.forward(L, th, s2, shape)[1][out].argmax(1)
        v = qt[np.arange(B), an]
    else:
        v = qt.max(1)
    v = np.where(d != 0, 0.0, v)
    y = v * np.float64(np.float32(0.99)) + r
    A = q.shape[1]
    diff = y - q[np.arange(B), a]
    dq = np.zeros_like(q)
    if huber:
        dq[np.arange(B), a] = -np.clip(diff, -huber, huber) / A
        ad = np.abs(diff)
        loss = np.where(ad <= huber, 0.5 * diff ** 2, huber * (ad - 0.5 * huber)) / A
    else:
        dq[np.arange(B), a] = -2.0 * diff / A
        loss = diff ** 2 / A
    g = O.backward(L, th, x64, outs, {out: dq})
    return dq, loss, g


@pytest.mark.parametrize('double', [False, True])
def test_dqn_raw_gradient_losses_and_chained_steps(device, double):
    agent = _dqn(device, double)
    model, tgt = agent.model, agent.target_model
    for k in range(3):
        before = _opt_state(model)
        tt = _np(tgt.theta)
        agent.at_step_start()
        agent.train_step()
        torch.cuda.synchronize()
        dq64, loss64, g64 = _dqn_f64(agent, before[0], tt)
        assert _rel(_np(agent.dq), dq64) < 1e-5, f'step {k}: dq {_rel(_np(agent.dq), dq64):.2e}'
        assert _rel(_np(agent.td_loss), loss64) < 1e-5, f'step {k}: per-sample loss'
        assert _rel(_np(agent.grad), g64) < 1e-4, f'step {k}: raw gradient {_rel(_np(agent.grad), g64):.2e}'
        _check_adam(model, before, g64)
    assert int(model.optimizer.iterations.item()) == 3


def test_dqn_huber_opt_in_vs_f64(device):
    """Opt-in Huber-TD (north_star; NOT the reference's loss, which is MSE): raw head
    gradient, per-sample loss and the CNN gradient vs float64."""
    agent = _dqn(device, False, huber=1.0)
    # scale the rewards up so some TD errors exceed delta
    agent.replay.rewards.mul_(3.0)
    before = _opt_state(agent.model)
    tt = _np(agent.target_model.theta)
    agent.at_step_start()
    agent.train_step()
    torch.cuda.synchronize()
    dq64, loss64, g64 = _dqn_f64(agent, before[0], tt, huber=1.0)
    assert _rel(_np(agent.dq), dq64) < 1e-5
    assert _rel(_np(agent.td_loss), loss64) < 1e-5
    assert _rel(_np(agent.grad), g64) < 1e-4
    B = agent.batch_size
    assert np.abs(dq64).max() * 6 <= 1.0 + 1e-6  # |dq| <= delta / A


# ---------------------------------------------------------------------------------------
# DDPG / TD3 (ddpg/agent.py:87-127, td3/agent.py:66-110)
# ---------------------------------------------------------------------------------------
def _ddpg(device, kind, huber=None, n=4, fused=True):
    """n envs with one RB2 each, batch 2 n. fused=False forces the layer-executor step (the
    path a non-MLP cfg takes) in place of xa_td3_update / xa_td3_act."""
    from xagents_amd import DDPG, TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('BipedalWalker-v3', n, device=device, seed=4, t_rec=64)
    kw = dict(seed=7, device=device, optimizer_kwargs=dict(learning_rate=LR))
    actor = create_model(envs, kind, 'actor_model', **kw)
    critic = create_model(envs, kind, 'critic_model', **kw)
    bufs = create_buffers(kind, 8 * n, 2 * n, n, initial_size=4 * n)
    cls = TD3 if kind == 'td3' else DDPG
    np.random.seed(2)
    random.seed(2)
    agent = cls(envs, actor, critic, bufs, gradient_steps=1, tau=0.05, seed=3, quiet=True,
                gamma=0.99, huber_delta=huber)
    if fused:
        assert agent._fused_args() is not None and agent._fused_act_args() is not None
    else:
        agent.__dict__['_fused'] = agent.__dict__['_fused_act'] = None
    agent.fill_buffers()
    return agent


def _critic_head_f64(v, y, huber):
    e = v - y
    if huber:
        ae = np.abs(e)
        return np.clip(e, -huber, huber), np.where(ae <= huber, 0.5 * e * e,
                                                   huber * (ae - 0.5 * huber))
    return 2 * e, e * e


@pytest.mark.parametrize('fused', [True, False], ids=['fused', 'executor'])
@pytest.mark.parametrize('kind,huber,n', [('td3', None, 4), ('ddpg', None, 4), ('td3', 0.5, 4),
                                          ('td3', None, 32), ('td3', None, 50),
                                          ('ddpg', None, 50)])
def test_critic_actor_raw_gradients_and_chained_steps(device, kind, huber, n, fused):
    """Both gradient-step paths (the fused xa_td3_update and the layer executor, which a
    non-MLP cfg takes) against float64 over 3 chained steps: dv and the per-sample loss at
    1e-5, g_critic / g_critic2 / g_actor at 1e-4 (magnitude, not sign: the chained Adam
    moments are non-zero). Batch 8 is one ragged row tile of the fused kernel; batch 64 (C5's)
    two full ones; batch 100 four with a ragged last, two 64-row weight-gradient k blocks and
    three column tiles per weight-gradient job, the cross-tile head tickets included."""
    import nets_f64 as O
    agent = _ddpg(device, kind, huber, n=n, fused=fused)
    assert agent.batch_size == 2 * n
    twin = kind == 'td3'
    critics = [agent.critic] + ([agent.critic2] if twin else [])
    tcrit = [agent.target_critic] + ([agent.target_critic2] if twin else [])
    fw = lambda m, th, x: O.forward(m.layers, th, x, m.input_shape)  # noqa: E731
    out = lambda m, res: res[1][m.outputs[0]]  # noqa: E731
    if huber:  # larger TD errors, so the Huber clip is exercised
        agent.replay.rewards.mul_(4.0)
    for k in range(3):
        b_crit = [_opt_state(c) for c in critics]
        b_act = _opt_state(agent.actor)
        tt = [_np(m.theta) for m in [agent.target_actor] + tcrit]
        agent.update_weights(1)
        torch.cuda.synchronize()
        s, a, r, d, s2 = (_np(x) for x in (agent.s, agent.a, agent.r, agent.d, agent.s2))
        B = s.shape[0]
        ta = out(agent.target_actor, fw(agent.target_actor, tt[0], s2))
        if twin:
            ta = np.clip(ta + _np(agent.noise), -1, 1)
        s2a2 = np.concatenate([s2, ta], 1)
        tvs = [out(c, fw(c, th, s2a2)) for c, th in zip(tcrit, tt[1:])]
        tv = np.minimum(*tvs) if twin else tvs[0]
        y = r[:, None] + (1 - d[:, None]) * np.float64(np.float32(0.99)) * tv
        sa = np.concatenate([s, a], 1)
        loss64 = np.zeros(B)
        for ci, (c, dv_dev, g_dev) in enumerate(zip(
                critics, [agent.dv1, agent.dv2], [agent.g_critic, getattr(agent, 'g_critic2', None)])):
            x64, o = fw(c, b_crit[ci][0], sa)
            v = o[c.outputs[0]]
            dv, lv = _critic_head_f64(v, y, huber)
            loss64 += lv[:, 0]
            assert _rel(_np(dv_dev), dv) < 1e-5, f'step {k} critic {ci}: dv'
            g = O.backward(c.layers, b_crit[ci][0], x64, o, {c.outputs[0]: dv})
            assert _rel(_np(g_dev), g) < 1e-4, f'step {k} critic {ci}: raw gradient {_rel(_np(g_dev), g):.2e}'
            _check_adam(c, b_crit[ci], g)
        assert _rel(_np(agent.critic_loss), loss64) < 1e-5, f'step {k}: per-sample critic loss'
        # actor: -mean Q(s, pi(s)) through the UPDATED critic1 (critics step first)
        act = agent.actor
        xa, oa = fw(act, b_act[0], s)
        spa = np.concatenate([s, oa[act.outputs[0]]], 1)
        c1 = _np(agent.critic.theta)
        xc, oc = fw(agent.critic, c1, spa)
        _, dx = O.backward(agent.critic.layers, c1, xc, oc,
                           {agent.critic.outputs[0]: -np.ones((B, 1)) / B}, want_input_grad=True)
        ga = O.backward(act.layers, b_act[0], xa, oa, {act.outputs[0]: dx[:, s.shape[1]:]})
        assert _rel(_np(agent.g_actor), ga) < 1e-4, f'step {k}: actor raw gradient'
        _check_adam(act, b_act, ga)


def test_mse_grad_kernel_vs_f64(device):
    """xa_mse_grad (tf.keras.losses.MSE + minimize, TRPO's critic): d = 2 (p - y) / n_out,
    loss = mean over the last axis."""
    from xagents_amd._lib import call, stream
    rng = np.random.default_rng(3)
    for B, A in ((64, 1), (37, 6)):
        p = rng.standard_normal((B, A)).astype(np.float32)
        y = rng.standard_normal((B, A)).astype(np.float32)
        tp, ty = torch.from_numpy(p).to(device), torch.from_numpy(y).to(device)
        d, l = torch.empty_like(tp), torch.empty(B, device=device)
        call('xa_mse_grad', tp.data_ptr(), ty.data_ptr(), B, A, d.data_ptr(), l.data_ptr(),
             stream())
        e = p.astype(np.float64) - y
        assert _rel(_np(d), 2 * e / A) < 1e-6
        assert _rel(_np(l), (e ** 2).mean(1)) < 1e-6


# ---------------------------------------------------------------------------------------
# CNN actor-critic (xa_ac_head_grad through the layer executor), PPO and A2C
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize('kind', ['ppo', 'a2c'])
def test_cnn_head_raw_gradient_losses_and_chained_updates(device, kind):
    import nets_f64 as O
    import oracle as OR
    from test_gpu_cnn_onpolicy import _heads_grad_f64, _ppo
    agent = _ppo(device, n=4, t=8, kind=kind)
    model = agent.model
    N, T = agent.n_envs, agent.n_steps
    for k in range(3):
        before = _opt_state(model)
        agent._executor_rollout()
        torch.cuda.synchronize()
        obs = agent.obs_buf[:T].cpu().numpy()
        x = obs.transpose(1, 0, 2, 3, 4).reshape(N * T, *obs.shape[2:])
        act = agent.b_act.cpu().numpy().reshape(-1)
        oldlp, oldv, ret = (_np(t).reshape(-1) for t in (agent.b_logp, agent.b_val, agent.b_ret))
        agent._executor_update()
        torch.cuda.synchronize()
        # ppo_epochs = mini_batches = 1: one minibatch, numpy's permutation of the batch
        n = agent.mb
        slots = agent._slots_flat[:n].cpu().numpy()
        xs, a_, lp_, v_, r_ = x[slots], act[slots], oldlp[slots], oldv[slots], ret[slots]
        x64, outs = O.forward(model.layers, before[0], xs, model.input_shape)
        logits, v = outs[model.outputs[0]], outs[model.outputs[1]][:, 0]
        dz, dv = _heads_grad_f64(logits, v, a_, lp_, v_, r_, kind)
        assert _rel(_np(agent.dlogits[:n]), dz) < 1e-4, f'step {k}: dlogits'
        assert _rel(_np(agent.dvalue[:n, 0]), dv) < 1e-4, f'step {k}: dvalue'
        lsm = OR.log_softmax(logits)
        H = -(np.exp(lsm) * lsm).sum(-1)
        hl = _np(agent.head_loss)
        np.testing.assert_allclose(hl[2], H.mean(), rtol=1e-4)
        g = O.backward(model.layers, before[0], x64, outs,
                       {model.outputs[0]: dz, model.outputs[1]: dv[:, None]})
        assert _rel(_np(agent.grad), g) < 1e-4, f'step {k}: raw gradient {_rel(_np(agent.grad), g):.2e}'
        gc = OR.clip_by_global_norm_f64(g, 0.5)[0]
        _check_adam(model, before, gc, step_tol=2e-3)
