"""GPU tests of the on-policy path for .cfg actor-critics run on the layer executor (the
CNN actor-critic, config C4): the batched categorical against an f32 restatement built
from the oracle's exp / log (bit-exact), the rollout bookkeeping, and one PPO update
against the float64 restatement (loss gradient through the CNN, global-norm clip, Keras
Adam)."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu
sys.path.insert(0, str(ROOT / 'oracle'))


def _categorical_ref(logits, u):
    import oracle as OR
    f = np.float32
    n, A = logits.shape
    act, lp_out, ent_out = [], [], []
    for i in range(n):
        l = logits[i].astype(f)
        m = l[0]
        for a in range(1, A):
            m = max(m, l[a])
        e = OR.math_f32('exp', (l - m).astype(f))
        s = f(0)
        for a in range(A):
            s = f(s + e[a])
        ls = OR.math_f32('log', np.array([s], f))[0]
        target = f(u[i] * s)
        c, k = f(0), A - 1
        for a in range(A):
            c = f(c + e[a])
            if target < c:
                k = a
                break
        inv = f(f(1) / s)
        en, lp = f(0), f(0)
        for a in range(A):
            la = f(f(l[a] - m) - ls)
            p = f(e[a] * inv)
            en = f(en - f(p * la))
            if a == k:
                lp = la
        act.append(k)
        lp_out.append(lp)
        ent_out.append(en)
    return np.array(act), np.array(lp_out, f), np.array(ent_out, f)


def test_categorical_bit_exact(device):
    from xagents_amd._lib import call, stream
    rng = np.random.default_rng(2)
    n, A = 300, 6
    logits = (rng.normal(size=(n, A)) * 3).astype(np.float32)
    u = rng.random(n).astype(np.float32)
    tl, tu = torch.from_numpy(logits).to(device), torch.from_numpy(u).to(device)
    act = torch.empty(n, dtype=torch.int32, device=device)
    lp, en = torch.empty(n, device=device), torch.empty(n, device=device)
    call('xa_categorical', tl.data_ptr(), A, n, A, tu.data_ptr(), None, 0, 0, None,
         act.data_ptr(), lp.data_ptr(), en.data_ptr(), 1, stream())
    ra, rl, re = _categorical_ref(logits, u)
    np.testing.assert_array_equal(act.cpu().numpy(), ra)
    np.testing.assert_array_equal(lp.cpu().numpy(), rl)
    np.testing.assert_array_equal(en.cpu().numpy(), re)


def _ppo(device, n=4, t=8, kind='ppo'):
    from xagents_amd import A2C, PPO
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_model
    envs = create_envs('BreakoutNoFrameskip-v4', n, device=device, seed=6)
    model = create_model(envs, kind, 'model', seed=4, device=device,
                         optimizer_kwargs=dict(learning_rate=1e-3))
    if kind == 'ppo':
        return PPO(envs, model, n_steps=t, seed=8, quiet=True, ppo_epochs=1, mini_batches=1)
    return A2C(envs, model, n_steps=t, seed=8, quiet=True)


def _heads_grad_f64(logits, v, act, oldlp, oldv, ret, kind, clip=0.1, ent_coef=0.01,
                    v_coef=0.5, eps=1e-8):
    import oracle as OR
    n, A = logits.shape
    lsm = OR.log_softmax(logits)
    p = np.exp(lsm)
    logp = lsm[np.arange(n), act]
    H = -(p * lsm).sum(-1)
    onehot = np.eye(A)[act]
    if kind == 'ppo':
        adv = ret - oldv
        adv = (adv - adv.mean()) / (adv.std() + eps)
        ratio = np.exp(logp - oldlp)
        pg1, pg2 = -adv * ratio, -adv * np.clip(ratio, 1 - clip, 1 + clip)
        r_in = (ratio >= 1 - clip) & (ratio <= 1 + clip)
        dlogp = np.where((pg1 >= pg2) | r_in, -adv * ratio, 0.0) / n
        dvo = v - oldv
        vclip = oldv + np.clip(dvo, -clip, clip)
        vl1, vl2 = (v - ret) ** 2, (vclip - ret) ** 2
        v_in = (dvo >= -clip) & (dvo <= clip)
        dv = v_coef * 0.5 * np.where(vl1 >= vl2, 2 * (v - ret),
                                     np.where(v_in, 2 * (vclip - ret), 0.0)) / n
    else:
        dlogp = -(ret - oldv) / n
        dv = v_coef * 2 * (v - ret) / n
    dz = dlogp[:, None] * (onehot - p) + (ent_coef / n) * p * (lsm + H[:, None])
    return dz, dv


@pytest.mark.parametrize('kind', ['ppo', 'a2c'])
def test_cnn_actor_critic_train_step_vs_f64(device, kind):
    import nets_f64 as O
    import oracle as OR
    agent = _ppo(device, kind=kind)
    model = agent.model
    th0 = model.theta.cpu().numpy().astype(np.float64)
    opt = model.optimizer
    agent._executor_rollout()
    torch.cuda.synchronize()
    N, T = agent.n_envs, agent.n_steps
    obs = agent.obs_buf[:T].cpu().numpy()                   # [T, N, ...]
    # env-major flat order i = env * T + t (concat_step_batches)
    x = obs.transpose(1, 0, 2, 3, 4).reshape(N * T, *obs.shape[2:])
    act = agent.b_act.cpu().numpy().reshape(-1)
    oldlp = agent.b_logp.cpu().numpy().reshape(-1).astype(np.float64)
    oldv = agent.b_val.cpu().numpy().reshape(-1).astype(np.float64)
    ret = agent.b_ret.cpu().numpy().reshape(-1).astype(np.float64)
    # rollout values / log-probs agree with the f64 forward on the stored frames
    x64, outs = O.forward(model.layers, th0, x, model.input_shape)
    logits, v = outs[model.outputs[0]], outs[model.outputs[1]][:, 0]
    np.testing.assert_allclose(oldv, v, rtol=1e-4, atol=1e-5)
    lp_ref = OR.log_softmax(logits)[np.arange(N * T), act]
    np.testing.assert_allclose(oldlp, lp_ref, rtol=1e-4, atol=1e-5)
    agent._executor_update()
    torch.cuda.synchronize()
    dz, dv = _heads_grad_f64(logits, v, act, oldlp, oldv, ret, kind)
    g = O.backward(model.layers, th0, x64, outs,
                   {model.outputs[0]: dz, model.outputs[1]: dv[:, None]})
    g = OR.clip_by_global_norm_f64(g, 0.5)[0]
    th1 = OR.keras_adam_f64(th0, 0, 0, g, 1, 1e-3, 0.9, 0.999, 1e-7)[0]
    got = model.theta.cpu().numpy()
    big = np.abs(g) > 1e-5 * np.abs(g).max()
    err = np.abs((got - th0)[big] - (th1 - th0)[big]).max() / 1e-3
    assert err < 3e-2, f'update mismatch {err:.3g} (units of lr)'
    assert int(opt.iterations.item()) == 1


def test_cnn_ppo_train_steps_and_stats(device):
    agent = _ppo(device, n=4, t=16)
    agent.ppo_epochs = 2
    for _ in range(3):
        agent.fused_train_step()
    agent._drain_episode_stats()
    torch.cuda.synchronize()
    assert agent.steps == 3 * 4 * 16
    assert int(agent.model.optimizer.iterations.item()) == 3 * 2
    assert np.isfinite(agent.model.theta.cpu().numpy()).all()
