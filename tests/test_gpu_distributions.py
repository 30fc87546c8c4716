"""A2C.get_distribution (xagents/a2c/agent.py:54-63) beyond Categorical(logits):
MultivariateNormalDiag(loc = actor output) for Box action spaces and Categorical(probs)
after a softmax output layer, through the layer-executor on-policy path, against float64
restatements of the TFP distributions (log-prob, entropy) and of the PPO / A2C loss
gradients through the model (oracle/nets_f64.py)."""
import shutil
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))
pytestmark = pytest.mark.gpu
LOG2PI = np.log(2 * np.pi)


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def _rel(got, want):
    want = np.asarray(want, np.float64)
    return float(np.linalg.norm(np.asarray(got, np.float64) - want) /
                 max(np.linalg.norm(want), 1e-30))


def test_diag_gaussian_kernel(device):
    """Given noise: a = mu + noise exactly, log-prob = -0.5|a - mu|^2 - 0.5 d log(2 pi),
    entropy 0.5 d (1 + log 2 pi); Philox draws are N(0, 1)."""
    from xagents_amd._lib import call, stream
    rng = np.random.default_rng(0)
    n, d = 300, 4
    mu = rng.normal(size=(n, d)).astype(np.float32)
    noise = rng.normal(size=(n, d)).astype(np.float32)
    tm, tn = torch.from_numpy(mu).to(device), torch.from_numpy(noise).to(device)
    act = torch.empty(n, d, device=device)
    lp, en = torch.empty(n, device=device), torch.empty(n, device=device)
    call('xa_diag_gaussian', tm.data_ptr(), d, n, d, tn.data_ptr(), None, 0, 0, None, d,
         act.data_ptr(), lp.data_ptr(), en.data_ptr(), 1, stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(act.cpu().numpy(), mu + noise)
    a64 = (mu + noise).astype(np.float64)
    ref = -0.5 * ((a64 - mu) ** 2).sum(1) - 0.5 * d * LOG2PI
    np.testing.assert_allclose(lp.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(en.cpu().numpy(), 0.5 * d * (1 + LOG2PI), rtol=1e-6)
    # log-prob of given actions, and Philox sampling statistics
    call('xa_diag_gaussian', tm.data_ptr(), d, n, d, None, None, 0, 0, act.data_ptr(), d, None,
         lp.data_ptr(), None, 1, stream())
    np.testing.assert_allclose(lp.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    N = 20000
    zero = torch.zeros(N, d, device=device)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    out = torch.empty(N, d, device=device)
    call('xa_diag_gaussian', zero.data_ptr(), d, N, d, None, ctr.data_ptr(), 1234, 3, None, d,
         out.data_ptr(), None, None, 1, stream())
    x = out.cpu().numpy()
    assert abs(x.mean()) < 0.02 and abs(x.std() - 1.0) < 0.02
    assert abs(np.corrcoef(x[:, 0], x[:, 1])[0, 1]) < 0.03
    # consecutive train-step counters draw independent noise: no dimension of counter c + 1
    # repeats (or correlates with) any dimension of counter c (a 4-D action, as the
    # BipedalWalker stand-in's)
    ctr.fill_(6)
    out2 = torch.empty(N, d, device=device)
    call('xa_diag_gaussian', zero.data_ptr(), d, N, d, None, ctr.data_ptr(), 1234, 3, None, d,
         out2.data_ptr(), None, None, 1, stream())
    ctr.fill_(7)
    out3 = torch.empty(N, d, device=device)
    call('xa_diag_gaussian', zero.data_ptr(), d, N, d, None, ctr.data_ptr(), 1234, 3, None, d,
         out3.data_ptr(), None, None, 1, stream())
    y, z = out2.cpu().numpy(), out3.cpu().numpy()
    for j in range(d):
        for jj in range(d):
            assert abs(np.corrcoef(y[:, j], z[:, jj])[0, 1]) < 0.03, (j, jj)
            if j != jj:
                assert abs(np.corrcoef(y[:, j], y[:, jj])[0, 1]) < 0.03, (j, jj)


def _heads_f64(out_a, v, act, oldlp, oldv, ret, kind, dist, clip=0.1, ent_coef=0.01,
               v_coef=0.5, eps=1e-8):
    """d loss / d actor output and d loss / d value (ppo/agent.py:96-137, a2c 190-218)
    for MultivariateNormalDiag(loc) or Categorical(probs = softmax(z))."""
    import oracle as OR
    n = out_a.shape[0]
    if dist == 'gauss':
        d = out_a.shape[1]
        diff = act - out_a
        logp = -0.5 * (diff ** 2).sum(1) - 0.5 * d * LOG2PI
        dlogp_dz = diff
        dH = np.zeros_like(out_a)
    else:
        lsm = OR.log_softmax(out_a)
        p = np.exp(lsm)
        logp = np.log(p[np.arange(n), act.astype(int)])  # Categorical(probs).log_prob
        H = -(p * lsm).sum(-1)
        dlogp_dz = np.eye(out_a.shape[1])[act.astype(int)] - p
        dH = -p * (lsm + H[:, None])  # dH/dz
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
    dz = dlogp[:, None] * dlogp_dz - (ent_coef / n) * dH
    return dz, dv, logp


def _softmax_cfg(tmp_path):
    src = ROOT / 'xagents_amd' / 'ppo' / 'models' / 'ann-actor-critic.cfg'
    text = src.read_text().replace('[dense-2]\n', '[dense-2]\nactivation=softmax\n')
    dst = Path(tmp_path) / 'ann-actor-critic-softmax.cfg'
    dst.write_text(text)
    return str(dst)


@pytest.mark.parametrize('kind,dist', [('ppo', 'gauss'), ('a2c', 'gauss'), ('ppo', 'softmax'),
                                       ('a2c', 'softmax')])
def test_policy_distribution_train_step_vs_f64(device, tmp_path, kind, dist):
    import nets_f64 as O
    from xagents_amd import A2C, PPO
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_model
    n, T = 4, 8
    if dist == 'gauss':
        envs = create_envs('BipedalWalker-v3', n, device=device, seed=5, t_rec=64)
        model = create_model(envs, kind, 'model', seed=3, device=device,
                             optimizer_kwargs=dict(learning_rate=1e-3))
    else:
        envs = create_envs('CartPole-v1', n, mode='transitions', device=device, seed=5,
                           t_rec=64)
        model = create_model(envs, kind, 'model', seed=3, device=device,
                             model_cfg=_softmax_cfg(tmp_path),
                             optimizer_kwargs=dict(learning_rate=1e-3))
    kw = dict(ppo_epochs=1, mini_batches=1) if kind == 'ppo' else {}
    agent = (PPO if kind == 'ppo' else A2C)(envs, model, n_steps=T, seed=8, quiet=True, **kw)
    assert agent.executor_path
    assert agent.distribution_type == ('MultivariateNormalDiag' if dist == 'gauss'
                                       else 'Categorical')
    assert agent.output_is_softmax == (dist == 'softmax')
    th0 = _np(model.theta)
    agent._executor_rollout()
    torch.cuda.synchronize()
    N = n
    obs = agent.obs_buf[:T].cpu().numpy()
    x = obs.transpose(1, 0, *range(2, obs.ndim)).reshape(N * T, *obs.shape[2:])
    act = _np(agent.b_act).reshape(N * T, -1)
    act = act if dist == 'gauss' else act[:, 0]
    oldlp, oldv, ret = (_np(t).reshape(-1) for t in (agent.b_logp, agent.b_val, agent.b_ret))
    x64, outs = O.forward(model.layers, th0, x, model.input_shape)
    za, v = outs[model.outputs[0]], outs[model.outputs[1]][:, 0]
    np.testing.assert_allclose(oldv, v, rtol=1e-4, atol=1e-5)
    _, _, lp_ref = _heads_f64(za, v, act, oldlp, oldv, ret, kind, dist)
    np.testing.assert_allclose(oldlp, lp_ref, rtol=1e-4, atol=1e-4)
    ent = _np(agent.b_ent).reshape(-1)
    if dist == 'gauss':
        np.testing.assert_allclose(ent, 0.5 * 4 * (1 + LOG2PI), rtol=1e-6)
    agent._executor_update()
    torch.cuda.synchronize()
    slots = agent._slots_flat[:agent.mb].cpu().numpy()
    x64, outs = O.forward(model.layers, th0, x[slots], model.input_shape)
    za, v = outs[model.outputs[0]], outs[model.outputs[1]][:, 0]
    dz, dv, _ = _heads_f64(za, v, act[slots], oldlp[slots], oldv[slots], ret[slots], kind, dist)
    assert _rel(_np(agent.dlogits[:agent.mb]), dz) < 1e-4
    assert _rel(_np(agent.dvalue[:agent.mb, 0]), dv) < 1e-4
    g = O.backward(model.layers, th0, x64, outs, {model.outputs[0]: dz, model.outputs[1]: dv[:, None]})
    assert _rel(_np(agent.grad), g) < 1e-4
    assert int(model.optimizer.iterations.item()) == 1
