"""BASELINE configs C3 / C4 / C5 at their single-GPU size: a few train
steps each with the counters and ring bookkeeping checked, plus one sampled minibatch's
raw gradient against the float64 restatement (oracle/nets_f64.py) at the full batch."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))
pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def _rel(got, want):
    want = np.asarray(want, np.float64)
    return float(np.linalg.norm(np.asarray(got, np.float64) - want) / np.linalg.norm(want))


def test_c3_dqn_32_envs_rb1_1m_batch_64(device):
    """C3: double DQN, 32 Pong-shaped envs, ReplayBuffer1 1M total (31,250 per env, the
    full 14 GB uint8 ring allocated), buffer batch 64 (2 per env)."""
    import nets_f64 as O
    from test_gpu_scale import _dqn_f64
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n = 32
    np.random.seed(3)
    random.seed(3)
    envs = create_envs('PongNoFrameskip-v4', n, device=device, seed=55)
    model = create_model(envs, 'dqn', 'model', seed=55, device=device,
                         optimizer_kwargs=dict(learning_rate=1e-4))
    bufs = create_buffers('dqn', 1_000_000, 64, n, initial_size=64 * n)
    assert [b.size for b in bufs] == [31250] * n and bufs[0].batch_size == 2
    agent = DQN(envs, model, bufs, double=True, seed=55, quiet=True, epsilon_start=0.5,
                epsilon_end=0.02)
    assert agent.replay.states.shape[:2] == (n, 31250) and agent.batch_size == 64
    # the 37632 x 512 layer's Keras Adam runs in its weight-gradient GEMM (xa_gemm_adam);
    # its raw gradient is written too on request, so the whole gradient is checked
    assert agent._fused_adam_layers()[0], 'the dense layer should take the fused Adam'
    agent.write_raw_grad = True
    agent.fill_buffers()
    assert [b.current_size for b in bufs] == [64] * n
    th0, tt0 = _np(model.theta), _np(agent.target_model.theta)
    agent.at_step_start()
    agent.train_step()
    torch.cuda.synchronize()
    dq64, loss64, g64 = _dqn_f64(agent, th0, tt0)
    # the TD head: diff = y - Q(s, a) cancels when the target is close to the estimate,
    # so an f32 diff carries an absolute error of a few ulps of |y| + |Q|, not of |diff|
    dq = _np(agent.dq)
    A = dq.shape[1]
    x64, outs = O.forward(model.layers, th0, agent.xb[:64].cpu().numpy(), model.input_shape)
    rows, act = np.arange(64), agent.b_act.cpu().numpy().reshape(-1)
    qa = outs[model.outputs[0]][rows, act]
    ya = qa - dq64[rows, act] * A / 2  # dq = -2 (y - Q) / A at the taken action
    scale = (np.abs(ya) + np.abs(qa)) * 2 / A
    err = np.abs(dq - dq64).sum(1)
    assert (err <= 1e-5 * np.abs(dq64).sum(1) + 8 * 2.0 ** -23 * scale).all(), \
        f'dq {_rel(dq, dq64):.2e}'
    # the backward through the CNN from the kernel's own head output: 1e-4
    # conv1's weight gradient sums 64 x 84 x 20 = 107,520 products of positive pixels with
    # mixed-sign gradients: f32 reductions of cancelling terms carry an error of a few ulps
    # of the sum of |terms| (S), which the bound adds to the 1e-4 relative tolerance
    S = np.zeros_like(g64)
    ex = agent.ex_online
    dev = {i: ex.outs[i][:64].cpu().numpy() for i, l in enumerate(model.layers)
           if l.kind != 'flatten'}
    gated, flips = O.adopt_gates(model.layers, outs, dev)
    g_head = O.backward(model.layers, th0, x64, gated, {model.outputs[0]: dq}, abs_terms=S)
    e = np.linalg.norm(_np(agent.grad) - g_head)
    bound = 1e-4 * np.linalg.norm(g_head) + 16 * 2.0 ** -24 * np.linalg.norm(S)
    sls, _ = O.param_slices(model.layers)
    per = []
    for sl in sls:
        for o, sh in sl or ():
            cnt = int(np.prod(sh))
            gg, ww, ss = _np(agent.grad)[o:o + cnt], g_head[o:o + cnt], S[o:o + cnt]
            per.append(f'{sh}: rel {_rel(gg, ww):.2e} err {np.linalg.norm(gg - ww):.2e} '
                       f'|g| {np.linalg.norm(ww):.2e} |S| {np.linalg.norm(ss):.2e} '
                       f'maxerr@{int(np.argmax(np.abs(gg - ww)))}')
    assert e <= bound, (f'backward {e / np.linalg.norm(g_head):.2e} (bound {bound:.3g}, '
                        f'err {e:.3g}, {flips} gate flips) ' + '; '.join(per))
    # end to end from the f64 head (its cancellation included), the device's gates
    g64 = O.backward(model.layers, th0, x64, gated, {model.outputs[0]: dq64})
    e = np.linalg.norm(_np(agent.grad) - g64)
    assert e <= 5e-4 * np.linalg.norm(g64) + 16 * 2.0 ** -24 * np.linalg.norm(S), \
        f'gradient {_rel(_np(agent.grad), g64):.2e}'
    assert _rel(_np(agent.td_loss), loss64) < 5e-4
    for _ in range(5):
        agent.at_step_start()
        agent.train_step()
        agent.at_step_end()
    torch.cuda.synchronize()
    assert agent.steps == 6 * n
    assert [b.current_size for b in bufs] == [64 + 6] * n
    assert int(model.optimizer.iterations.item()) == 6
    assert np.isfinite(_np(model.theta)).all()


def test_c4_ppo_cnn_128_env_shard(device):
    """C4, one rank's shard: PPO with the CNN actor-critic on 128 Breakout-shaped envs x 128
    steps (batch 16,384), 4 epochs x 4 minibatches of 4,096. ALL 16 optimizer steps of one
    train_step (xagents/ppo/agent.py:157-191) are teacher-forced: each step's gradient,
    taken at the device's own parameters theta_k on the minibatch the step drew, against
    the float64 restatement (oracle/nets_torch64.py on the test GPU, pinned to
    oracle/nets_f64.py by tests/test_oracle.py) at 1e-4 relative; then the applied clip +
    Keras Adam step against its float64 restatement from the device's own gradient and
    moments (moments 1e-5; the step theta_k+1 - theta_k 5e-5, since storing theta_k+1 in
    f32 rounds it by half an ulp of |theta|). The 1e-4 gradient bound (above the 1e-5 of
    the MLP path) covers ReLU gates that flip between the f32 and f64 forwards at
    pre-activations ~0 and the cancelling f32 sums of the conv weight gradients."""
    import nets_torch64 as OT
    import oracle as OR
    from test_gpu_cnn_onpolicy import _heads_grad_f64
    from xagents_amd import PPO
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_model
    n, T = 128, 128
    envs = create_envs('BreakoutNoFrameskip-v4', n, device=device, seed=55)
    model = create_model(envs, 'ppo', 'model', seed=55, device=device)
    agent = PPO(envs, model, n_steps=T, seed=55, quiet=True)
    assert agent.executor_path and agent.mb == 4096 and agent.n_mb == 4
    B, mb, E = n * T, agent.mb, agent.ppo_epochs
    opt = model.optimizer
    trace = []
    step_fn = agent._minibatch_step

    def traced(nn, k=None):
        before = (model.theta.clone(), opt.m.clone(), opt.v.clone())
        step_fn(nn, k)
        trace.append((k, nn) + before + (agent.grad.clone(),))

    agent._minibatch_step = traced
    np.random.seed(9)
    it0 = int(opt.iterations.item())
    agent.fused_train_step()
    agent._drain_episode_stats()
    torch.cuda.synchronize()
    del agent._minibatch_step
    assert [t[0] for t in trace] == list(range(E * 4)) and all(t[1] == mb for t in trace)
    assert int(opt.iterations.item()) - it0 == E * 4
    assert agent.steps == n * T
    slots = agent._slots_flat[:E * B].clone()
    act_all = agent.b_act.reshape(-1)
    logp_all, val_all, ret_all = (x.reshape(-1).double() for x in
                                  (agent.b_logp, agent.b_val, agent.b_ret))
    final = (model.theta.clone(), opt.m.clone(), opt.v.clone())
    f32 = lambda x: float(np.float32(x))  # noqa: E731
    o_logits, o_value = model.outputs
    for k, nn, th, m, v_, gd in trace:
        e, mi = divmod(k, 4)
        idx = slots[e * B + mi * mb:e * B + mi * mb + nn]
        x = agent.obs_buf[idx % T, idx // T]  # flat env-major index i = env * T + t
        thg = th.double().requires_grad_(True)
        _, outs = OT.forward(model.layers, thg, x, model.input_shape)
        logits, val = outs[o_logits], outs[o_value][:, 0]
        dz, dv = _heads_grad_f64(logits.detach().cpu().numpy(), val.detach().cpu().numpy(),
                                 act_all[idx].cpu().numpy(), logp_all[idx].cpu().numpy(),
                                 val_all[idx].cpu().numpy(), ret_all[idx].cpu().numpy(), 'ppo')
        g, = torch.autograd.grad([logits, outs[o_value]], [thg], grad_outputs=[
            torch.from_numpy(dz).to(device), torch.from_numpy(dv[:, None]).to(device)])
        del outs, logits, val, thg
        g = g.cpu().numpy()
        gn = _np(gd)
        assert _rel(gn, g) < 1e-4, f'step {k}: gradient {_rel(gn, g):.2e}'
        nxt = trace[k + 1][2:5] if k + 1 < len(trace) else final
        gc = OR.clip_by_global_norm_f64(gn, agent.grad_norm)[0]
        # the hyper-parameters as the f32 values TF's ApplyAdam computes with (1 - beta_2 of
        # the f32 0.999 is 0.99998713e-3, 1.3e-5 off the decimal 1e-3)
        th0n = _np(th)
        th1, m1, v1 = OR.keras_adam_f64(th0n, _np(m), _np(v_), gc, it0 + k + 1,
                                        f32(opt.learning_rate), f32(opt.beta_1),
                                        f32(opt.beta_2), f32(opt.epsilon))
        em, ev = _rel(_np(nxt[1]), m1), _rel(_np(nxt[2]), v1)
        assert em < 1e-5 and ev < 1e-5, f'step {k}: moments m {em:.2e} v {ev:.2e}'
        es = _rel(_np(nxt[0]) - th0n, th1 - th0n)
        assert es < 5e-5, f'step {k}: Adam step {es:.2e}'
    del trace
    # more full train steps
    it0 = int(opt.iterations.item())
    agent.fused_train_step()
    agent._drain_episode_stats()
    torch.cuda.synchronize()
    assert int(model.optimizer.iterations.item()) - it0 == 16
    assert agent.steps == 2 * n * T
    assert np.isfinite(_np(model.theta)).all()


@pytest.mark.parametrize('fused', [True, False], ids=['fused', 'executor'])
def test_c5_td3_64_envs_rb2(device, fused):
    """C5 on one GPU: TD3, 64 BipedalWalker-shaped envs, ReplayBuffer2 (1M total, per-buffer
    batch 100 // 64 = 1), gradient_steps 1; three chained gradient steps vs float64 on both
    the fused xa_td3_update and the layer-executor step: both critics' and (on the policy
    steps) the actor's raw gradients at 1e-4."""
    from test_gpu_scale import _critic_head_f64
    import nets_f64 as O
    from xagents_amd import TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n = 64
    np.random.seed(4)
    random.seed(4)
    envs = create_envs('BipedalWalker-v3', n, device=device, seed=55)
    kw = dict(seed=55, device=device)
    actor = create_model(envs, 'td3', 'actor_model', **kw)
    critic = create_model(envs, 'td3', 'critic_model', **kw)
    bufs = create_buffers('td3', 1_000_000, 100, n, initial_size=n * 64)
    assert bufs[0].batch_size == 1 and bufs[0].size == 1_000_000 // n
    agent = TD3(envs, actor, critic, bufs, gradient_steps=1, seed=55, quiet=True)
    assert agent.batch_size == 64
    if fused:
        assert agent._fused_args() is not None
    else:
        agent.__dict__['_fused'] = agent.__dict__['_fused_act'] = None
    agent.fill_buffers()
    fw = lambda m, th, x: O.forward(m.layers, th, x, m.input_shape)  # noqa: E731
    # three chained gradient steps, each teacher-forced at the device's own critic and
    # target parameters (the twin critics, the delayed actor and the Polyak targets move
    # in between): the critic gradients vs float64 at 1e-4 every step and the actor's
    # through the device's updated critic 1 (each update_weights(1) call runs its gradient
    # step 0, a policy step)
    for step in range(3):
        c1, c2 = _np(agent.critic.theta), _np(agent.critic2.theta)
        ac0 = _np(agent.actor.theta)
        tt = [_np(m.theta) for m in (agent.target_actor, agent.target_critic, agent.target_critic2)]
        it_a = int(agent.actor.optimizer.iterations.item())
        agent.update_weights(1)
        torch.cuda.synchronize()
        s, a, r, d, s2 = (_np(x) for x in (agent.s, agent.a, agent.r, agent.d, agent.s2))
        ta = fw(agent.target_actor, tt[0], s2)[1][agent.target_actor.outputs[0]]
        ta = np.clip(ta + _np(agent.noise), -1, 1)
        s2a2 = np.concatenate([s2, ta], 1)
        tv = np.minimum(*[fw(c, th, s2a2)[1][c.outputs[0]]
                          for c, th in zip((agent.target_critic, agent.target_critic2), tt[1:])])
        y = r[:, None] + (1 - d[:, None]) * np.float64(np.float32(0.99)) * tv
        for name, c, th, gd in (('critic 1', agent.critic, c1, agent.g_critic),
                                ('critic 2', agent.critic2, c2, agent.g_critic2)):
            x64, o = fw(c, th, np.concatenate([s, a], 1))
            dv, _ = _critic_head_f64(o[c.outputs[0]], y, None)
            g = O.backward(c.layers, th, x64, o, {c.outputs[0]: dv})
            e = _rel(_np(gd), g)
            assert e < 1e-4, f'step {step}: {name} gradient {e:.2e}'
        # update_weights(1) runs gradient step 0 of its call: a policy step every call
        assert int(agent.actor.optimizer.iterations.item()) == it_a + 1
        act = agent.actor
        xa, oa = fw(act, ac0, s)
        spa = np.concatenate([s, oa[act.outputs[0]]], 1)
        c1n = _np(agent.critic.theta)
        xc, oc = fw(agent.critic, c1n, spa)
        _, dx = O.backward(agent.critic.layers, c1n, xc, oc,
                           {agent.critic.outputs[0]: -np.ones((len(s), 1)) / len(s)},
                           want_input_grad=True)
        ga = O.backward(act.layers, ac0, xa, oa, {act.outputs[0]: dx[:, s.shape[1]:]})
        e = _rel(_np(agent.g_actor), ga)
        assert e < 1e-4, f'step {step}: actor gradient {e:.2e}'
    for _ in range(100):
        agent.train_step()
    agent._drain_episode_stats()
    torch.cuda.synchronize()
    it = int(agent.critic.optimizer.iterations.item())
    assert it == 3 + agent.games and agent.games > 0
    assert agent.steps == 100 * n
    assert np.isfinite(_np(agent.actor.theta)).all()
