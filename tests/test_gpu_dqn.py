"""GPU tests of the off-policy path: device replay rings (index semantics of the
reference's ReplayBuffer1 / ReplayBuffer2, bytes bit-exact), the fused env step, and one
DQN / double-DQN train step against the float64 restatement (targets, MSE gradient,
CNN backward, Keras Adam)."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _host_transitions(env, n_steps, actions):
    """The transitions step_envs would store, read from the env's host record."""
    rep_obs, rep_state = env.rep_obs.cpu().numpy(), env.rep_state.cpu().numpy()
    rew, done = env.rep_rew.cpu().numpy(), env.rep_done.cpu().numpy()
    state = env.s0.cpu().numpy().copy()
    out = []
    for t in range(n_steps):
        c = t % env.t_rec
        tr = [(state[i].copy(), actions[t][i], rew[i, c], done[i, c], rep_obs[i, c].copy())
              for i in range(env.n_envs)]
        out.append(tr)
        state = rep_state[:, c].copy()
    return out


@pytest.mark.parametrize('kind', ['rb1', 'rb2'])
def test_device_replay_matches_reference_buffers(device, kind):
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.buffers import ReplayBuffer1, ReplayBuffer2
    from xagents_amd.utils.common import create_model
    n, size, k, steps = 3, 5, 2, 13
    envs = create_envs('PongNoFrameskip-v4', n, device=device, seed=7)
    mk = (lambda: ReplayBuffer1(size, batch_size=k)) if kind == 'rb1' else (
        lambda: ReplayBuffer2(size, 5, batch_size=k))
    bufs = [mk() for _ in range(n)]
    model = create_model(envs, 'dqn', 'model', seed=3, device=device)
    agent = DQN(envs, model, bufs, seed=11, quiet=True)
    rng = np.random.default_rng(0)
    acts = rng.integers(0, 6, (steps, n)).astype(np.int32)
    for t in range(steps):
        agent._env_step(torch.from_numpy(acts[t]).to(device))
    torch.cuda.synchronize()
    # reference buffers fed with the same transitions
    ref = [mk() for _ in range(n)]
    for tr in _host_transitions(envs, steps, acts):
        for i in range(n):
            ref[i].append(*tr[i])
    assert [b.current_size for b in bufs] == [b.current_size for b in ref]
    random.seed(5)
    np.random.seed(5)
    samples = [b.get_sample() for b in ref]
    random.seed(5)
    np.random.seed(5)
    batch = agent.concat_buffer_samples()
    torch.cuda.synchronize()
    got = [t.cpu().numpy() for t in batch]
    for f in range(5):
        exp = np.concatenate([s[f] for s in samples]).reshape(got[f].shape)
        np.testing.assert_array_equal(got[f], exp.astype(got[f].dtype))


def _train_step_vs_oracle(device, double):
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    import oracle as OR
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=3)
    model = create_model(envs, 'dqn', 'model', seed=9, device=device,
                         optimizer_kwargs=dict(learning_rate=1e-3))
    bufs = create_buffers('dqn', 40, 4, 2, initial_size=20)
    agent = DQN(envs, model, bufs, double=double, seed=2, quiet=True, epsilon_start=0.0,
                epsilon_end=0.0, gamma=0.99)
    agent.fill_buffers()
    # make the target differ from the online net so double DQN matters
    agent.target_model.theta.mul_(0.97)
    th0 = model.theta.cpu().numpy().astype(np.float64)
    tt0 = agent.target_model.theta.cpu().numpy().astype(np.float64)
    opt = model.optimizer
    m0, v0 = opt.m.cpu().numpy(), opt.v.cpu().numpy()
    it0 = int(opt.iterations.item())
    agent.at_step_start()
    agent.train_step()
    torch.cuda.synchronize()
    B = agent.batch_size
    s = agent.xb[:B].cpu().numpy()
    s2 = agent.xb[B:].cpu().numpy()
    a = agent.b_act.cpu().numpy()
    r = agent.b_rew.cpu().numpy().astype(np.float64)
    d = agent.b_done.cpu().numpy()
    L, shape = model.layers, model.input_shape
    x64, outs = O.forward(L, th0, s, shape)
    q = outs[model.outputs[0]]
    qt = O.forward(L, tt0, s2, shape)[1][model.outputs[0]]
    if double:
        an = O.forward(L, th0, s2, shape)[1][model.outputs[0]].argmax(1)
        v = qt[np.arange(B), an]
    else:
        v = qt.max(1)
    v = np.where(d != 0, 0.0, v)
    y = v * 0.99 + r
    dq = np.zeros_like(q)
    dq[np.arange(B), a] = -2.0 * (y - q[np.arange(B), a]) / q.shape[1]
    g = O.backward(L, th0, x64, outs, {model.outputs[0]: dq})
    th1, _, _ = OR.keras_adam_f64(th0, m0, v0, g, it0 + 1, 1e-3, 0.9, 0.999, 1e-7)
    got = model.theta.cpu().numpy()
    step_ref = th1 - th0
    step_got = got - th0
    # Adam's first step is ~lr * sign(g): compare the update where |g| is not tiny
    big = np.abs(g) > 1e-6 * np.abs(g).max()
    err = np.abs(step_got[big] - step_ref[big]).max() / 1e-3
    assert err < 2e-2, f'Adam step mismatch {err:.3g} (units of lr)'
    assert agent.steps == 2


@pytest.mark.parametrize('double', [False, True])
def test_dqn_train_step_vs_f64(device, double):
    _train_step_vs_oracle(device, double)


def test_dqn_fit_epsilon_and_target_sync(device):
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('PongNoFrameskip-v4', 4, device=device, seed=1)
    model = create_model(envs, 'dqn', 'model', seed=9, device=device)
    bufs = create_buffers('dqn', 400, 8, 4, initial_size=40)
    agent = DQN(envs, model, bufs, seed=2, quiet=True, epsilon_decay_steps=200,
                target_sync_steps=40)
    agent.fit(max_steps=400)
    torch.cuda.synchronize()
    assert agent.steps >= 400
    assert agent.epsilon == pytest.approx(max(0.02, 1.0 - (agent.steps - 4) / 200))
    # 400 % 40 == 0 -> the target was synced at the last step
    np.testing.assert_array_equal(agent.target_model.theta.cpu().numpy(),
                                  model.theta.cpu().numpy())
    assert len(agent.total_rewards) == agent.games
    assert int(model.optimizer.iterations.item()) == agent.steps // 4


@pytest.mark.parametrize('double', [False, True])
def test_dqn_captured_learner_matches_eager(device, double, monkeypatch):
    """The learner phase (gather -> TD gradient -> backward -> Adam) replayed as a hipGraph
    from the third train step on (XA_DQN_LEARN_GRAPH=1; direct launches are the default)
    gives bit-identical weights to eager launches."""
    import random
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    out = []
    for use_graph in (False, True):
        monkeypatch.setenv('XA_DQN_LEARN_GRAPH', '1' if use_graph else '0')
        np.random.seed(4)
        random.seed(4)
        envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=3)
        model = create_model(envs, 'dqn', 'model', seed=9, device=device)
        agent = DQN(envs, model, create_buffers('dqn', 40, 4, 2, initial_size=20),
                    double=double, seed=2, quiet=True, epsilon_decay_steps=20,
                    target_sync_steps=6)
        agent.use_graph = use_graph
        agent.fill_buffers()
        for _ in range(8):
            agent.at_step_start()
            agent.train_step()
            agent.at_step_end()
        torch.cuda.synchronize()
        assert (getattr(agent, '_lgraph', None) is not None) == use_graph
        out.append([model.theta.cpu().numpy(), agent.target_model.theta.cpu().numpy(),
                    agent.model.optimizer.m.cpu().numpy(), agent.b_act.cpu().numpy()])
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('double', [False, True])
def test_fused_dense_adam_is_bit_identical(device, double):
    """The dense 37632 x 512 layer's Keras Adam inside its weight-gradient GEMM
    (xa_gemm_adam, the gradient never written) against the unfused path (gradient GEMM ->
    xa_clip_adam over every parameter): the same arithmetic per element, so parameters,
    moments and step counters are bit-identical after 3 chained train steps, and so are the
    raw gradients when the fused path is asked to write them."""
    import random
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    out = []
    for fused, raw in ((False, False), (True, False), (True, True)):
        envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=3)
        model = create_model(envs, 'dqn', 'model', seed=9, device=device,
                             optimizer_kwargs=dict(learning_rate=1e-3))
        bufs = create_buffers('dqn', 40, 4, 2, initial_size=20)
        np.random.seed(1)
        random.seed(1)
        agent = DQN(envs, model, bufs, double=double, seed=2, quiet=True, epsilon_start=0.0,
                    epsilon_end=0.0, gamma=0.99)
        if not fused:
            agent.__dict__['_fused_adam'] = ([], [])
        else:
            assert agent._fused_adam_layers()[0]
        agent.write_raw_grad = raw
        agent.fill_buffers()
        grads = []
        for _ in range(3):
            agent.at_step_start()
            agent.train_step()
            agent.at_step_end()
            grads.append(agent.grad.clone())
        torch.cuda.synchronize()
        opt = model.optimizer
        out.append(([t.cpu().numpy() for t in (model.theta, opt.m, opt.v, opt.iterations)],
                    [g.cpu().numpy() for g in grads]))
    for x, y in zip(out[0][0], out[1][0]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(out[0][0], out[2][0]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(out[0][1], out[2][1]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize('double', [False, True])
def test_fused_q_head_is_bit_identical(device, double, monkeypatch):
    """xa_dqn_head (argmax / TD target + gradient inside the Q head's row-dot launch) and
    xa_gemm_head (the 512-unit layer's split reduce + the head + that step in one launch)
    against the separate xa_gemm + xa_dqn_act / xa_dqn_td_grad launches: actions, the TD
    gradient and per-sample losses, parameters, moments and step counter bit-identical over
    3 chained greedy train steps, in every combination."""
    import random
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    out = []
    for fused, gemm_head in ((False, '0'), (True, '0'), (True, '1'), (False, '1')):
        monkeypatch.setenv('XA_GEMM_HEAD', gemm_head)
        envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=4)
        model = create_model(envs, 'dqn', 'model', seed=5, device=device,
                             optimizer_kwargs=dict(learning_rate=1e-3))
        bufs = create_buffers('dqn', 40, 4, 2, initial_size=20)
        np.random.seed(2)
        random.seed(2)
        agent = DQN(envs, model, bufs, double=double, seed=2, quiet=True, epsilon_start=0.0,
                    epsilon_end=0.0, gamma=0.99)
        agent.__dict__['_hf'] = fused
        assert agent._head_fused() == fused
        for ex in (agent.ex_act, agent.ex_online, agent.ex_target):
            assert (ex._fused_head_layer() is not None) == (gemm_head == '1')
        agent.fill_buffers()
        rec = []
        for _ in range(3):
            agent.at_step_start()
            agent.train_step()
            agent.at_step_end()
            rec += [agent.actions.clone(), agent.dq.clone(), agent.td_loss.clone()]
        torch.cuda.synchronize()
        opt = model.optimizer
        out.append([t.cpu().numpy() for t in rec + [model.theta, opt.m, opt.v, opt.iterations]])
    for other in out[1:]:
        for x, y in zip(out[0], other):
            np.testing.assert_array_equal(x, y)
