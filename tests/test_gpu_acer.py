"""GPU tests of ACER (xagents_amd/acer): the xa_acer_grad kernel and xa_ema against the
float64 restatement (oracle/acer_f64.py), and one ACER update through the CNN against the
float64 layer restatement (oracle/nets_f64.py) + tf.clip_by_global_norm + Keras Adam."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu
sys.path.insert(0, str(ROOT / 'oracle'))


def _kernel(device, logits, q, avg, mu, act, rew, done, trust_region, **kw):
    from xagents_amd._lib import XaAcerArgs, call, stream
    N, T = act.shape
    A = logits.shape[1]
    t = lambda x, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(x)).to(device, dt)  # noqa
    tl, tq, ta, tmu = t(logits), t(q), t(avg), t(mu)
    tact, trew, tdone = t(act, torch.int32), t(rew), t(done)
    dz, dq = torch.empty(N * (T + 1), A, device=device), torch.empty(N * (T + 1), A,
                                                                     device=device)
    ret, el = torch.empty(N, T, device=device), torch.empty(N, 4, device=device)
    h = XaAcerArgs()
    h.n_envs, h.n_steps, h.n_actions, h.n_total = N, T, A, N * T
    h.logits, h.ld_logits, h.q, h.ld_q = tl.data_ptr(), A, tq.data_ptr(), A
    h.avg_logits, h.ld_avg, h.mu_logits = ta.data_ptr(), A, tmu.data_ptr()
    h.actions, h.rewards, h.dones = tact.data_ptr(), trew.data_ptr(), tdone.data_ptr()
    h.gamma, h.epsilon, h.importance_c = kw['gamma'], kw['eps'], kw['importance_c']
    h.delta, h.entropy_coef, h.value_coef = kw['delta'], kw['entropy_coef'], kw['value_coef']
    h.trust_region = int(trust_region)
    h.dlogits, h.ld_dlogits, h.dq, h.ld_dq = dz.data_ptr(), A, dq.data_ptr(), A
    h.returns, h.env_loss = ret.data_ptr(), el.data_ptr()
    call('xa_acer_grad', ctypes.byref(h), stream())
    torch.cuda.synchronize()
    return dz.cpu().numpy(), dq.cpu().numpy(), ret.cpu().numpy(), el.cpu().numpy()


@pytest.mark.parametrize('trust_region', [True, False])
@pytest.mark.parametrize('N,T,A', [(3, 5, 4), (16, 20, 6), (2, 100, 18)])
def test_acer_grad_kernel_vs_f64(device, trust_region, N, T, A):
    import acer_f64 as AO
    rng = np.random.default_rng(N * 100 + T)
    f = np.float32
    logits = (rng.normal(size=(N * (T + 1), A)) * 2).astype(f)
    q = rng.normal(size=(N * (T + 1), A)).astype(f)
    avg = (logits + 0.3 * rng.normal(size=logits.shape)).astype(f)
    mu = (rng.normal(size=(N, T, A)) * 2).astype(f)
    act = rng.integers(0, A, (N, T)).astype(np.int32)
    rew = rng.normal(size=(N, T)).astype(f)
    done = (rng.random((N, T)) < 0.1).astype(f)
    kw = dict(gamma=0.99, eps=1e-6, importance_c=10.0, delta=1.0, entropy_coef=0.01,
              value_coef=0.5)
    dz, dq, ret, el = _kernel(device, logits, q, avg, mu, act, rew, done, trust_region, **kw)
    rz, rq, rret, losses = AO.acer_output_grads(
        logits.astype(np.float64), q.astype(np.float64), avg.astype(np.float64),
        mu.astype(np.float64), act, rew, done, trust_region=trust_region, **kw)
    # Retrace returns: f32 recurrence vs f64 (1e-5 relative, north_star tolerance)
    np.testing.assert_allclose(ret, rret, rtol=1e-5, atol=1e-5 * np.abs(rret).max())
    scale = lambda x: np.abs(x).max()  # noqa: E731
    np.testing.assert_allclose(dz, rz, rtol=1e-4, atol=1e-5 * scale(rz))
    np.testing.assert_allclose(dq, rq, rtol=1e-4, atol=1e-5 * scale(rq))
    s = el.astype(np.float64).sum(0)
    n = N * T
    np.testing.assert_allclose(-s[0] / n, losses['action_loss'], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(s[1] / n, losses['entropy'], rtol=1e-5)
    np.testing.assert_allclose(s[2] / n * 0.5, losses['value_loss'], rtol=1e-4)
    if trust_region:
        assert int(s[3]) == losses['adjusted']


def test_ema_kernel(device):
    import acer_f64 as AO
    from xagents_amd._lib import call, stream
    rng = np.random.default_rng(3)
    s = rng.normal(size=100003).astype(np.float32)
    v = rng.normal(size=100003).astype(np.float32)
    ts, tv = torch.from_numpy(s).to(device), torch.from_numpy(v).to(device)
    call('xa_ema', ts.data_ptr(), tv.data_ptr(), s.size, 0.99, stream())
    torch.cuda.synchronize()
    ref = s - (s - v) * (np.float32(1) - np.float32(0.99))
    np.testing.assert_array_equal(ts.cpu().numpy(), ref)
    np.testing.assert_allclose(ts.cpu().numpy(), AO.ema(s.astype(np.float64), v, 0.99),
                               rtol=1e-6, atol=1e-7)


def _acer(device, n=3, t=5, trust_region=True, replay_ratio=0, initial=1):
    from xagents_amd import ACER
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('PongNoFrameskip-v4', n, device=device, seed=6)
    model = create_model(envs, 'acer', 'model', seed=4, device=device,
                         optimizer_kwargs=dict(learning_rate=1e-3))
    buffers = create_buffers('acer', 8 * n, 1, n, initial_size=initial * n)
    return ACER(envs, model, buffers, n_steps=t, seed=8, quiet=True,
                trust_region=trust_region, replay_ratio=replay_ratio, grad_norm=10.0)


@pytest.mark.parametrize('trust_region', [True, False])
def test_acer_update_vs_f64(device, trust_region):
    import acer_f64 as AO
    import nets_f64 as O
    import oracle as OR
    agent = _acer(device, trust_region=trust_region)
    model = agent.model
    assert model.layers[model.outputs[agent.actor_out]].activation == 'softmax'
    th0 = model.theta.cpu().numpy().astype(np.float64)
    slot = agent._acer_rollout()
    torch.cuda.synchronize()
    N, T = agent.n_envs, agent.n_steps
    frames = agent.r_frames[slot].cpu().numpy()       # [N, T + 1, 84, 84, 1]
    mu = agent.r_mu[slot].cpu().numpy().astype(np.float64)
    act = agent.r_act[slot].cpu().numpy().astype(np.int64)
    rew = agent.r_rew[slot].cpu().numpy()
    done = agent.r_done[slot].cpu().numpy()
    # the trajectory's frames: policy inputs then the get_states() bootstrap frame
    np.testing.assert_array_equal(frames[:, 0], agent.obs_buf[0].cpu().numpy())
    np.testing.assert_array_equal(frames[:, T], agent.envs.state.cpu().numpy())
    x = frames.reshape(N * (T + 1), *frames.shape[2:])
    x64, outs = O.forward(model.layers, th0, x, model.input_shape)
    logits = outs[model.outputs[agent.actor_out]]
    q = outs[model.outputs[agent.critic_out]]
    # behaviour logits stored by the rollout = the model's actor logits on the same frames
    np.testing.assert_allclose(mu, logits.reshape(N, T + 1, -1)[:, :T], rtol=1e-4, atol=1e-5)
    agent._acer_update(*agent._slot_views(slot))
    torch.cuda.synchronize()
    dz, dq, R, _ = AO.acer_output_grads(logits, q, logits, mu, act, rew, done,
                                        trust_region=trust_region, gamma=agent.gamma)
    np.testing.assert_allclose(agent.returns.cpu().numpy(), R, rtol=1e-4,
                               atol=1e-5 * np.abs(R).max())
    d = {model.outputs[agent.actor_out]: dz, model.outputs[agent.critic_out]: dq}
    g = O.backward(model.layers, th0, x64, outs, d)
    g = OR.clip_by_global_norm_f64(g, 10.0)[0]
    th1 = OR.keras_adam_f64(th0, 0, 0, g, 1, 1e-3, 0.9, 0.999, 1e-7)[0]
    got = model.theta.cpu().numpy()
    big = np.abs(g) > 1e-5 * np.abs(g).max()
    err = np.abs((got - th0)[big] - (th1 - th0)[big]).max() / 1e-3
    assert err < 3e-2, f'update mismatch {err:.3g} (units of lr)'
    # first ema.apply: the average model equals the updated weights
    np.testing.assert_array_equal(agent.avg_model.theta.cpu().numpy(), got)


def test_acer_train_steps_with_replay(device):
    import random
    agent = _acer(device, n=4, t=6, replay_ratio=3, initial=2)
    random.seed(1)
    np.random.seed(1)
    for _ in range(5):
        agent.train_step()
    agent._drain_episode_stats()
    torch.cuda.synchronize()
    assert agent.steps == 5 * 4 * 6
    np.random.seed(1)
    # replays from step 2 on; the count is drawn once per run (the reference draws it
    # while tracing its tf.function train_step, acer/agent.py:376-380)
    expected = 5 + 4 * np.random.poisson(3)
    assert int(agent.model.optimizer.iterations.item()) == expected
    assert np.isfinite(agent.model.theta.cpu().numpy()).all()
    # a gathered batch holds each env's sampled trajectory
    random.seed(7)
    slots = agent.sample_slots()
    frames, mu, act, rew, done = agent._gather(slots)
    torch.cuda.synchronize()
    for i, s in enumerate(slots):
        assert torch.equal(frames[i], agent.r_frames[s, i])
        assert torch.equal(mu[i], agent.r_mu[s, i])
        assert torch.equal(act[i], agent.r_act[s, i])
    # the average model moved towards the weights, not onto them
    th, av = agent.model.theta, agent.avg_model.theta
    assert not torch.equal(th, av)


def test_acer_graph_rollout_matches_eager(device):
    """The captured rollout (replayed from step 3 on) stores the same trajectories and
    yields the same weights as eager launches."""
    agents = []
    for use_graph in (True, False):
        ag = _acer(device, n=4, t=6)
        ag.use_graph = use_graph
        for _ in range(4):
            ag.train_step()
        torch.cuda.synchronize()
        agents.append(ag)
    g, e = agents
    assert g._graph is not None and e._graph is None
    for name in ('r_frames', 'r_act', 'r_mu', 'r_rew', 'r_done'):
        assert torch.equal(getattr(g, name), getattr(e, name)), name
    assert torch.equal(g.model.theta, e.model.theta)
    assert torch.equal(g.avg_model.theta, e.avg_model.theta)


@pytest.mark.parametrize('world', [2])
def test_acer_data_parallel_processes_on_one_gpu(device, world):
    """ACER's DP path (gradient all-reduce, replay count broadcast) with W processes sharing
    the test GPU over a gloo group (tests/acer_dp_worker.py)."""
    import os
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={world}', '--master-addr=127.0.0.1', f'--master-port={port}',
           str(ROOT / 'tests' / 'acer_dp_worker.py')]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110,
                         cwd=str(ROOT))
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    for r in range(world):
        assert f'ACER DP OK {r}' in out, out[-4000:]


def test_acer_fit_runs(device):
    """BaseAgent.fit (base.py:566-593) drives ACER.train_step until max_steps."""
    np.random.seed(2)
    agent = _acer(device, n=4, t=6, replay_ratio=1, initial=1)
    agent.fit(max_steps=4 * 6 * 3)
    assert agent.steps >= 4 * 6 * 3
    assert np.isfinite(agent.model.theta.cpu().numpy()).all()
    assert np.isfinite(agent.avg_model.theta.cpu().numpy()).all()
