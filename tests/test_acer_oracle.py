"""CPU tests of the ACER float64 restatement (oracle/acer_f64.py) and the host-side replay
index rule of xagents_amd.acer (no GPU)."""
import random
import sys
from collections import deque
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))


def _batch(seed, N=3, T=5, A=4):
    rng = np.random.default_rng(seed)
    logits = rng.normal(size=(N * (T + 1), A))
    q = rng.normal(size=(N * (T + 1), A))
    avg = logits + 0.3 * rng.normal(size=logits.shape)
    mu = rng.normal(size=(N, T, A))
    act = rng.integers(0, A, (N, T))
    rew = rng.normal(size=(N, T))
    done = (rng.random((N, T)) < 0.2).astype(np.float64)
    return logits, q, avg, mu, act, rew, done


def test_retrace_known_answers():
    import acer_f64 as AO
    N, T = 2, 4
    rng = np.random.default_rng(0)
    r, v, qa = rng.normal(size=(N, T)), rng.normal(size=(N, T + 1)), rng.normal(size=(N, T))
    d = np.zeros((N, T))
    d[0, 1] = 1
    # importance 0: one-step TD targets r_t + gamma V_{t+1} (1 - d_t)
    R0 = AO.retrace_returns(r, d, v, qa, np.zeros((N, T)), 0.9)
    np.testing.assert_allclose(R0, r + 0.9 * v[:, 1:] * (1 - d))
    # importance 1 with Q_a = V: discounted n-step returns bootstrapped on V_T
    R1 = AO.retrace_returns(r, d, v, v[:, :T], np.ones((N, T)), 0.9)
    ref = np.zeros((N, T))
    cur = v[:, T]
    for t in reversed(range(T)):
        cur = r[:, t] + 0.9 * cur * (1 - d[:, t])
        ref[:, t] = cur
    np.testing.assert_allclose(R1, ref)


def test_gradient_pinned_by_finite_differences():
    import acer_f64 as AO
    logits, q, avg, mu, act, rew, done = _batch(1)
    kw = dict(gamma=0.99, eps=1e-6, importance_c=10.0, entropy_coef=0.01, value_coef=0.5)
    dz, dq, _, _ = AO.acer_output_grads(logits, q, avg, mu, act, rew, done, trust_region=False,
                                        **kw)
    f = lambda z, qq: AO.acer_loss_fixed(z, qq, (logits, q), mu, act, rew, done, **kw)  # noqa
    h = 1e-6
    for arr, grad, which in ((logits, dz, 0), (q, dq, 1)):
        for idx in [(0, 0), (1, 2), (5, 3), (7, 1), (12, 0), (17, 2)]:
            plus, minus = arr.copy(), arr.copy()
            plus[idx] += h
            minus[idx] -= h
            args_p = (plus, q) if which == 0 else (logits, plus)
            args_m = (minus, q) if which == 0 else (logits, minus)
            fd = (f(*args_p) - f(*args_m)) / (2 * h)
            assert abs(fd - grad[idx]) < 1e-7 + 1e-5 * abs(fd), (which, idx, fd, grad[idx])


def test_trust_region_projection():
    import acer_f64 as AO
    logits, q, avg, mu, act, rew, done = _batch(2)
    N, T, A = 3, 5, 4
    common = dict(gamma=0.99, eps=1e-6, importance_c=10.0, entropy_coef=0.01, value_coef=0.5)
    # an unreachable delta switches the adjustment off: the actor gradient of both modes agree
    dz_tr, dq_tr, _, l_tr = AO.acer_output_grads(logits, q, avg, mu, act, rew, done,
                                                 trust_region=True, delta=1e12, **common)
    dz_pl, dq_pl, _, _ = AO.acer_output_grads(logits, q, avg, mu, act, rew, done,
                                              trust_region=False, **common)
    np.testing.assert_allclose(dz_tr, dz_pl, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(dq_tr * 0.5, dq_pl, rtol=1e-12)  # coef vs coef^2
    assert l_tr['adjusted'] == 0
    # delta 0: rows whose k . g exceeds it get adjusted (calculate_grads 281-287)
    _, _, _, l = AO.acer_output_grads(logits, q, avg, mu, act, rew, done, trust_region=True,
                                      delta=0.0, **common)
    assert l['adjusted'] > 0


def test_sample_slots_follow_reference_deque_sampling():
    """ACER.sample_slots == random.sample(deque, 1) per env in env order
    (concat_buffer_samples base.py:344-368 over ReplayBuffer1.get_sample)."""
    from xagents_amd.acer.agent import ACER
    agent = object.__new__(ACER)
    agent.n_envs, agent.capacity = 3, 5
    deques = [deque(maxlen=5) for _ in range(3)]
    for count in (1, 3, 5, 6, 9, 13):
        while len(deques[0]) < min(count, 5) or deques[0][-1] != count - 1:
            n = (deques[0][-1] + 1) if deques[0] else 0
            for dq in deques:
                dq.append(n)  # trajectory id = append counter
        agent.count = count
        random.seed(count)
        slots = agent.sample_slots()
        random.seed(count)
        ids = [random.sample(dq, 1)[0] for dq in deques]
        assert list(slots) == [i % 5 for i in ids]


def test_acer_default_model_units_and_softmax_actor():
    """create_model('acer') (common.py:447-487): the registered cnn-actor-critic.cfg, output
    units [n_actions, n_actions], softmax actor output first, critic Q over the actions."""
    import xagents_amd
    from xagents_amd.envs import Box, Discrete
    from xagents_amd.utils.common import create_model

    class _Env:
        observation_space = Box(0, 255, (84, 84, 1), np.uint8)
        action_space = Discrete(6)

    assert xagents_amd.agents['acer']['model']['cnn']
    m = create_model(_Env(), 'acer', 'model', seed=1, device='cpu')
    outs = [m.layers[i] for i in m.outputs]
    assert [l.units for l in outs] == [6, 6]
    assert outs[0].activation == 'softmax' and outs[1].activation in (None, 'linear')
