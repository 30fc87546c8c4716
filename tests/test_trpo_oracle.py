"""The TRPO float64 restatement (oracle/trpo_f64.py) pinned on CPU: its Fisher-vector
product equals a central finite difference of the mean-KL gradient (the Hessian-vector
product the reference's double tape computes, xagents/trpo/agent.py:121-148), and its
surrogate gradient equals a finite difference of surrogate_loss (trpo/agent.py:200-223)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))
import nets_f64 as O  # noqa: E402
import trpo_f64 as TR  # noqa: E402


def _actor(seed=3):
    from xagents_amd.nets import LayerSpec
    layers = [LayerSpec('dense-0', 'dense', units=8, activation='tanh', input_index=-1,
                        in_features=4),
              LayerSpec('dense-1', 'dense', units=8, activation='relu', input_index=0,
                        in_features=8),
              LayerSpec('dense-2', 'dense', units=3, activation=None, input_index=1,
                        in_features=8, output=True)]
    _, P = O.param_slices(layers)
    rng = np.random.default_rng(seed)
    return layers, rng.normal(size=P) * 0.7


def test_fvp_is_kl_hessian_vector_product():
    layers, theta = _actor()
    rng = np.random.default_rng(4)
    x = rng.normal(size=(11, 4))
    v = rng.normal(size=theta.size)
    _, outs = O.forward(layers, theta, x, (4,))
    p_old = np.exp(TR.log_softmax(outs[2]))

    def kl_grad(th):
        _, o = O.forward(layers, th, x, (4,))
        p_new = np.exp(TR.log_softmax(o[2]))
        # d mean KL(old || new) / d logits_new = (p_new - p_old) / n
        return O.backward(layers, th, x, o, {2: (p_new - p_old) / x.shape[0]})

    eps = 1e-5
    fd = (kl_grad(theta + eps * v) - kl_grad(theta - eps * v)) / (2 * eps)
    got = TR.fvp(layers, theta, x, v, damping=0.0)
    assert np.abs(got - fd).max() < 1e-6 * max(1.0, np.abs(fd).max())
    got_d = TR.fvp(layers, theta, x, v, damping=0.1)
    np.testing.assert_allclose(got_d - got, 0.1 * v, rtol=1e-12, atol=1e-12)


def test_surrogate_gradient_finite_difference():
    layers, theta = _actor(5)
    rng = np.random.default_rng(6)
    x = rng.normal(size=(9, 4))
    actions = rng.integers(0, 3, 9)
    adv = rng.normal(size=9)
    _, outs = O.forward(layers, theta, x, (4,))
    old = outs[2]
    dl = TR.surrogate_grad_logits(old, actions, adv, 0.01)
    g = O.backward(layers, theta, x, outs, {2: dl})
    v = rng.normal(size=theta.size)
    eps = 1e-6

    def gain(th):
        _, o = O.forward(layers, th, x, (4,))
        lpn, lpo = TR.log_softmax(o[2]), TR.log_softmax(old)
        idx = np.arange(9)
        ratio = np.exp(lpn[idx, actions] - lpo[idx, actions])
        pn = np.exp(lpn)
        return (ratio * adv).mean() + 0.01 * (-(pn * lpn).sum(-1)).mean()

    fd = (gain(theta + eps * v) - gain(theta - eps * v)) / (2 * eps)
    assert abs(g @ v - fd) < 1e-6 * max(1.0, abs(fd))
    s_fd = (TR.surrogate(O.forward(layers, theta + eps * v, x, (4,))[1][2], old, actions, adv,
                         0.01)[0]
            - TR.surrogate(O.forward(layers, theta - eps * v, x, (4,))[1][2], old, actions,
                           adv, 0.01)[0]) / (2 * eps)
    assert abs(s_fd - fd) < 1e-8
