"""TEST INFRASTRUCTURE ONLY -- float64 restatement of one ACER update
(xagents/acer/agent.py:171-347) for tests/test_acer_oracle.py and tests/test_gpu_acer.py.
Only tests/ import it.

Inputs are the batch as ACER.update_gradients sees it: rows env-major
[n_envs, n_steps + 1] (get_batch's reshape, acer/agent.py:164-169); logits / q / avg_logits
are the model's actor (pre-softmax), critic and the average model's actor outputs on every
row; mu_logits [n_envs, n_steps, A] the behaviour policy's actor logits; actions / rewards /
dones [n_envs, n_steps].

* retrace_returns: calculate_returns (195-208), a literal restatement of the reversed loop
  over flat_to_steps slices (69-82);
* acer_output_grads: the gradient with respect to the actor's probabilities of the loss
  calculate_losses returns (232-260), trust-region adjusted as calculate_grads does
  (276-288), pushed through the softmax to the logits; and the critic gradient of the
  value loss (292); bootstrap rows get zeros (clip_last_step 84-94);
* acer_loss_fixed: the non-trust-region loss (256-260) as a scalar function of
  (logits, q) with its stop-gradient inputs (returns, advantages, importance weights)
  held at the values of the given point, for finite-difference pinning.

Parity: TensorFlow is absent, so this restates the reference source (unpinned by TF
outputs); the gradient formulas are pinned by finite differences of acer_loss_fixed.
"""
import numpy as np


def softmax(z):
    z = np.asarray(z, np.float64)
    e = np.exp(z - z.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def _split(x, N, T):
    """[N*(T+1), ...] -> (steps [N, T, ...], bootstrap [N, ...])."""
    x = x.reshape(N, T + 1, *x.shape[1:])
    return x[:, :T], x[:, T]


def retrace_returns(rewards, dones, values, selected_q, importance_bar, gamma):
    """rewards / dones / selected_q / importance_bar [N, T]; values [N, T + 1]."""
    N, T = rewards.shape
    current = values[:, T].astype(np.float64)
    out = np.zeros((N, T))
    for i in reversed(range(T)):
        current = rewards[:, i] + gamma * current * (1.0 - dones[:, i])
        out[:, i] = current
        current = importance_bar[:, i] * (current - selected_q[:, i]) + values[:, i]
    return out


def _batch_terms(logits, q, mu_logits, actions, rewards, dones, gamma, eps):
    N, T = actions.shape
    p_all = softmax(logits)
    q = np.asarray(q, np.float64)
    values = (p_all * q).sum(-1).reshape(N, T + 1)
    p, _ = _split(p_all, N, T)
    qs, _ = _split(q, N, T)
    mu = softmax(mu_logits)
    idx = (np.arange(N)[:, None], np.arange(T)[None, :], actions)
    rho = p[idx] / (mu[idx] + eps)
    R = retrace_returns(rewards.astype(np.float64), dones.astype(np.float64), values,
                        qs[idx], np.minimum(1.0, rho), gamma)
    return p, qs, values, rho, R, idx


def acer_output_grads(logits, q, avg_logits, mu_logits, actions, rewards, dones, *,
                      gamma=0.99, eps=1e-6, importance_c=10.0, delta=1.0, entropy_coef=0.01,
                      value_coef=0.5, trust_region=True, n_total=None):
    """-> (dlogits [N(T+1), A], dq [N(T+1), A], returns [N, T], losses dict)."""
    N, T = actions.shape
    A = logits.shape[-1]
    n = n_total or N * T
    p, qs, values, rho, R, idx = _batch_terms(logits, q, mu_logits, actions, rewards, dones,
                                              gamma, eps)
    adv = R - values[:, :T]
    w = adv * np.minimum(importance_c, rho)
    onehot = np.eye(A)[actions]
    # d/dp of (sum gain + c_e n H), loss = -(action_loss - c_e H) n  (250-255)
    g = onehot * (w / (p[idx] + eps))[..., None] \
        - entropy_coef * (np.log(p + eps) + p / (p + eps))
    if trust_region:
        avg, _ = _split(softmax(avg_logits), N, T)
        k = -avg / (p + eps)
        adj = np.maximum(0.0, ((k * g).sum(-1) - delta) / ((k * k).sum(-1) + eps))
        g = g - adj[..., None] * k
        vcoef = value_coef
    else:
        adj = np.zeros((N, T))
        vcoef = value_coef * value_coef
    G = -g / n
    dz = p * (G - (p * G).sum(-1, keepdims=True))
    dq = np.zeros((N, T, A))
    dq[idx] = -(R - qs[idx]) * vcoef / n
    dlogits = np.zeros((N, T + 1, A))
    dlogits[:, :T] = dz
    dqf = np.zeros((N, T + 1, A))
    dqf[:, :T] = dq
    ent = -(p * np.log(p + eps)).sum(-1)
    losses = {'action_loss': -(np.log(p[idx] + eps) * w).mean(), 'entropy': ent.mean(),
              'value_loss': (0.5 * (R - qs[idx]) ** 2).mean() * value_coef,
              'adjusted': int((adj > 0).sum())}
    return dlogits.reshape(N * (T + 1), A), dqf.reshape(N * (T + 1), A), R, losses


def acer_loss_fixed(logits, q, point, mu_logits, actions, rewards, dones, *, gamma=0.99,
                    eps=1e-6, importance_c=10.0, entropy_coef=0.01, value_coef=0.5):
    """Non-trust-region loss (256-260) at (logits, q) with the stop-gradient terms
    (returns, advantage x truncated importance) frozen at `point` = (logits0, q0)."""
    N, T = actions.shape
    _, _, values0, rho0, R0, idx = _batch_terms(point[0], point[1], mu_logits, actions,
                                                rewards, dones, gamma, eps)
    w = (R0 - values0[:, :T]) * np.minimum(importance_c, rho0)
    p, _ = _split(softmax(logits), N, T)
    qs, _ = _split(np.asarray(q, np.float64), N, T)
    ent = (-(p * np.log(p + eps)).sum(-1)).mean()
    action_loss = -(np.log(p[idx] + eps) * w).mean()
    value_loss = (0.5 * (R0 - qs[idx]) ** 2).mean() * value_coef
    return action_loss + value_coef * value_loss - entropy_coef * ent


def ema(shadow, var, decay):
    """tf.train.ExponentialMovingAverage update without zero-debias."""
    return shadow - (shadow - var) * (1.0 - decay)
