"""TEST INFRASTRUCTURE ONLY -- float64 restatement of one TRPO update
(xagents/trpo/agent.py:121-348) for tests/test_gpu_trpo.py. Only tests/ import it.

Given the batch a rollout produced (env-major states, actions, returns, values), it runs
the reference's train_step math in float64 on the .cfg models (oracle/nets_f64.py):
advantages normalised over the batch (321-324); surrogate_loss = mean(ratio adv) +
entropy_coef mean(H) and its gradient (200-223); conjugate gradients (150-177) with the
Fisher-vector product of the KL Hessian at actor == old actor, i.e. the Gauss-Newton form
J^T (diag(p) - p p^T) J v / n + damping v on states[::fvp_n_steps] (121-148), J v by
forward-mode differentiation; shs, the Lagrange multiplier and the backtracking line
search (235-278, 329-345); critic_iterations x PPO minibatches of mean((V - R)^2) with
Keras Adam (280-299), minibatch permutations supplied by the caller.
Parity: TensorFlow is absent, so this restates the reference source (unpinned by TF
outputs); the Fisher-vector product is pinned in the tests by finite differences of the
surrogate-free KL gradient.
"""
import numpy as np

import nets_f64 as O


def log_softmax(z):
    m = z.max(-1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(-1, keepdims=True))


def dense_jvp(layers, theta, x, outs, v):
    """Forward-mode tangents of every layer output along parameter direction v (dense
    and flatten layers; relu / tanh / linear)."""
    sls, _ = O.param_slices(layers)
    touts = []
    B = x.shape[0]
    for i, l in enumerate(layers):
        src = x if l.input_index == -1 else outs[l.input_index]
        tsrc = None if l.input_index == -1 else touts[l.input_index]
        if l.kind == 'flatten':
            touts.append(None if tsrc is None else tsrc.reshape(B, -1))
            continue
        assert l.kind == 'dense', 'the oracle JVP covers dense models'
        W, _ = O._weights(theta, sls[i])
        dW, db = O._weights(v, sls[i])
        dz = src.reshape(B, -1) @ dW + db
        if tsrc is not None:
            dz = dz + tsrc.reshape(B, -1) @ W
        y = outs[i]
        if l.activation == 'relu':
            dz = dz * (y > 0)
        elif l.activation == 'tanh':
            dz = dz * (1.0 - y * y)
        touts.append(dz)
    return touts


def surrogate(logits_new, logits_old, actions, adv, entropy_coef):
    lpn, lpo = log_softmax(logits_new), log_softmax(logits_old)
    idx = np.arange(len(actions))
    ratio = np.exp(lpn[idx, actions] - lpo[idx, actions])
    pn, po = np.exp(lpn), np.exp(lpo)
    H = -(pn * lpn).sum(-1)
    kl = (po * (lpo - lpn)).sum(-1)
    return (ratio * adv).mean() + entropy_coef * H.mean(), kl.mean(), ratio, pn, lpn, H


def surrogate_grad_logits(logits, actions, adv, entropy_coef):
    """d surrogate_loss / d logits at logits_new == logits_old (ratio = 1)."""
    n, A = logits.shape
    lp = log_softmax(logits)
    p = np.exp(lp)
    H = -(p * lp).sum(-1, keepdims=True)
    onehot = np.zeros_like(p)
    onehot[np.arange(n), actions] = 1.0
    return (adv[:, None] * (onehot - p) + entropy_coef * (-p * (lp + H))) / n


def fvp(layers, theta, x, v, damping):
    _, outs = O.forward(layers, theta, x, x.shape[1:])
    out_i = [i for i, l in enumerate(layers) if l.output][0]
    t = dense_jvp(layers, theta, x.astype(np.float64), outs, v)[out_i]
    p = np.exp(log_softmax(outs[out_i]))
    u = p * (t - (p * t).sum(-1, keepdims=True)) / x.shape[0]
    return O.backward(layers, theta, x.astype(np.float64), outs, {out_i: u}) + damping * v


def conjugate_gradients(layers, theta, x, g, iters, tol, damping):
    p, r = g.copy(), g.copy()
    sol = np.zeros_like(g)
    rdr = r @ r
    it = 0
    while it < iters and rdr > tol:
        z = fvp(layers, theta, x, p, damping)
        v = rdr / (p @ z)
        sol += v * p
        r -= v * z
        new = r @ r
        p = r + (new / rdr) * p
        rdr = new
        it += 1
    return sol


def keras_adam(theta, m, v, g, t, lr=7e-4, b1=0.9, b2=0.999, eps=1e-7):
    lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    return theta - lr_t * m / (np.sqrt(v) + eps), m, v


def trpo_update(actor_layers, actor_theta, critic_layers, critic_theta, states, actions,
                returns, values, perms, *, entropy_coef=0.01, max_kl=1e-3, cg_iterations=10,
                cg_residual_tolerance=1e-10, cg_damping=1e-3, actor_iterations=10,
                critic_iterations=3, fvp_n_steps=5, mini_batch_size=None, adam_t0=0,
                lr=7e-4):
    """Returns (new actor theta, new critic theta, diagnostics)."""
    x = states.astype(np.float64)
    B = x.shape[0]
    at = actor_theta.astype(np.float64)
    out_i = [i for i, l in enumerate(actor_layers) if l.output][0]
    adv = returns.astype(np.float64) - values.astype(np.float64)
    adv = (adv - adv.mean()) / adv.std()
    _, outs = O.forward(actor_layers, at, x, x.shape[1:])
    old_logits = outs[out_i]
    dl = surrogate_grad_logits(old_logits, actions, adv, entropy_coef)
    g = O.backward(actor_layers, at, x, outs, {out_i: dl})
    loss0 = surrogate(old_logits, old_logits, actions, adv, entropy_coef)[0]
    xs = x[::fvp_n_steps]
    step = conjugate_gradients(actor_layers, at, xs, g, cg_iterations, cg_residual_tolerance,
                               cg_damping)
    shs = 0.5 * step @ fvp(actor_layers, at, xs, step, cg_damping)
    full_step = step / np.sqrt(shs / max_kl)
    lr_ls = 1.0
    new_theta = at
    for _ in range(actor_iterations):
        cand = at + full_step * lr_ls
        _, o2 = O.forward(actor_layers, cand, x, x.shape[1:])
        loss, kl = surrogate(o2[out_i], old_logits, actions, adv, entropy_coef)[:2]
        if np.isfinite([loss, kl]).all() and kl <= max_kl * 1.5 and loss - loss0 > 0:
            new_theta = cand
            break
        lr_ls *= 0.5
    # critic
    ct = critic_theta.astype(np.float64)
    cout = [i for i, l in enumerate(critic_layers) if l.output][0]
    m = np.zeros_like(ct)
    vv = np.zeros_like(ct)
    t = adam_t0
    mb = mini_batch_size or B
    ret = returns.astype(np.float64)
    for perm in perms:
        for i in range(0, B, mb):
            idx = perm[i:i + mb]
            xb = x[idx]
            _, co = O.forward(critic_layers, ct, xb, xb.shape[1:])
            v = co[cout][:, 0]
            dv = (2.0 * (v - ret[idx]) / len(idx))[:, None]
            gc = O.backward(critic_layers, ct, xb, co, {cout: dv})
            t += 1
            ct, m, vv = keras_adam(ct, m, vv, gc, t, lr=lr)
    return new_theta, ct, {'flat_grads': g, 'step': step, 'shs': shs, 'ls_lr': lr_ls,
                           'loss0': loss0}
