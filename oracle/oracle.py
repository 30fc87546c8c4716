"""TEST INFRASTRUCTURE ONLY -- the parity oracle for libxagents_hip.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product (xagents_amd) never does.

Two layers:
1. `lib()`: ctypes handle of oracle/_build/libxa_oracle.so (oracle/xa_oracle.c),
   the exact f32 restatement of the kernels' operation order -> bit-exact checks
   (integer actions, rollout buffers, GAE / n-step returns, Adam step).
2. float64 numpy restatement of the reference's TF math, used for tolerance
   checks of losses and gradients (rtol 1e-5 in f32 terms):
     actor-critic forward  xagents/a2c/agent.py:65-94, xagents/utils/common.py:239-258
     PPO loss              xagents/ppo/agent.py:112-133 (+ adv normalisation 180-183)
     A2C loss              xagents/a2c/agent.py:199-214
     tf.clip_by_global_norm + Keras Adam   ppo/agent.py:135-137
   Gradients are analytic (TF autodiff semantics for max/clip_by_value ties) and are
   themselves pinned by central finite differences in tests/test_oracle.py.

Parity status: GAE, n-step returns, env-major batching and the replay buffers are
pinned to the reference's own numpy code (tests/golden/*.npz). The TF/TFP math
(losses, autodiff, Keras Adam, Categorical) cannot run here (no TensorFlow): that
part is restated from the reference source and pinned by known-answer tests only.
"""
import ctypes
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_uint32, c_uint64, c_void_p
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / '_build' / 'libxa_oracle.so'
H = 64

_lib = None


def build():
    subprocess.run(['make', '-s', '-C', str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / 'xa_oracle.c').stat().st_mtime:
            build()
        _lib = ctypes.CDLL(str(LIB_PATH))
        _lib.xo_expf.restype = c_float
        _lib.xo_expf.argtypes = [c_float]
        _lib.xo_mlp_param_count.restype = c_int
        _lib.xo_clip_adam.argtypes = [c_void_p] * 4 + [c_int] + [c_float] * 6 + [c_int, c_void_p]
        _lib.xo_gae.argtypes = [c_void_p] * 5 + [c_int, c_int, c_float, c_float]
        _lib.xo_nstep.argtypes = [c_void_p] * 4 + [c_int, c_int, c_float]
        _lib.xo_philox.argtypes = [c_uint32] * 6 + [c_void_p]
        _lib.xo_shuffle_perm.argtypes = [c_int, c_int, c_uint64, c_uint64, c_void_p]
        _lib.xo_walker_step.argtypes = ([c_int, c_void_p, c_void_p, c_void_p, ctypes.c_long,
                                         c_uint64, c_int] + [c_void_p] * 4)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# ----------------------------------------------------------------------------
# exact f32 restatement (C)
# ----------------------------------------------------------------------------
def math_f32(fn, x):
    x = _f32(x)
    y = np.empty_like(x)
    getattr(lib(), f'xo_{fn}f_arr')(_p(x), _p(y), c_int(x.size))
    return y


def gae(rewards, values, dones, next_values, gamma, gamma_lam):
    """env-major rewards/values [N,T], dones [N,T+1], next_values [N]."""
    rewards, values, dones, nv = map(_f32, (rewards, values, dones, next_values))
    n, t = rewards.shape
    out = np.empty_like(rewards)
    lib().xo_gae(_p(rewards), _p(values), _p(dones), _p(nv), _p(out), n, t, gamma, gamma_lam)
    return out


def nstep(rewards, dones, next_values, gamma):
    rewards, dones, nv = map(_f32, (rewards, dones, next_values))
    n, t = rewards.shape
    out = np.empty_like(rewards)
    lib().xo_nstep(_p(rewards), _p(dones), _p(nv), _p(out), n, t, gamma)
    return out


def mlp_forward(theta, obs, n_actions, actions=None, uniforms=None):
    theta, obs = _f32(theta), _f32(obs)
    b, obs_dim = obs.shape
    act = np.empty(b, np.int32)
    logp, value, ent = (np.empty(b, np.float32) for _ in range(3))
    logits = np.empty((b, n_actions), np.float32)
    a_in = None if actions is None else np.ascontiguousarray(actions, np.int32)
    u = None if uniforms is None else _f32(uniforms)
    lib().xo_mlp_forward(_p(theta), _p(obs), c_int(b), c_int(obs_dim), c_int(n_actions),
                         _p(a_in), _p(u), _p(act), _p(logp), _p(value), _p(ent), _p(logits))
    return (act if actions is None else a_in), logp, value, ent, logits


def walker_step(state, episode, actions, seed, reset_only=False):
    """Mirror of xa_walker_step (the BipedalWalker-v3 device stand-in): state [N, 18] f32
    and episode [N] i32 are mutated in place; actions [N, 4] f32 (ignored on reset).
    Returns (obs [N, 24], post [N, 24], reward [N], done [N]) (obs / reward / done are
    None on reset)."""
    n = state.shape[0]
    assert state.dtype == np.float32 and state.flags.c_contiguous and state.shape[1] == 18
    assert episode.dtype == np.int32 and episode.flags.c_contiguous
    post = np.empty((n, 24), np.float32)
    if reset_only:
        lib().xo_walker_step(c_int(n), _p(state), _p(episode), None, 4, c_uint64(seed), 1,
                             None, _p(post), None, None)
        return None, post, None, None
    act = _f32(actions).reshape(n, 4)
    obs = np.empty((n, 24), np.float32)
    rew = np.empty(n, np.float32)
    done = np.empty(n, np.float32)
    lib().xo_walker_step(c_int(n), _p(state), _p(episode), _p(act), 4, c_uint64(seed), 0,
                         _p(obs), _p(post), _p(rew), _p(done))
    return obs, post, rew, done


def mlp_rollout(theta, n_actions, env, n_steps, uniforms=None, seed=0, ctr=0,
                return_kind=1, gamma=0.99, gamma_lam=None):
    """Mirror of xa_mlp_rollout. `env` is a dict of numpy arrays (mutated in place):
    kind, state [N,obs], done [N], cursor [N] i32, ep_return [N], and for replay
    rep_obs/rep_state/rep_rew/rep_done, for cartpole state64 [N,4] f64."""
    theta = _f32(theta)
    n, obs_dim = env['state'].shape
    T = n_steps
    out = dict(obs=np.empty((n, T, obs_dim), np.float32), act=np.empty((n, T), np.int32),
               logp=np.empty((n, T), np.float32), val=np.empty((n, T), np.float32),
               ent=np.empty((n, T), np.float32), rew=np.empty((n, T), np.float32),
               done=np.empty((n, T + 1), np.float32), epret=np.empty((n, T), np.float32),
               next_val=np.empty(n, np.float32), ret=np.empty((n, T), np.float32))
    kind = env['kind']
    t_rec = env['rep_obs'].shape[1] if kind == 0 else 0
    if gamma_lam is None:
        gamma_lam = float(np.float32(0.99 * 0.95))
    u = None if uniforms is None else _f32(uniforms)
    L = lib()
    L.xo_mlp_rollout(
        c_int(n), c_int(T), c_int(obs_dim), c_int(n_actions), _p(theta), c_int(kind),
        _p(env['state']), _p(env.get('state64')), _p(env['done']), _p(env['cursor']),
        _p(env['ep_return']), _p(env.get('rep_obs')), _p(env.get('rep_state')),
        _p(env.get('rep_rew')), _p(env.get('rep_done')), c_int(t_rec), c_int(500), _p(u),
        c_uint64(seed), c_uint64(ctr), _p(out['obs']), _p(out['act']), _p(out['logp']),
        _p(out['val']), _p(out['ent']), _p(out['rew']), _p(out['done']), _p(out['epret']),
        _p(out['next_val']), _p(out['ret']), c_int(return_kind), c_float(gamma),
        c_float(gamma_lam))
    return out


def clip_adam(theta, m, v, g, t, lr, beta1, beta2, eps, clip_norm=0.0, grad_scale=1.0):
    """In-place on float32 copies; returns (theta, m, v, gnorm)."""
    theta, m, v, g = (_f32(x).copy() for x in (theta, m, v, g))
    gn = np.zeros(1, np.float32)
    lib().xo_clip_adam(_p(theta), _p(m), _p(v), _p(g), theta.size, grad_scale, clip_norm, lr,
                       beta1, beta2, eps, t, _p(gn))
    return theta, m, v, float(gn[0])


def philox(c, k):
    out = np.zeros(4, np.uint32)
    lib().xo_philox(*[int(x) & 0xffffffff for x in c], *[int(x) & 0xffffffff for x in k], _p(out))
    return out


def shuffle_perm(n, epoch, seed, ctr):
    out = np.empty(n, np.int32)
    lib().xo_shuffle_perm(n, epoch, c_uint64(seed), c_uint64(ctr), _p(out))
    return out


# ----------------------------------------------------------------------------
# float64 restatement of the reference TF math
# ----------------------------------------------------------------------------
def unpack(theta, obs_dim, A):
    theta = np.asarray(theta, np.float64)
    shapes = [(obs_dim, H), (H,), (H, H), (H,), (H, A), (A,), (H, 1), (1,)]
    out, off = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(theta[off:off + n].reshape(s))
        off += n
    return out


def pack(parts):
    return np.concatenate([np.asarray(p, np.float64).ravel() for p in parts])


def forward_f64(theta, obs, obs_dim, A):
    """Keras Dense stack: y = x @ W + b (xagents/utils/common.py:239-258)."""
    W1, b1, W2, b2, W3, b3, W4, b4 = unpack(theta, obs_dim, A)
    x = np.asarray(obs, np.float64)
    h1 = np.tanh(x @ W1 + b1)
    h2 = np.tanh(h1 @ W2 + b2)
    return x, h1, h2, h2 @ W3 + b3, (h2 @ W4 + b4)[:, 0]


def log_softmax(z):
    m = z.max(-1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(-1, keepdims=True))


def normalize_advantages(returns, values, eps=1e-8):
    """(adv - mean) / (population std + eps) (xagents/ppo/agent.py:180-183)."""
    adv = np.asarray(returns, np.float64) - np.asarray(values, np.float64)
    return (adv - adv.mean()) / (adv.std() + eps)


def ac_loss_grad_f64(theta, obs, actions, returns, old_values, A, kind='ppo', old_logp=None,
                     advantages=None, clip=0.1, ent_coef=0.01, v_coef=0.5):
    """Loss terms and d(loss)/d(theta) in float64.

    PPO (xagents/ppo/agent.py:112-133):
        L = mean(max(-adv*r, -adv*clip(r,1-c,1+c))) - ent_coef*mean(H)
            + v_coef * 0.5*mean(max((v-R)^2, (v_clip-R)^2)),  r = exp(logp-old_logp)
    A2C (xagents/a2c/agent.py:199-214), adv = R - V_old:
        L = -mean(adv*logp) - ent_coef*mean(H) + v_coef*mean((v-R)^2)
    TF tie semantics: tf.maximum sends the gradient to the first argument when
    x >= y; tf.clip_by_value passes it when lo <= x <= hi.
    """
    obs = np.asarray(obs, np.float64)
    n, obs_dim = obs.shape
    W1, b1, W2, b2, W3, b3, W4, b4 = unpack(theta, obs_dim, A)
    x, h1, h2, logits, v = forward_f64(theta, obs, obs_dim, A)
    lsm = log_softmax(logits)
    p = np.exp(lsm)
    a = np.asarray(actions, np.int64)
    logp = lsm[np.arange(n), a]
    H_ = -(p * lsm).sum(-1)
    R = np.asarray(returns, np.float64)
    oldv = np.asarray(old_values, np.float64)
    onehot = np.eye(A)[a]
    if kind == 'ppo':
        adv = np.asarray(advantages, np.float64)
        ratio = np.exp(logp - np.asarray(old_logp, np.float64))
        pg1 = -adv * ratio
        pg2 = -adv * np.clip(ratio, 1 - clip, 1 + clip)
        pg = np.maximum(pg1, pg2)
        r_in = (ratio >= 1 - clip) & (ratio <= 1 + clip)
        dlogp = np.where((pg1 >= pg2) | r_in, -adv * ratio, 0.0) / n
        dvo = v - oldv
        vclip = oldv + np.clip(dvo, -clip, clip)
        vl1, vl2 = (v - R) ** 2, (vclip - R) ** 2
        vl = np.maximum(vl1, vl2)
        value_loss = 0.5 * vl.mean()
        v_in = (dvo >= -clip) & (dvo <= clip)
        dv = v_coef * 0.5 * np.where(vl1 >= vl2, 2 * (v - R),
                                     np.where(v_in, 2 * (vclip - R), 0.0)) / n
    else:
        adv = R - oldv
        pg = -adv * logp
        dlogp = -adv / n
        vl = (v - R) ** 2
        value_loss = vl.mean()
        dv = v_coef * 2 * (v - R) / n
    loss = pg.mean() - ent_coef * H_.mean() + v_coef * value_loss
    dz3 = dlogp[:, None] * (onehot - p) + (ent_coef / n) * p * (lsm + H_[:, None])
    gW3, gb3 = h2.T @ dz3, dz3.sum(0)
    gW4, gb4 = h2.T @ dv[:, None], np.array([dv.sum()])
    dh2 = dz3 @ W3.T + dv[:, None] @ W4.T
    da2 = dh2 * (1 - h2 ** 2)
    gW2, gb2 = h1.T @ da2, da2.sum(0)
    dh1 = da2 @ W2.T
    da1 = dh1 * (1 - h1 ** 2)
    gW1, gb1 = x.T @ da1, da1.sum(0)
    grad = pack([gW1, gb1, gW2, gb2, gW3, gb3, gW4, gb4])
    terms = dict(loss=loss, pg_loss=pg.mean(), value_loss=value_loss, entropy=H_.mean(),
                 pg_sum=pg.sum(), vl_sum=vl.sum(), ent_sum=H_.sum())
    return terms, grad


def clip_by_global_norm_f64(g, clip):
    gn = np.sqrt((np.asarray(g, np.float64) ** 2).sum())
    return g * clip * min(1.0 / gn, 1.0 / clip), gn


def keras_adam_f64(theta, m, v, g, t, lr, b1, b2, eps):
    """training_ops ApplyAdam as driven by Keras OptimizerV2 Adam."""
    alpha = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = m + (g - m) * (1 - b1)
    v = v + (g * g - v) * (1 - b2)
    return theta - m * alpha / (np.sqrt(v) + eps), m, v
