"""Tensor-level wrappers over libxagents_hip.so (one function per C entry point).

Shapes follow the C ABI (include/xagents_hip.h): env-major [n_envs, n_steps, ...].
Every function runs asynchronously on torch's current stream and raises on error.
"""
import ctypes

import numpy as np
import torch

from xagents_amd import _lib
from xagents_amd._lib import (XA_LOSS_A2C, XA_LOSS_PPO, XaAcGradArgs, XaAdam, XaAdamTail,
                              XaMinibatchArgs, XaPpoUpdateArgs, XaRolloutArgs, XaShuffle, call,
                              ptr, stream)


def _f32(x):
    return ctypes.c_float(float(np.float32(x)))


def gamma_lam_f32(gamma, lam):
    """The reference forms gamma*lam as a Python (f64) product before the f32 multiply
    (xagents/ppo/agent.py:92)."""
    return float(np.float32(float(gamma) * float(lam)))


# (obs_dim, n_actions) instantiations of the fused MLP kernels (mlp_rollout.hip,
# ac_update.hip, ppo_update.hip)
FUSED_MLP_SHAPES = frozenset({(4, 2), (6, 3), (8, 4), (2, 3)})


def mlp_param_count(obs_dim, n_actions):
    return _lib.load().xa_mlp_param_count(obs_dim, n_actions)


def gae(rewards, values, dones, next_values, gamma, lam, out=None):
    """GAE returns (PPO.calculate_returns, xagents/ppo/agent.py:48-94).

    rewards/values [N,T], dones [N,T+1], next_values [N] -> returns [N,T] f32.
    """
    n, t = rewards.shape
    out = torch.empty_like(rewards) if out is None else out
    call('xa_gae', ptr(rewards), ptr(values), ptr(dones), ptr(next_values), ptr(out), n, t,
         _f32(gamma), _f32(gamma_lam_f32(gamma, lam)), stream())
    return out


def nstep_returns(rewards, dones, next_values, gamma, out=None):
    """n-step returns (A2C.calculate_returns, xagents/a2c/agent.py:141-171)."""
    n, t = rewards.shape
    out = torch.empty_like(rewards) if out is None else out
    call('xa_nstep_returns', ptr(rewards), ptr(dones), ptr(next_values), ptr(out), n, t,
         _f32(gamma), stream())
    return out


def mlp_forward(theta, obs, n_actions, actions=None, uniforms=None, want_logits=False):
    """Actor-critic forward (A2C.get_model_outputs, xagents/a2c/agent.py:65-94).

    Returns (actions, log_probs, values, entropies, logits-or-None).
    """
    b, obs_dim = obs.shape
    dev = obs.device
    act_out = None if actions is not None else torch.empty(b, dtype=torch.int32, device=dev)
    if actions is not None and actions.dtype != torch.int32:
        actions = actions.to(torch.int32)
    if actions is None and uniforms is None:
        raise ValueError('mlp_forward: sampling needs `uniforms`')
    logp = torch.empty(b, dtype=torch.float32, device=dev)
    value = torch.empty(b, dtype=torch.float32, device=dev)
    ent = torch.empty(b, dtype=torch.float32, device=dev)
    logits = torch.empty(b, n_actions, dtype=torch.float32, device=dev) if want_logits else None
    call('xa_mlp_forward', ptr(theta), ptr(obs.contiguous()), b, obs_dim, n_actions, ptr(actions),
         ptr(uniforms), ptr(act_out), ptr(logp), ptr(value), ptr(ent), ptr(logits), stream())
    return (actions if actions is not None else act_out), logp, value, ent, logits


def rollout(args: XaRolloutArgs):
    call('xa_mlp_rollout', ctypes.byref(args), stream())


def counter_bump(counter):
    call('xa_counter_bump', ptr(counter), stream())


def minibatches(args: XaMinibatchArgs):
    """Shuffle + gather + per-chunk advantage sums for a whole PPO train step."""
    call('xa_ppo_minibatches', ctypes.byref(args), stream())


def adv_stats(returns, values, batch, mb_size, epochs, shuffle: XaShuffle, stats):
    """Advantage sums only (no gather)."""
    a = XaMinibatchArgs()
    a.batch, a.mb_size, a.epochs, a.obs_dim = batch, mb_size, epochs, 0
    a.shuffle = shuffle
    a.returns, a.values, a.stats = ptr(returns), ptr(values), ptr(stats)
    minibatches(a)


def ac_grad_blocks(mb_size):
    import os
    cap = int(os.environ.get('XA_AC_BLOCKS', '0'))  # experiment knob: fewer, longer blocks
    nb = _lib.load().xa_ac_grad_blocks(mb_size)
    return min(nb, cap) if cap > 0 else nb


def ac_grad(args: XaAcGradArgs):
    call('xa_ac_grad', ctypes.byref(args), stream())


def ppo_update_blocks(obs_dim, n_actions, mb_size):
    """Workgroups of the persistent PPO update: one per 32-sample tile of a minibatch, at most
    as many as can be resident at once (0 if the device cannot be queried)."""
    return _lib.load().xa_ppo_update_blocks(obs_dim, n_actions, mb_size)


def ppo_update_workspace_bytes(obs_dim, n_actions, batch, mb_size, epochs, n_blocks):
    return _lib.load().xa_ppo_update_workspace_bytes(obs_dim, n_actions, batch, mb_size, epochs,
                                                     n_blocks)


def ppo_update(args: XaPpoUpdateArgs):
    """Every optimizer step of a PPO train step in one persistent launch
    (xagents/ppo/agent.py:96-191)."""
    call('xa_ppo_update', ctypes.byref(args), stream())


def adv_stats_size(batch, mb_size, epochs):
    return _lib.load().xa_ppo_adv_stats_size(batch, mb_size, epochs)


def grad_reduce(partials, grad, adam_step=None):
    nb, p = partials.shape
    call('xa_grad_reduce', ptr(partials), nb, p, ptr(grad), ptr(adam_step), stream())


def grad_reduce_adam(partials, grad, tail):
    """grad_reduce whose last block applies clip + Keras Adam (`tail`, an XaAdamTail)."""
    nb, p = partials.shape
    call('xa_grad_reduce_adam', ptr(partials), nb, p, ptr(grad), ctypes.byref(tail), stream())


def adam_tail(theta, m, v, adam_step, arrivals, lr, beta1, beta2, eps, clip_norm=None,
              grad_scale=1.0, bump=True, gnorm_out=None):
    """XaAdamTail for an in-place optimizer step on (theta, m, v); `arrivals` is a zeroed
    int32 device tensor the tail's kernels use to elect their last block."""
    t = XaAdamTail()  # launch arguments only: pointers are taken, nothing runs here
    t.theta, t.m, t.v = theta.data_ptr(), m.data_ptr(), v.data_ptr()
    t.adam_step, t.bump, t.arrivals = adam_step.data_ptr(), int(bool(bump)), arrivals.data_ptr()
    t.gnorm_out = None if gnorm_out is None else gnorm_out.data_ptr()
    t.adam = adam_struct(lr, beta1, beta2, eps, clip_norm=clip_norm, grad_scale=grad_scale)
    return t


def adam_struct(lr, beta1, beta2, eps, clip_norm=None, grad_scale=1.0):
    a = XaAdam()
    a.lr, a.beta1, a.beta2, a.eps = lr, beta1, beta2, eps
    a.clip_norm = clip_norm if clip_norm is not None else 0.0
    a.grad_scale = grad_scale
    return a


def clip_adam(theta, m, v, grad, adam_step, lr, beta1, beta2, eps, clip_norm=None,
              grad_scale=1.0, workspace=None, gnorm_out=None, out=None):
    """tf.clip_by_global_norm + Keras Adam (xagents/ppo/agent.py:135-137).
    `out` = (theta_out, m_out, v_out) for an out-of-place step (default in place)."""
    to, mo, vo = out if out is not None else (None, None, None)
    call('xa_clip_adam', ptr(theta), ptr(m), ptr(v), ptr(grad), theta.numel(), _f32(grad_scale),
         _f32(clip_norm if clip_norm is not None else 0.0), _f32(lr), _f32(beta1), _f32(beta2),
         _f32(eps), ptr(adam_step), ptr(workspace), ptr(gnorm_out), ptr(to), ptr(mo), ptr(vo),
         stream())


__all__ = [
    'XA_LOSS_A2C', 'XA_LOSS_PPO', 'XaAcGradArgs', 'XaRolloutArgs', 'XaShuffle', 'gae',
    'nstep_returns', 'mlp_forward', 'rollout', 'counter_bump', 'adv_stats', 'ac_grad',
    'ac_grad_blocks', 'ppo_update', 'ppo_update_blocks', 'ppo_update_workspace_bytes', 'grad_reduce', 'grad_reduce_adam', 'adam_tail', 'clip_adam', 'mlp_param_count', 'gamma_lam_f32',
]
