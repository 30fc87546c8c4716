"""ctypes binding of libxagents_hip.so (C ABI declared in include/xagents_hip.h).

There is no CPU fallback: if the HIP library is missing or fails to load, every
device op raises. Torch tensors are passed as raw device pointers plus sizes; the
stream is torch's current HIP stream so the calls compose with torch ops and can
be captured into a hipGraph (torch.cuda.CUDAGraph).
"""
import ctypes
from ctypes import (POINTER, Structure, c_double, c_float, c_int, c_int64, c_uint64,
                    c_void_p)
from pathlib import Path

import torch

LIB_PATH = Path(__file__).resolve().parent / 'libxagents_hip.so'

XA_ENV_REPLAY = 0
XA_ENV_CARTPOLE = 1
XA_RETURNS_NONE = 0
XA_RETURNS_GAE = 1
XA_RETURNS_NSTEP = 2
XA_LOSS_PPO = 0
XA_LOSS_A2C = 1
XA_DIST_CATEGORICAL = 0
XA_DIST_DIAG_GAUSSIAN = 1
MLP_HIDDEN = 64
XA_PPO_PLACE_AUTO = 0
XA_PPO_PLACE_SPREAD = 1
XA_PPO_PLACE_LOCAL = 2
XA_PPO_STATS_SLOTS = 16  # host slots of the persistent update's in-launch statistics


class XaRolloutArgs(Structure):
    _fields_ = [
        ('n_envs', c_int),
        ('n_steps', c_int),
        ('obs_dim', c_int),
        ('n_actions', c_int),
        ('theta', c_void_p),
        ('env_kind', c_int),
        ('env_state', c_void_p),
        ('env_state64', c_void_p),
        ('env_done', c_void_p),
        ('env_cursor', c_void_p),
        ('ep_return', c_void_p),
        ('rep_obs', c_void_p),
        ('rep_state', c_void_p),
        ('rep_rew', c_void_p),
        ('rep_done', c_void_p),
        ('t_rec', c_int),
        ('max_episode_steps', c_int),
        ('uniforms', c_void_p),
        ('seed', c_uint64),
        ('rng_counter', c_void_p),
        ('obs_out', c_void_p),
        ('act_out', c_void_p),
        ('logp_out', c_void_p),
        ('val_out', c_void_p),
        ('ent_out', c_void_p),
        ('rew_out', c_void_p),
        ('done_out', c_void_p),
        ('epret_out', c_void_p),
        ('next_val', c_void_p),
        ('ret_out', c_void_p),
        ('return_kind', c_int),
        ('gamma', c_float),
        ('gamma_lam', c_float),
    ]


class XaShuffle(Structure):
    _fields_ = [('perm', c_void_p), ('seed', c_uint64), ('rng_counter', c_void_p)]


class XaMinibatchArgs(Structure):
    _fields_ = [
        ('batch', c_int),
        ('mb_size', c_int),
        ('epochs', c_int),
        ('obs_dim', c_int),
        ('shuffle', XaShuffle),
        ('returns', c_void_p),
        ('values', c_void_p),
        ('obs', c_void_p),
        ('actions', c_void_p),
        ('old_logp', c_void_p),
        ('stats', c_void_p),
        ('mb_obs', c_void_p),
        ('mb_actions', c_void_p),
        ('mb_old_logp', c_void_p),
        ('mb_values', c_void_p),
        ('mb_returns', c_void_p),
    ]


class XaAdam(Structure):
    _fields_ = [('lr', c_float), ('beta1', c_float), ('beta2', c_float), ('eps', c_float),
                ('clip_norm', c_float), ('grad_scale', c_float)]


class XaAcGradArgs(Structure):
    _fields_ = [
        ('obs_dim', c_int),
        ('n_actions', c_int),
        ('loss_kind', c_int),
        ('theta', c_void_p),
        ('batch', c_int),
        ('mb_size', c_int),
        ('epoch', c_int),
        ('mb_index', c_int),
        ('shuffle', XaShuffle),
        ('gathered', c_int),
        ('obs', c_void_p),
        ('actions', c_void_p),
        ('old_logp', c_void_p),
        ('old_values', c_void_p),
        ('returns', c_void_p),
        ('adv_stats', c_void_p),
        ('adv_count', c_double),
        ('adv_in', c_void_p),
        ('clip_norm', c_float),
        ('entropy_coef', c_float),
        ('value_coef', c_float),
        ('adv_eps', c_float),
        ('loss_scale', c_float),
        ('n_blocks', c_int),
        ('partials', c_void_p),
        ('loss_partials', c_void_p),
        ('pend_grad', c_void_p),
        ('pend_m', c_void_p),
        ('pend_v', c_void_p),
        ('theta_out', c_void_p),
        ('m_out', c_void_p),
        ('v_out', c_void_p),
        ('adam_step', c_void_p),
        ('adam', XaAdam),
    ]


class XaPpoUpdateArgs(Structure):
    _fields_ = [
        ('obs_dim', c_int), ('n_actions', c_int),
        ('batch', c_int), ('mb_size', c_int), ('epochs', c_int),
        ('shuffle', XaShuffle),
        ('obs', c_void_p), ('actions', c_void_p), ('old_logp', c_void_p),
        ('old_values', c_void_p), ('returns', c_void_p),
        ('clip_norm', c_float), ('entropy_coef', c_float), ('value_coef', c_float),
        ('adv_eps', c_float),
        ('theta', c_void_p), ('adam_m', c_void_p), ('adam_v', c_void_p), ('adam_step', c_void_p),
        ('adam', XaAdam),
        ('workspace', c_void_p), ('workspace_bytes', ctypes.c_size_t),
        ('loss_out', c_void_p),
        ('grad_out', c_void_p),
        ('status', c_void_p),
        ('n_blocks', c_int),
        ('bump_counter', c_int),
        ('dp_world', c_int), ('dp_rank', c_int),
        ('dp_blocks', c_void_p * 16),
        ('placement', c_int),
        ('theta_trace', c_void_p), ('grad_trace', c_void_p),
        ('stats_src', c_void_p), ('stats_dst', c_void_p * XA_PPO_STATS_SLOTS),
        ('stats_words', c_int),
    ]


class XaAdamTail(Structure):
    _fields_ = [
        ('theta', c_void_p), ('m', c_void_p), ('v', c_void_p),
        ('adam_step', c_void_p),
        ('bump', c_int),
        ('arrivals', c_void_p),
        ('gnorm_out', c_void_p),
        ('adam', XaAdam),
    ]


XA_ADAM_TAIL_MAX_PARAMS = 65536


class XaGemmArgs(Structure):
    _fields_ = [
        ('M', c_int), ('N', c_int), ('K', c_int),
        ('a', c_void_p),
        ('a_u8', c_int),
        ('a_pm', c_int64), ('a_rm', c_int64), ('a_sm', c_int64),
        ('a_pk', c_int64), ('a_rk', c_int64), ('a_sk', c_int64),
        ('b', c_void_p),
        ('b_ks', c_int64), ('b_ns', c_int64),
        ('c', c_void_p),
        ('ldc', c_int64),
        ('splits', c_int),
        ('partials', c_void_p),
        ('bias', c_void_p),
        ('act', c_int),
        ('gate', c_void_p),
        ('ld_gate', c_int64),
        ('beta', c_int),
        ('force_small', c_int),
        ('a_ones_row', c_int),
    ]


class XaAdamApply(Structure):
    _fields_ = [
        ('theta', c_void_p), ('m', c_void_p), ('v', c_void_p), ('step', c_void_p),
        ('lr', c_float), ('beta1', c_float), ('beta2', c_float), ('eps', c_float),
        ('grad_scale', c_float),
    ]


class XaConvStackArgs(Structure):
    _fields_ = [
        ('x', c_void_p), ('x_u8', c_int), ('rows', c_int),
        ('w1', c_void_p), ('b1', c_void_p), ('w2', c_void_p), ('b2', c_void_p),
        ('w3', c_void_p), ('b3', c_void_p),
        ('h1', c_void_p), ('h2', c_void_p), ('h3', c_void_p),
    ]


class XaConvStackBwdArgs(Structure):
    _fields_ = [
        ('x', c_void_p), ('x_u8', c_int), ('rows', c_int),
        ('w2', c_void_p), ('w3', c_void_p),
        ('h1', c_void_p), ('h2', c_void_p), ('dz3', c_void_p),
        ('ws', c_void_p), ('ws_floats', ctypes.c_size_t), ('grad', c_void_p), ('accumulate', c_int),
        ('adam_on', c_int), ('write_grad', c_int), ('adam', XaAdamApply), ('rest', XaAdamApply),
        ('rest_grad', c_void_p), ('n_rest', c_int),
    ]


class XaDqnHeadArgs(Structure):
    _fields_ = [
        ('mode', c_int), ('actions', c_void_p), ('q', c_void_p), ('q_next_online', c_void_p),
        ('act', c_void_p), ('rewards', c_void_p), ('dones', c_void_p),
        ('gamma', c_float), ('huber', c_float), ('dq', c_void_p), ('loss', c_void_p),
        ('adam_step', c_void_p),
    ]


class XaAtariStepArgs(Structure):
    _fields_ = [
        ('n_envs', c_int), ('t_raw', c_int), ('height', c_int), ('width', c_int),
        ('out_h', c_int), ('out_w', c_int),
        ('frames', c_void_p), ('raw_rew', c_void_p), ('raw_done', c_void_p),
        ('raw_cursor', c_void_p),
        ('skips', c_int), ('max_frame', c_int), ('reset_only', c_int),
        ('xofs', c_void_p), ('alpha', c_void_p), ('yofs', c_void_p), ('beta', c_void_p),
        ('out_step', c_void_p), ('out_post', c_void_p), ('out_rew', c_void_p),
        ('out_done', c_void_p),
    ]


class XaWalkerStepArgs(Structure):
    _fields_ = [
        ('n_envs', c_int), ('state', c_void_p), ('episode', c_void_p), ('actions', c_void_p),
        ('act_ld', c_int64), ('seed', c_uint64), ('reset_only', c_int),
        ('out_obs', c_void_p), ('out_post', c_void_p), ('out_rew', c_void_p),
        ('out_done', c_void_p),
    ]


class XaHostCopyArgs(Structure):
    _fields_ = [
        ('n_segments', c_int), ('src', c_void_p * 4), ('dst', c_void_p * 4),
        ('bytes', c_int64 * 4),
    ]


class XaTrpoHeadArgs(Structure):
    _fields_ = [
        ('n', c_int), ('n_actions', c_int),
        ('logits_new', c_void_p), ('logits_old', c_void_p), ('ld_logits', c_int64),
        ('actions', c_void_p), ('advantages', c_void_p),
        ('entropy_coef', c_float), ('inv_n', c_float),
        ('dlogits', c_void_p), ('ld_dlogits', c_int64),
        ('partials', c_void_p),
    ]


XA_GATHER_MAX_FIELDS = 8


class XaGatherField(Structure):
    _fields_ = [('ring', c_void_p), ('dst', c_void_p), ('item_bytes', c_int64)]


class XaGatherArgs(Structure):
    _fields_ = [('field', XaGatherField * XA_GATHER_MAX_FIELDS), ('n_fields', c_int),
                ('n_items', c_int), ('slots', c_void_p)]


class XaReplayStepArgs(Structure):
    _fields_ = [
        ('n_envs', c_int), ('t_rec', c_int),
        ('obs_bytes', c_int64),
        ('rep_obs', c_void_p), ('rep_state', c_void_p), ('rep_rew', c_void_p),
        ('rep_done', c_void_p),
        ('state', c_void_p), ('cursor', c_void_p), ('ep_return', c_void_p), ('done', c_void_p),
        ('actions', c_void_p), ('act_bytes', c_int64),
        ('capacity', c_int64), ('ring_kind', c_int), ('ring_count', c_void_p),
        ('ring_states', c_void_p), ('ring_new_states', c_void_p), ('ring_actions', c_void_p),
        ('ring_rewards', c_void_p), ('ring_dones', c_void_p),
        ('out_states', c_void_p), ('out_new_states', c_void_p), ('out_rewards', c_void_p),
        ('out_dones', c_void_p), ('done_epret', c_void_p), ('out_ld', c_int64),
    ]


class XaHeadGradArgs(Structure):
    _fields_ = [
        ('n', c_int), ('n_actions', c_int), ('loss_kind', c_int),
        ('logits', c_void_p), ('ld_logits', c_int64),
        ('values', c_void_p), ('ld_values', c_int64),
        ('actions', c_void_p), ('old_logp', c_void_p), ('old_values', c_void_p),
        ('returns', c_void_p),
        ('clip_norm', c_float), ('entropy_coef', c_float), ('value_coef', c_float),
        ('adv_eps', c_float),
        ('dlogits', c_void_p), ('dvalues', c_void_p), ('loss', c_void_p),
        ('stats_mode', c_int), ('adv_stats', c_void_p),
        ('dist_kind', c_int), ('actions_f', c_void_p), ('ld_actions', c_int64),
    ]


class XaAcerArgs(Structure):
    _fields_ = [
        ('n_envs', c_int), ('n_steps', c_int), ('n_actions', c_int), ('n_total', c_int),
        ('logits', c_void_p), ('ld_logits', c_int64),
        ('q', c_void_p), ('ld_q', c_int64),
        ('avg_logits', c_void_p), ('ld_avg', c_int64),
        ('mu_logits', c_void_p), ('actions', c_void_p), ('rewards', c_void_p),
        ('dones', c_void_p),
        ('gamma', c_float), ('epsilon', c_float), ('importance_c', c_float), ('delta', c_float),
        ('entropy_coef', c_float), ('value_coef', c_float),
        ('trust_region', c_int),
        ('dlogits', c_void_p), ('ld_dlogits', c_int64),
        ('dq', c_void_p), ('ld_dq', c_int64),
        ('returns', c_void_p), ('env_loss', c_void_p),
    ]


XA_PEER_MAX = 16
XA_DTYPE_F32 = 0
XA_DTYPE_F64 = 1


class XaPeerAllReduceArgs(Structure):
    _fields_ = [
        ('blocks', c_void_p * XA_PEER_MAX),
        ('rank', c_int), ('world', c_int),
        ('dtype', c_int),
        ('count', c_int64),
        ('slot_bytes', ctypes.c_size_t),
        ('src', c_void_p), ('dst', c_void_p),
        ('state', c_void_p),
        ('timeout_ticks', c_uint64),
        ('has_tail', c_int),
        ('tail', XaAdamTail),
    ]


class XaTdNet(Structure):
    _fields_ = [('theta', c_void_p), ('m', c_void_p), ('v', c_void_p), ('step', c_void_p),
                ('lr', c_float), ('beta1', c_float), ('beta2', c_float), ('eps', c_float)]


class XaTd3UpdateArgs(Structure):
    _fields_ = [
        ('batch', c_int), ('obs_dim', c_int), ('act_dim', c_int), ('h1', c_int), ('h2', c_int),
        ('twin', c_int), ('smooth', c_int), ('actor_update', c_int),
        ('gamma', c_float), ('tau', c_float), ('noise_sigma', c_float), ('noise_clip', c_float),
        ('huber_delta', c_float),
        ('ring_states', c_void_p), ('ring_new_states', c_void_p), ('ring_actions', c_void_p),
        ('ring_rewards', c_void_p), ('ring_dones', c_void_p), ('slots', c_void_p),
        ('rng_counter', c_void_p), ('seed', c_uint64),
        ('actor', XaTdNet), ('critic1', XaTdNet), ('critic2', XaTdNet),
        ('target_actor', XaTdNet), ('target_critic1', XaTdNet), ('target_critic2', XaTdNet),
        ('out_s', c_void_p), ('out_a', c_void_p), ('out_r', c_void_p), ('out_d', c_void_p),
        ('out_s2', c_void_p), ('noise_out', c_void_p), ('dv1', c_void_p), ('dv2', c_void_p),
        ('loss_out', c_void_p), ('g_actor', c_void_p), ('g_critic1', c_void_p),
        ('g_critic2', c_void_p),
        ('workspace', c_void_p), ('workspace_bytes', ctypes.c_size_t),
        ('n_blocks', c_int), ('status', c_void_p),
        ('stage', c_int), ('critic_grad_scale', c_float), ('actor_grad_scale', c_float),
    ]


class XaTd3ActArgs(Structure):
    _fields_ = [
        ('n', c_int), ('obs_dim', c_int), ('act_dim', c_int), ('h1', c_int), ('h2', c_int),
        ('states', c_void_p), ('theta', c_void_p),
        ('sigma', c_float), ('noise_clip', c_float), ('lo', c_float), ('hi', c_float),
        ('rng_counter', c_void_p), ('seed', c_uint64), ('bump', c_int),
        ('out', c_void_p), ('ld_out', c_int), ('noise_out', c_void_p),
        ('workspace', c_void_p), ('workspace_bytes', ctypes.c_size_t),
        ('n_blocks', c_int), ('status', c_void_p),
    ]


XA_RING_DEQUE = 0
XA_RING_RB2 = 1
XA_ACT_NONE = 0
XA_ACT_RELU = 1
XA_ACT_TANH = 2

_SIGNATURES = {
    'xa_abi_version': (c_int, []),
    'xa_last_error': (ctypes.c_char_p, []),
    'xa_build_hash': (ctypes.c_char_p, []),
    'xa_mlp_param_count': (c_int, [c_int, c_int]),
    'xa_counter_bump': (c_int, [c_void_p, c_void_p]),
    'xa_gae': (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float,
         c_void_p],
    ),
    'xa_nstep_returns': (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    ),
    'xa_mlp_rollout': (c_int, [POINTER(XaRolloutArgs), c_void_p]),
    'xa_mlp_forward': (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    'xa_ppo_adv_stats_size': (c_int, [c_int, c_int, c_int]),
    'xa_ppo_minibatches': (c_int, [POINTER(XaMinibatchArgs), c_void_p]),
    'xa_ac_grad': (c_int, [POINTER(XaAcGradArgs), c_void_p]),
    'xa_ac_grad_blocks': (c_int, [c_int]),
    'xa_grad_reduce': (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    'xa_grad_reduce_adam': (c_int, [c_void_p, c_int, c_int, c_void_p, POINTER(XaAdamTail),
                                    c_void_p]),
    'xa_clip_adam': (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_float, c_float, c_float,
         c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p],
    ),
    'xa_ppo_update_blocks': (c_int, [c_int, c_int, c_int]),
    'xa_ppo_update_workspace_bytes': (ctypes.c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    'xa_ppo_update': (c_int, [POINTER(XaPpoUpdateArgs), c_void_p]),
    'xa_gemm': (c_int, [POINTER(XaGemmArgs), c_void_p]),
    'xa_gemm_adam': (c_int, [POINTER(XaGemmArgs), POINTER(XaAdamApply), c_void_p]),
    'xa_conv_stack_fwd': (c_int, [POINTER(XaConvStackArgs), c_void_p]),
    'xa_dqn_head': (c_int, [POINTER(XaGemmArgs), POINTER(XaDqnHeadArgs), c_void_p]),
    'xa_gemm_head': (c_int, [POINTER(XaGemmArgs), POINTER(XaGemmArgs), POINTER(XaDqnHeadArgs),
                             c_void_p]),
    'xa_gemm_head_ok': (c_int, [POINTER(XaGemmArgs), POINTER(XaGemmArgs)]),
    'xa_head_bwd': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                            c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    'xa_conv_stack_bwd': (c_int, [POINTER(XaConvStackBwdArgs), c_void_p]),
    'xa_conv_stack_bwd_workspace_floats': (ctypes.c_size_t, [c_int]),
    'xa_gemm_splits': (c_int, [c_int, c_int, c_int]),
    'xa_gemm_shape': (c_int, [c_int, c_int, c_int, c_int]),
    'xa_gemm_workspace_floats': (ctypes.c_size_t, [c_int, c_int, c_int, c_int]),
    'xa_conv1d_input_grad': (
        c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    ),
    'xa_conv1d_dgrad': (
        c_int,
        [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
         c_void_p, c_void_p],
    ),
    'xa_conv1d_wgrad_workspace_floats': (ctypes.c_size_t, [c_int, c_int, c_int]),
    'xa_conv1d_wgrad': (
        c_int,
        [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
         c_void_p, c_int, c_void_p, ctypes.c_size_t, c_void_p],
    ),
    'xa_trpo_head_blocks': (c_int, [c_int]),
    'xa_trpo_head': (c_int, [POINTER(XaTrpoHeadArgs), c_void_p, c_void_p]),
    'xa_categorical_fisher': (
        c_int,
        [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_float, c_void_p, c_int64,
         c_void_p],
    ),
    'xa_vec_dot': (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    'xa_axpby': (c_int, [c_float, c_void_p, c_float, c_void_p, c_void_p, c_int64, c_void_p]),
    'xa_normalized_advantages': (c_int, [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p]),
    'xa_dqn_act': (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    'xa_dqn_td_grad': (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
         c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    'xa_ring_scatter': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    'xa_ring_gather': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    'xa_ring_gather_fields': (c_int, [c_void_p, c_void_p]),
    'xa_polyak': (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p]),
    'xa_adam_step_bump': (c_int, [c_void_p, c_void_p]),
    'xa_replay_env_step': (c_int, [POINTER(XaReplayStepArgs), c_void_p]),
    'xa_atari_step': (c_int, [POINTER(XaAtariStepArgs), c_void_p]),
    'xa_ppo_update_dp_block_bytes': (ctypes.c_size_t, [c_int] * 7),
    'xa_walker_step': (c_int, [POINTER(XaWalkerStepArgs), c_void_p]),
    'xa_copy_to_host': (c_int, [POINTER(XaHostCopyArgs), c_void_p]),
    'xa_host_device_pointer': (c_int, [c_void_p, POINTER(c_void_p)]),
    'xa_mse_grad': (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    'xa_copy_block': (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p]),
    'xa_categorical': (
        c_int,
        [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p,
         c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    ),
    'xa_ac_head_grad': (c_int, [POINTER(XaHeadGradArgs), c_void_p]),
    'xa_td3_update_workspace_bytes': (ctypes.c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    'xa_td3_update': (c_int, [POINTER(XaTd3UpdateArgs), c_void_p]),
    'xa_td3_act_workspace_bytes': (ctypes.c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    'xa_td3_act': (c_int, [POINTER(XaTd3ActArgs), c_void_p]),
    'xa_minibatch_adv_sums': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                      c_void_p, c_void_p]),
    'xa_diag_gaussian': (
        c_int,
        [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_int64,
         c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    ),
    'xa_acer_grad': (c_int, [POINTER(XaAcerArgs), c_void_p]),
    'xa_ema': (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p]),
    'xa_noisy_actions': (
        c_int,
        [c_void_p, c_int64, c_int, c_int, c_float, c_float, c_float, c_float, c_void_p,
         c_uint64, c_void_p, c_int64, c_void_p, c_void_p],
    ),
    'xa_critic_td_grad': (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_float,
         c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    'xa_activation_grad': (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    'xa_peer_block_bytes': (ctypes.c_size_t, [ctypes.c_size_t, c_int]),
    'xa_peer_state_words': (c_int, [ctypes.c_size_t]),
    'xa_peer_block_alloc': (c_int, [ctypes.c_size_t, POINTER(c_void_p)]),
    'xa_peer_block_free': (c_int, [c_void_p]),
    'xa_peer_ipc_handle': (c_int, [c_void_p, c_void_p]),
    'xa_peer_ipc_open': (c_int, [c_void_p, POINTER(c_void_p)]),
    'xa_peer_ipc_close': (c_int, [c_void_p]),
    'xa_peer_allreduce': (c_int, [POINTER(XaPeerAllReduceArgs), c_void_p]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


class HipLibraryError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and return the ctypes handle. Raises if the .so is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise HipLibraryError(
            f'{p} not found: build it with `python -m xagents_amd._build` '
            f'(or __graft_entry__.build()). There is no CPU fallback.'
        )
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        # the product library must be built from the sources in this tree (diagnostic
        # builds loaded by path are exempt)
        from xagents_amd._build import source_hash
        built, want = lib.xa_build_hash().decode(), source_hash()
        if built != want:
            raise HipLibraryError(
                f'{p} is stale: built from sources {built}, this tree is {want}; rebuild with '
                f'`python -m xagents_amd._build` (or __graft_entry__.build())')
        _lib = lib
    return lib


def check(ret, name):
    if ret != 0:
        msg = load().xa_last_error().decode()
        raise HipLibraryError(f'{name} failed ({ret}): {msg}')


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise HipLibraryError('xagents_amd device ops need tensors on a HIP device')
    if not t.is_contiguous():
        raise HipLibraryError('xagents_amd device ops need contiguous tensors')
    return t.data_ptr()


if hasattr(torch._C, '_cuda_getCurrentRawStream') and hasattr(torch._C, '_cuda_getDevice'):
    _raw_stream, _cur_dev = torch._C._cuda_getCurrentRawStream, torch._C._cuda_getDevice

    def stream():
        """The current HIP stream of the current device (a capture stream inside hipGraph
        capture), as a raw handle: two C calls instead of torch.cuda.current_stream()'s
        Python wrappers (~3 us per launch on the C3 host path, tools/c3_host_profile.py)."""
        return _raw_stream(_cur_dev())
else:
    def stream():
        return torch.cuda.current_stream().cuda_stream


def call(name, *args):
    check(getattr(load(), name)(*args), name)
