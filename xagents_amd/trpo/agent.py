"""TRPO with the xagents class surface (xagents/trpo/agent.py:6-348) on device.

Actor and critic are separate .cfg models run by the layer executor (xagents_amd/layers.py).
One train step:
    rollout  T x [actor forward -> Categorical sample (xa_categorical), critic forward,
             env step (xa_replay_env_step)], V(get_states()), GAE (xa_gae)
    batch    env-major gather of the states (xa_ring_gather); advantages normalised over
             the batch (xa_normalized_advantages)
    gradient actor forward = old logits (actor == old actor after at_step_start),
             d surrogate_loss / d logits (xa_trpo_head), actor backward -> flat g
    CG       cg_iterations x Fisher-vector products on states[::fvp_n_steps]:
             J v (executor jvp) -> (diag(p) - p p^T) (xa_categorical_fisher) -> J^T
             (executor backward) + damping v; vector algebra xa_vec_dot / xa_axpby
    step     shs = 0.5 s.Fs, full_step = s / sqrt(shs / max_kl); backtracking line search
             on (surrogate gain, KL) with xa_trpo_head (host reads 3 floats per trial)
    critic   critic_iterations x PPO minibatches: MSE value loss, Keras Adam
Scalars that steer control flow (CG residual, line-search conditions) are read back to
the host exactly where the reference leaves the graph (tf.numpy_function / python
control flow). Minibatch permutations use numpy's global RNG (the reference's
tf.random.shuffle stream cannot be reproduced without TF).
"""
import ctypes

import numpy as np
import torch

from xagents_amd import kernels
from xagents_amd._lib import (XA_RETURNS_GAE, XaReplayStepArgs, XaTrpoHeadArgs, call, load,
                              stream)
from xagents_amd.base import OnPolicy
from xagents_amd.envs import Discrete
from xagents_amd.layers import LayerExecutor
from xagents_amd.ppo.agent import PPO


class TRPO(PPO):
    """Trust Region Policy Optimization https://arxiv.org/abs/1502.05477"""

    return_kind = XA_RETURNS_GAE

    def __init__(
        self,
        envs,
        actor_model,
        critic_model,
        max_kl=1e-3,
        cg_iterations=10,
        cg_residual_tolerance=1e-10,
        cg_damping=1e-3,
        actor_iterations=10,
        critic_iterations=3,
        fvp_n_steps=5,
        lam=0.95,
        ppo_epochs=4,
        mini_batches=4,
        advantage_epsilon=1e-8,
        clip_norm=0.1,
        entropy_coef=0.01,
        value_loss_coef=0.5,
        grad_norm=0.5,
        use_graph=True,
        **kwargs,
    ):
        # PPO / A2C attributes (ppo/agent.py:14-52, a2c/agent.py:14-45) without their
        # fused actor-critic setup: TRPO's actor and critic are separate models
        self.lam = lam
        self.ppo_epochs = ppo_epochs
        self.mini_batches = mini_batches
        self.advantage_epsilon = advantage_epsilon
        self.clip_norm = clip_norm
        n_envs = len(envs)
        self.batch_size = n_envs * kwargs.get('n_steps', 1)
        self.mini_batch_size = self.batch_size // self.mini_batches
        assert (
            self.mini_batch_size > 0
        ), f'Invalid batch size to mini-batch size ratio {self.batch_size}: {self.mini_batches}'
        OnPolicy.__init__(self, envs, actor_model, **kwargs)
        self.entropy_coef = entropy_coef
        self.value_loss_coef = value_loss_coef
        self.grad_norm = grad_norm
        self.use_graph = use_graph  # rollout replayed from a hipGraph after one eager pass
        self._rgraph = None
        self.executor_path = True
        if not isinstance(self.envs[0].action_space, Discrete):
            raise NotImplementedError('Only Categorical(logits) policies are supported')
        self.output_models.append(critic_model)
        self.actor = self.model
        self.critic = critic_model
        self.cg_iterations = cg_iterations
        self.cg_residual_tolerance = cg_residual_tolerance
        self.cg_damping = cg_damping
        self.max_kl = max_kl
        self.critic_iterations = critic_iterations
        self.actor_iterations = actor_iterations
        self.fvp_n_steps = fvp_n_steps
        self.distributed, self.world_size, self.rank = False, 1, 0
        self._setup_trpo()

    # ---- device state ----------------------------------------------------------
    def _setup_trpo(self):
        env = self.envs
        if not hasattr(env, 'fill_step_args'):
            raise NotImplementedError('TRPO runs on a transition-replay device env '
                                      "(create_envs(..., mode='transitions'))")
        if len(self.actor.outputs) != 1 or len(self.critic.outputs) != 1:
            raise NotImplementedError('TRPO needs a one-output actor and a one-output critic')
        N, T, B = self.n_envs, self.n_steps, self.batch_size
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        A = self.n_actions
        self.obs_buf = torch.zeros((T + 1, N) + env.obs_shape, dtype=env.state.dtype,
                                   device=dev)
        self.b_act = torch.zeros(N, T, dtype=torch.int32, device=dev)
        self.b_logp, self.b_val = torch.zeros(N, T, **f32), torch.zeros(N, T, **f32)
        self.b_ent, self.b_rew = torch.zeros(N, T, **f32), torch.zeros(N, T, **f32)
        self.b_done = torch.zeros(N, T + 1, **f32)
        self.b_dstep = torch.zeros(N, T, **f32)
        self.b_epret = torch.zeros(N, T, **f32)
        self.b_ret = torch.zeros(N, T, **f32)
        self.next_val = torch.zeros(N, **f32)
        self.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        seed = self.seed if self.seed is not None else int(np.random.SeedSequence().entropy % 2**63)
        self.rng_seed = (int(seed) * 1000003 + 17) % 2**64
        self.ex_actor_roll = LayerExecutor(self.actor, N)
        self.ex_critic_roll = LayerExecutor(self.critic, N)
        self._sa = XaReplayStepArgs()
        env.fill_step_args(self._sa)
        self._sa.ring_states = None
        # whole-batch executors (update) and the FVP subsample states[::fvp_n_steps]
        self.ex_actor = LayerExecutor(self.actor, B)
        self.fvp_idx = np.arange(0, B, self.fvp_n_steps)
        self.n_fvp = len(self.fvp_idx)
        self.ex_fvp = LayerExecutor(self.actor, self.n_fvp)
        mb = self.mini_batch_size
        self.ex_critic = LayerExecutor(self.critic, mb)
        self.batch_states = torch.zeros((B,) + env.obs_shape, dtype=env.state.dtype, device=dev)
        self.fvp_states = torch.zeros((self.n_fvp,) + env.obs_shape, dtype=env.state.dtype,
                                      device=dev)
        self._ident = torch.arange(B, dtype=torch.int64, device=dev)
        obs_slots = (np.arange(B) % T) * N + np.arange(B) // T  # env-major i -> frame t N + env
        self._batch_slots = torch.from_numpy(obs_slots.astype(np.int64)).to(dev)
        self._fvp_slots = torch.from_numpy(self.fvp_idx.astype(np.int64)).to(dev)
        self.adv = torch.zeros(B, **f32)
        self.old_logits = torch.zeros(B, A, **f32)
        self.fvp_logits = torch.zeros(self.n_fvp, A, **f32)
        self.dlogits = torch.zeros(B, A, **f32)
        self.fisher_u = torch.zeros(self.n_fvp, A, **f32)
        self.head_parts = torch.zeros(max(load().xa_trpo_head_blocks(B), 1), 3,
                                      dtype=torch.float64, device=dev)
        self.head_out = torch.zeros(3, **f32)
        self.dot_out = torch.zeros(1, dtype=torch.float64, device=dev)
        P = self.actor.n_params
        self.flat_grads = torch.zeros(P, **f32)
        self.cg = {k: torch.zeros(P, **f32) for k in ('x', 'r', 'p', 'z')}
        self.fvp_out = torch.zeros(P, **f32)
        self.w0 = torch.zeros(P, **f32)
        self.full_step = torch.zeros(P, **f32)
        # critic minibatch buffers
        self.critic_slots = None
        self.mb_states = torch.zeros((mb,) + env.obs_shape, dtype=env.state.dtype, device=dev)
        self.mb_ret = torch.zeros(mb, **f32)
        self.dvalue = torch.zeros(mb, 1, **f32)
        self.critic_grad = torch.zeros(self.critic.n_params, **f32)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        self.last_losses = None

    # ---- reference hooks -----------------------------------------------------------
    def at_step_start(self):
        """self.old_actor.set_weights(self.actor.get_weights()) (trpo/agent.py:225-233):
        the old logits are recomputed from the actor at the start of train_step, before the
        line search moves it, which is the same thing."""

    def get_batch(self):
        """Rollout of n_steps with the actor and the critic (A2C.get_batch,
        a2c/agent.py:96-139) + GAE; env-major flat [states, actions, returns, values,
        log_probs] (concat_step_batches order)."""
        self._rollout()
        B = self.batch_size
        return [self.batch_states, self.b_act.reshape(B).float(), self.b_ret.reshape(B),
                self.b_val.reshape(B), self.b_logp.reshape(B)]

    def _rollout(self):
        """The rollout launches (~11 per env step) are host-bound when launched one by one
        from Python; after one eager pass they are captured once and replayed."""
        if not self.use_graph:
            self._rollout_kernels()
        elif self._rgraph is not None:
            self._rgraph.replay()
        elif getattr(self, '_rollout_warm', False):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._rollout_kernels()
            self._rgraph = g
            g.replay()
        else:
            self._rollout_kernels()
            self._rollout_warm = True
        self.steps += self.n_envs * self.n_steps
        self._queue_episode_stats(self.b_done, self.b_epret)

    def _play_chunk(self):
        """play(): one eager rollout (actor samples); env 0's rewards and step dones."""
        self._sync_stats_copy()
        self._rollout_kernels()
        return self.b_rew[0].cpu().numpy(), self.b_done[0, 1:].cpu().numpy()

    def _rollout_kernels(self):
        N, T = self.n_envs, self.n_steps
        env, a = self.envs, self._sa
        self.obs_buf[0].copy_(env.state)
        call('xa_copy_block', env.done.data_ptr(), 1, self.b_done.data_ptr(), T + 1, N, 1,
             stream())
        ob = env.obs_bytes
        A = self.n_actions
        for t in range(T):
            logits = self.ex_actor_roll.forward(self.obs_buf[t])[0]
            call('xa_categorical', logits.data_ptr(), A, N, A, None, self.rng_counter.data_ptr(),
                 self.rng_seed, t, None, self.b_act.data_ptr() + 4 * t,
                 self.b_logp.data_ptr() + 4 * t, self.b_ent.data_ptr() + 4 * t, T, stream())
            value = self.ex_critic_roll.forward(self.obs_buf[t])[0]
            call('xa_copy_block', value.data_ptr(), 1, self.b_val.data_ptr() + 4 * t, T, N, 1,
                 stream())
            a.actions, a.act_bytes = self.b_act.data_ptr() + 4 * t, 4
            a.out_new_states = self.obs_buf.data_ptr() + (t + 1) * N * ob
            a.out_rewards = self.b_rew.data_ptr() + 4 * t
            a.out_dones = self.b_dstep.data_ptr() + 4 * t
            a.done_epret = self.b_epret.data_ptr() + 4 * t
            a.out_ld = T
            if hasattr(env, 'pre_step'):
                env.pre_step()
            call('xa_replay_env_step', ctypes.byref(a), stream())
        call('xa_copy_block', self.b_dstep.data_ptr(), T, self.b_done.data_ptr() + 4, T + 1, N,
             T, stream())
        value = self.ex_critic_roll.forward(env.state)[0]
        call('xa_copy_block', value.data_ptr(), 1, self.next_val.data_ptr(), 1, N, 1, stream())
        kernels.gae(self.b_rew, self.b_val, self.b_done, self.next_val, self.gamma, self.lam,
                    out=self.b_ret)
        kernels.counter_bump(self.rng_counter)
        # env-major batch of the states the reference concatenates (base.py:549-564)
        call('xa_ring_gather', self.obs_buf.data_ptr(), self.batch_states.data_ptr(),
             self._batch_slots.data_ptr(), self.batch_size, env.obs_bytes, stream())

    # ---- actor pieces ------------------------------------------------------------------
    def _head(self, logits_new, dlogits=None, out=None):
        h = XaTrpoHeadArgs()
        h.n, h.n_actions = self.batch_size, self.n_actions
        h.logits_new, h.logits_old = logits_new.data_ptr(), self.old_logits.data_ptr()
        h.ld_logits = self.n_actions
        h.actions, h.advantages = self.b_act.data_ptr(), self.adv.data_ptr()
        h.entropy_coef, h.inv_n = float(self.entropy_coef), 1.0 / self.batch_size
        h.dlogits = None if dlogits is None else dlogits.data_ptr()
        h.ld_dlogits = self.n_actions
        h.partials = self.head_parts.data_ptr()
        call('xa_trpo_head', ctypes.byref(h), None if out is None else out.data_ptr(), stream())

    def _dot(self, x, y):
        call('xa_vec_dot', x.data_ptr(), y.data_ptr(), x.numel(), self.dot_out.data_ptr(),
             stream())
        return np.float32(self.dot_out.item())

    def _axpby(self, a, x, b, y, out):
        call('xa_axpby', float(a), x.data_ptr(), float(b), y.data_ptr(), out.data_ptr(),
             out.numel(), stream())

    def calculate_fvp(self, flat_tangent, out=None):
        """Fisher-vector product on states[::fvp_n_steps] + cg_damping v
        (trpo/agent.py:121-148); needs _prepare_fvp() for the current actor."""
        out = self.fvp_out if out is None else out
        t = self.ex_fvp.jvp(flat_tangent)[0]
        call('xa_categorical_fisher', self.fvp_logits.data_ptr(), self.n_actions, t.data_ptr(),
             self.n_actions, self.n_fvp, self.n_actions, 1.0 / self.n_fvp,
             self.fisher_u.data_ptr(), self.n_actions, stream())
        self.ex_fvp.backward([self.fisher_u], out)
        self._axpby(1.0, out, self.cg_damping, flat_tangent, out)
        return out

    def _prepare_fvp(self):
        call('xa_ring_gather', self.batch_states.data_ptr(), self.fvp_states.data_ptr(),
             self._fvp_slots.data_ptr(), self.n_fvp, self.envs.obs_bytes, stream())
        lg = self.ex_fvp.forward(self.fvp_states)[0]
        self.fvp_logits.copy_(lg)

    def conjugate_gradients(self, flat_grads):
        """trpo/agent.py:150-177, scalars in f32 as TF computes them."""
        x, r, p = self.cg['x'], self.cg['r'], self.cg['p']
        p.copy_(flat_grads)
        r.copy_(flat_grads)
        x.zero_()
        r_dot_r = self._dot(r, r)
        iterations = 0
        while iterations < self.cg_iterations and r_dot_r > self.cg_residual_tolerance:
            z = self.calculate_fvp(p, self.cg['z'])
            v = np.float32(r_dot_r / self._dot(p, z))
            self._axpby(1.0, x, v, p, x)
            self._axpby(1.0, r, -v, z, r)
            new_r_dot_r = self._dot(r, r)
            mu = np.float32(new_r_dot_r / r_dot_r)
            self._axpby(1.0, r, mu, p, p)
            r_dot_r = new_r_dot_r
            iterations += 1
        return x

    def calculate_losses(self):
        """(surrogate_loss, mean KL) of the current actor against the old logits
        (trpo/agent.py:200-223)."""
        lg = self.ex_actor.forward(self.batch_states)[0]
        self._head(lg, out=self.head_out)
        loss, kl, _ = self.head_out.tolist()
        return np.float32(loss), np.float32(kl)

    def update_actor_weights(self, surrogate_loss):
        """Backtracking line search (trpo/agent.py:235-278)."""
        theta = self.actor.theta
        self.w0.copy_(theta)
        learning_rate = 1.0
        for _ in range(self.actor_iterations):
            self._axpby(1.0, self.w0, learning_rate, self.full_step, theta)
            new_surrogate_loss, new_kl_divergence = self.calculate_losses()
            improvement = new_surrogate_loss - surrogate_loss
            ok_conditions = [
                np.isfinite([new_surrogate_loss, new_kl_divergence]).all(),
                new_kl_divergence <= self.max_kl * 1.5,
                improvement > 0,
            ]
            if all(ok_conditions):
                break
            learning_rate *= 0.5
        else:
            theta.copy_(self.w0)

    def update_critic_weights(self):
        """critic_iterations x PPO minibatches of mean((V - R)^2), Keras Adam
        (trpo/agent.py:280-299). Every epoch's permutation (numpy's global RNG, one per
        epoch as get_mini_batches draws them) is uploaded in one copy; the minibatch
        launches are captured once and replayed like the rollout."""
        B = self.batch_size
        n_perm = self.critic_iterations * self.ppo_epochs
        perms = np.stack([np.random.permutation(B) for _ in range(n_perm)])
        if getattr(self, 'critic_slots', None) is None or self.critic_slots.shape[0] != n_perm:
            self.critic_slots = torch.zeros(n_perm, B, dtype=torch.int64, device=self.device)
            self._cgraph = None
        self.critic_slots.copy_(torch.from_numpy(perms), non_blocking=False)
        if not self.use_graph:
            self._critic_kernels()
        elif self._cgraph is not None:
            self._cgraph.replay()
        elif getattr(self, '_critic_warm', False):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._critic_kernels()
            self._cgraph = g
            g.replay()
        else:
            self._critic_kernels()
            self._critic_warm = True

    def _on_lr_change(self):
        """The plateau reducer changes the LAST output model's learning rate (the critic,
        base.py:277-284); it is a launch argument of the captured critic minibatches, so
        drop the capture (the next update re-warms and re-captures)."""
        super()._on_lr_change()
        self._cgraph = None
        self._critic_warm = False

    def _critic_kernels(self):
        B, mb = self.batch_size, self.mini_batch_size
        opt = self.critic.optimizer
        ret = self.b_ret.reshape(B)
        for k in range(self.critic_slots.shape[0]):
            for i in range(0, B, mb):  # a ragged last slice as ppo/agent.py:152
                n = min(mb, B - i)
                slots = self.critic_slots.data_ptr() + 8 * (k * B + i)
                call('xa_ring_gather', self.batch_states.data_ptr(), self.mb_states.data_ptr(),
                     slots, n, self.envs.obs_bytes, stream())
                call('xa_ring_gather', ret.data_ptr(), self.mb_ret.data_ptr(), slots, n, 4,
                     stream())
                v = self.ex_critic.forward(self.mb_states)[0]
                # d mean((v - R)^2) / dv = 2 (v - R) / n: xa_mse_grad gives 2 (v - R),
                # the 1 / n rides on Adam's grad_scale (rows past n are never used)
                call('xa_mse_grad', v.data_ptr(), self.mb_ret.data_ptr(), n, 1,
                     self.dvalue.data_ptr(), None, stream())
                self.ex_critic.backward([self.dvalue[:n]], self.critic_grad, batch=n)
                call('xa_adam_step_bump', opt.iterations.data_ptr(), stream())
                kernels.clip_adam(self.critic.theta, opt.m, opt.v, self.critic_grad,
                                  opt.iterations, opt.learning_rate, opt.beta_1, opt.beta_2,
                                  opt.epsilon, grad_scale=1.0 / n, workspace=self.adam_ws)

    def train_step(self):
        """trpo/agent.py:301-348."""
        self.get_batch()
        B = self.batch_size
        call('xa_normalized_advantages', self.b_ret.data_ptr(), self.b_val.data_ptr(), B, 0.0,
             self.adv.data_ptr(), stream())
        # old logits (actor == old actor here) and d surrogate_loss / d theta
        lg = self.ex_actor.forward(self.batch_states)[0]
        self.old_logits.copy_(lg)
        self._head(self.old_logits, dlogits=self.dlogits, out=self.head_out)
        self.ex_actor.backward([self.dlogits], self.flat_grads)
        surrogate_loss = np.float32(self.head_out[0].item())
        self._prepare_fvp()
        step_direction = self.conjugate_gradients(self.flat_grads)
        shs = np.float32(0.5) * self._dot(step_direction, self.calculate_fvp(step_direction))
        lagrange_multiplier = np.float32(np.sqrt(shs / np.float32(self.max_kl)))
        self._axpby(1.0 / float(lagrange_multiplier), step_direction, 0.0, step_direction,
                    self.full_step)
        self.update_actor_weights(surrogate_loss)
        self.update_critic_weights()
        self.last_losses = {'surrogate_loss': float(surrogate_loss), 'shs': float(shs)}
