"""ACER with the xagents class surface (xagents/acer/agent.py:8-387) on the layer executor.

Train step (ACER.train_step, acer/agent.py:363-387):

    rollout, n_steps x [actor-critic forward, Categorical sample, env step] into fixed
    staging buffers, captured once and replayed as a hipGraph (it is launch-bound at
    batch n_envs); then stored as this step's trajectory ring slot (one RB1 entry per env:
    frames [T + 1] incl. the get_states() bootstrap frame -- one xa_ring_gather turns the
    time-major frames env-major --, behaviour logits [T, A], actions, rewards, dones;
    ACER.get_batch / store_batch 127-169)
    update on the fresh trajectories
    once buffer_current_size >= initial_size: poisson(replay_ratio) more updates, each on
    one trajectory per env drawn with random.sample (RB1 batch size 1, buffers.py:59-98)

One update (ACER.update_gradients 295-347):

    model forward on all n_envs (T + 1) frames (xa_gemm per layer, chunks of <= 4096 rows)
    average-model forward on the same frames (trust region only)
    xa_acer_grad: softmax, V = sum p Q, truncated importance, Retrace returns, the
        trust-region-adjusted actor gradient and the critic gradient (acer.hip)
    model backward -> [RCCL all-reduce] -> tf.clip_by_global_norm + Keras Adam (xa_clip_adam)
    xa_ema: average model <- ExponentialMovingAverage(ema_alpha) of the weights

Layouts in HBM: frames uint8 [capacity, n_envs, T + 1, *obs] (an env's trajectory is one
contiguous block, so a sampled batch is one gather of n_envs blocks and the update reads
rows in the reference's env-major order); per-step scalars [capacity, n_envs, T].

Differences from the reference, by design:
* the behaviour policy is kept as its actor logits; mu = softmax(logits) in the kernel
  (the reference stores the softmax output, the same numbers up to f32 rounding);
* the average model starts as a copy of the initial weights (the reference's
  clone_model re-runs the seeded initializers, which give the same values);
* float observations are refused: ACER.get_batch casts states to uint8
  (acer/agent.py:60,167), which only makes sense for image frames.

Reference behaviour kept: the number of replays per train step is drawn ONCE,
np.random.poisson(replay_ratio) at the first step that replays (the reference draws it
while tracing its tf.function train_step, acer/agent.py:363-387); redraw_replays=True
draws it every step (the per-step ACER of the paper).
"""
import ctypes
import random

import numpy as np
import torch
import torch.distributed as dist

from xagents_amd import kernels
from xagents_amd._lib import XaAcerArgs, XaReplayStepArgs, call, stream
from xagents_amd.a2c.agent import A2C
from xagents_amd.base import OnPolicy
from xagents_amd.envs import Discrete
from xagents_amd.layers import LayerExecutor


class ACER(A2C):
    """Sample Efficient Actor-Critic with Experience Replay.
    https://arxiv.org/abs/1611.01224"""

    CHUNK = 4096

    def __init__(
        self,
        envs,
        model,
        buffers,
        ema_alpha=0.99,
        replay_ratio=4,
        epsilon=1e-6,
        importance_c=10.0,
        delta=1,
        trust_region=True,
        entropy_coef=0.01,
        value_loss_coef=0.5,
        grad_norm=0.5,
        use_graph=True,
        redraw_replays=False,
        **kwargs,
    ):
        OnPolicy.__init__(self, envs, model, **kwargs)
        self.redraw_replays = redraw_replays
        self._replay_count = None
        self.entropy_coef = entropy_coef
        self.value_loss_coef = value_loss_coef
        self.grad_norm = grad_norm
        assert (
            len(model.layers) + 1 > 2
        ), f'Expected a model that has at least 3 layers, got {len(model.layers) + 1}'
        activations = [layer.activation for layer in model.layers[-2:]]
        self.output_is_softmax = 'softmax' in activations
        self.distribution_type = 'Categorical'
        self.assert_valid_env(envs[0], Discrete)
        self.buffers = buffers
        assert (
            buffers[0].batch_size == 1
        ), f'Buffer batch size should be 1 for ACER, got {buffers[0].batch_size}'
        self.buffer_current_size = 0
        self.replay_ratio = replay_ratio
        self.epsilon = epsilon
        self.importance_c = importance_c
        self.delta = delta
        self.trust_region = trust_region
        self.ema_alpha = ema_alpha
        self.batch_dtypes = ['uint8', 'float32', 'int32', 'float32', 'float32']
        self.use_graph = use_graph
        self._graph = None
        self._rollout_warm = False
        self.executor_path = True
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        self._setup_acer()

    # ---- device state ------------------------------------------------------------
    def _setup_acer(self):
        env = self.envs
        if not hasattr(env, 'fill_step_args'):
            raise NotImplementedError('ACER needs a transition-replay device env '
                                      '(create_envs for Atari ids)')
        if env.state.dtype != torch.uint8:
            raise NotImplementedError(
                'ACER stores states as uint8 (acer/agent.py:60,167): image observations only')
        if len(self.model.outputs) != 2:
            raise NotImplementedError('ACER models need [actor, critic] outputs')
        outs = self.model.outputs
        self.actor_out = next((k for k, i in enumerate(outs)
                               if self.model.layers[i].activation == 'softmax'), 0)
        self.critic_out = 1 - self.actor_out
        N, T, A = self.n_envs, self.n_steps, self.n_actions
        for i in outs:
            assert self.model.layers[i].units == A, 'ACER actor and critic output n_actions'
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.ob = env.obs_bytes
        assert self.ob % 4 == 0, 'frames are moved as 4-byte words'
        cap = self.buffers[0].size
        self.capacity = cap
        obs_shape = env.obs_shape
        self.obs_buf = torch.zeros((T + 1, N) + obs_shape, dtype=torch.uint8, device=dev)
        # trajectory ring (one RB1 deque entry per env per train step)
        self.r_frames = torch.zeros((cap, N, T + 1) + obs_shape, dtype=torch.uint8, device=dev)
        self.r_mu = torch.zeros(cap, N, T, A, **f32)
        self.r_act = torch.zeros(cap, N, T, dtype=torch.int32, device=dev)
        self.r_rew = torch.zeros(cap, N, T, **f32)
        self.r_done = torch.zeros(cap, N, T, **f32)
        self.count = 0  # trajectories appended per env
        # sampled batch
        self.s_frames = torch.zeros((N, T + 1) + obs_shape, dtype=torch.uint8, device=dev)
        self.s_mu = torch.zeros(N, T, A, **f32)
        self.s_act = torch.zeros(N, T, dtype=torch.int32, device=dev)
        self.s_rew, self.s_done = torch.zeros(N, T, **f32), torch.zeros(N, T, **f32)
        self.s_slots = torch.zeros(N, dtype=torch.int64, device=dev)
        # rollout staging (fixed addresses: the rollout is captured once as a hipGraph and
        # replayed; the ring-slot store runs after it)
        self.g_act = torch.zeros(N, T, dtype=torch.int32, device=dev)
        self.g_mu = torch.zeros(N, T, A, **f32)
        self.g_rew, self.g_done = torch.zeros(N, T, **f32), torch.zeros(N, T, **f32)
        # frame item j = env (T + 1) + t of a trajectory slot <- obs_buf item t N + env
        j = np.arange(N * (T + 1))
        self.frame_perm = torch.from_numpy((j % (T + 1)) * N + j // (T + 1)).to(dev)
        # rollout bookkeeping (episode statistics)
        self.b_logp, self.b_ent = torch.zeros(N, T, **f32), torch.zeros(N, T, **f32)
        self.b_done = torch.zeros(N, T + 1, **f32)
        self.b_epret = torch.zeros(N, T, **f32)
        self.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        seed = self.seed if self.seed is not None else int(np.random.SeedSequence().entropy % 2**63)
        self.rng_seed = (int(seed) * 1000003 + self.rank * 7919 + 17) % 2**64
        self.ex_roll = LayerExecutor(self.model, N)
        self.ex_roll.keep_hidden = False  # forward only
        self._sa = XaReplayStepArgs()
        env.fill_step_args(self._sa)
        self._sa.ring_states = None
        # update: n_envs (T + 1) rows in chunks; chunks keep their activations for backward
        B = N * (T + 1)
        self.B = B
        chunk = min(B, self.CHUNK)
        self.chunk = chunk
        self.ex_chunks = [LayerExecutor(self.model, min(chunk, B - c0))
                          for c0 in range(0, B, chunk)]
        ex0 = self.ex_chunks[0]
        for ex in self.ex_chunks[1:]:
            ex.workspace, ex.dcol = ex0.workspace, ex0.dcol
            ex.douts = [None if d is None else d0[:ex.B] for d, d0 in zip(ex.douts, ex0.douts)]
        self.avg_model = self.model.clone()
        self.avg_ex = {}
        if self.trust_region:
            for ex in self.ex_chunks:
                if ex.B not in self.avg_ex:
                    self.avg_ex[ex.B] = LayerExecutor(self.avg_model, ex.B)
        self.ema_started = False
        self.u_logits, self.u_q = torch.zeros(B, A, **f32), torch.zeros(B, A, **f32)
        self.u_avg = torch.zeros(B, A, **f32)
        self.dlogits, self.dq = torch.zeros(B, A, **f32), torch.zeros(B, A, **f32)
        self.returns = torch.zeros(N, T, **f32)
        self.env_loss = torch.zeros(N, 4, **f32)
        self.grad = torch.zeros(self.model.n_params, **f32)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        if self.distributed:
            dist.broadcast(self.model.theta, 0)
            self.avg_model.theta.copy_(self.model.theta)

    # ---- rollout (A2C.get_batch + ACER.get_batch / store_batch) -----------------------
    def _rollout_kernels(self):
        """n_steps x [forward, Categorical sample, behaviour logits, env step] into the
        staging buffers; obs_buf[t] = the policy input of step t (step t + 1's input is the
        pre-reset obs of step t), obs_buf[T] = get_states() (the bootstrap frame)."""
        N, T, A = self.n_envs, self.n_steps, self.n_actions
        env = self.envs
        a = self._sa
        self.obs_buf[0].copy_(env.state)
        call('xa_copy_block', env.done.data_ptr(), 1, self.b_done.data_ptr(), T + 1, N, 1,
             stream())
        act0, mu0 = self.g_act.data_ptr(), self.g_mu.data_ptr()
        rew0, done0 = self.g_rew.data_ptr(), self.g_done.data_ptr()
        for t in range(T):
            outs = self.ex_roll.forward(self.obs_buf[t])
            logits = outs[self.actor_out]
            call('xa_categorical', logits.data_ptr(), A, N, A, None,
                 self.rng_counter.data_ptr(), self.rng_seed, t, None, act0 + 4 * t,
                 self.b_logp.data_ptr() + 4 * t, self.b_ent.data_ptr() + 4 * t, T, stream())
            call('xa_copy_block', logits.data_ptr(), A, mu0 + 4 * t * A, T * A, N, A, stream())
            a.out_new_states = self.obs_buf.data_ptr() + (t + 1) * N * self.ob
            a.out_rewards = rew0 + 4 * t
            a.out_dones = done0 + 4 * t
            a.done_epret = self.b_epret.data_ptr() + 4 * t
            a.out_ld = T
            if hasattr(env, 'pre_step'):
                env.pre_step()
            call('xa_replay_env_step', ctypes.byref(a), stream())
        call('xa_copy_block', done0, T, self.b_done.data_ptr() + 4, T + 1, N, T, stream())
        self.obs_buf[T].copy_(env.state)
        kernels.counter_bump(self.rng_counter)

    def _play_chunk(self):
        """play(): one eager rollout into the staging buffers (not stored in the ring);
        env 0's rewards and step dones."""
        self._sync_stats_copy()
        self._rollout_kernels()
        return self.g_rew[0].cpu().numpy(), self.g_done[0].cpu().numpy()

    def _acer_rollout(self):
        """One rollout (eager the first time, then a captured hipGraph; envs with a host-side
        pre_step stay eager), stored as this step's trajectory ring slot."""
        N, T = self.n_envs, self.n_steps
        if not self.use_graph or hasattr(self.envs, 'pre_step'):
            self._rollout_kernels()
        elif self._graph is not None:
            self._graph.replay()
        elif self._rollout_warm:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._rollout_kernels()
            self._graph = g
            g.replay()
        else:
            self._rollout_kernels()
            self._rollout_warm = True
        slot = self.count % self.capacity
        call('xa_ring_gather', self.obs_buf.data_ptr(), self.r_frames[slot].data_ptr(),
             self.frame_perm.data_ptr(), N * (T + 1), self.ob, stream())
        self.r_act[slot].copy_(self.g_act)
        self.r_mu[slot].copy_(self.g_mu)
        self.r_rew[slot].copy_(self.g_rew)
        self.r_done[slot].copy_(self.g_done)
        self.count += 1
        for b in self.buffers:
            b.current_size = min(b.current_size + 1, b.size)
        return slot

    # ---- replay (concat_buffer_samples with RB1 batch size 1) --------------------------
    def sample_slots(self):
        """Ring slot of one sampled trajectory per env: random.sample over each env's
        deque (oldest first), in env order (base.py:344-368, buffers.py:89-98)."""
        length = min(self.count, self.capacity)
        first = self.count - length
        return np.array([(first + random.sample(range(length), 1)[0]) % self.capacity
                         for _ in range(self.n_envs)], np.int64)

    def _gather(self, slots):
        N, T, A = self.n_envs, self.n_steps, self.n_actions
        rows = torch.from_numpy(slots * N + np.arange(N, dtype=np.int64))
        self.s_slots.copy_(rows)
        sp = self.s_slots.data_ptr()
        for ring, dst, nb in ((self.r_frames, self.s_frames, (T + 1) * self.ob),
                              (self.r_mu, self.s_mu, 4 * T * A), (self.r_act, self.s_act, 4 * T),
                              (self.r_rew, self.s_rew, 4 * T), (self.r_done, self.s_done, 4 * T)):
            call('xa_ring_gather', ring.data_ptr(), dst.data_ptr(), sp, N, nb, stream())
        return self.s_frames, self.s_mu, self.s_act, self.s_rew, self.s_done

    def _slot_views(self, slot):
        return (self.r_frames[slot], self.r_mu[slot], self.r_act[slot], self.r_rew[slot],
                self.r_done[slot])

    # ---- update (ACER.update_gradients) ----------------------------------------------
    def _acer_update(self, frames, mu, act, rew, done):
        N, T, A, B = self.n_envs, self.n_steps, self.n_actions, self.B
        x = frames.reshape((B,) + self.envs.obs_shape)
        for j, ex in enumerate(self.ex_chunks):
            c0 = j * self.chunk
            outs = ex.forward(x[c0:c0 + ex.B])
            call('xa_copy_block', outs[self.actor_out].data_ptr(), A,
                 self.u_logits.data_ptr() + 4 * c0 * A, A, ex.B, A, stream())
            call('xa_copy_block', outs[self.critic_out].data_ptr(), A,
                 self.u_q.data_ptr() + 4 * c0 * A, A, ex.B, A, stream())
            if self.trust_region:
                avg = self.avg_ex[ex.B].forward(x[c0:c0 + ex.B])[self.actor_out]
                call('xa_copy_block', avg.data_ptr(), A, self.u_avg.data_ptr() + 4 * c0 * A, A,
                     ex.B, A, stream())
        h = XaAcerArgs()
        h.n_envs, h.n_steps, h.n_actions = N, T, A
        h.n_total = N * T  # local mean; the all-reduced sum is scaled by 1 / world in Adam
        h.logits, h.ld_logits = self.u_logits.data_ptr(), A
        h.q, h.ld_q = self.u_q.data_ptr(), A
        h.avg_logits, h.ld_avg = (self.u_avg.data_ptr() if self.trust_region else None), A
        h.mu_logits, h.actions = mu.data_ptr(), act.data_ptr()
        h.rewards, h.dones = rew.data_ptr(), done.data_ptr()
        h.gamma, h.epsilon = float(self.gamma), float(self.epsilon)
        h.importance_c, h.delta = float(self.importance_c), float(self.delta)
        h.entropy_coef, h.value_coef = float(self.entropy_coef), float(self.value_loss_coef)
        h.trust_region = int(bool(self.trust_region))
        h.dlogits, h.ld_dlogits = self.dlogits.data_ptr(), A
        h.dq, h.ld_dq = self.dq.data_ptr(), A
        h.returns, h.env_loss = self.returns.data_ptr(), self.env_loss.data_ptr()
        call('xa_acer_grad', ctypes.byref(h), stream())
        d = [None, None]
        for j, ex in enumerate(self.ex_chunks):
            c0 = j * self.chunk
            d[self.actor_out] = self.dlogits[c0:c0 + ex.B]
            d[self.critic_out] = self.dq[c0:c0 + ex.B]
            ex.backward(d, self.grad, batch=ex.B, accumulate=j > 0)
        if self.distributed:
            dist.all_reduce(self.grad)
        opt = self.model.optimizer
        call('xa_adam_step_bump', opt.iterations.data_ptr(), stream())
        kernels.clip_adam(self.model.theta, opt.m, opt.v, self.grad, opt.iterations,
                          opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                          clip_norm=self.grad_norm, grad_scale=1.0 / self.world_size,
                          workspace=self.adam_ws)
        # ema.apply: the shadow starts at the variable's value on the first apply
        if self.ema_started:
            call('xa_ema', self.avg_model.theta.data_ptr(), self.model.theta.data_ptr(),
                 self.model.n_params, float(np.float32(self.ema_alpha)), stream())
        else:
            self.avg_model.theta.copy_(self.model.theta)
            self.ema_started = True

    def update_avg_weights(self):
        """The average model already holds the moving averages (xa_ema)."""

    def losses(self):
        """Batch-mean [action gain, entropy, value loss] and trust-region adjustment count
        of the last update (host sync)."""
        s = self.env_loss.sum(0).cpu().numpy()
        n = self.n_envs * self.n_steps
        return {'action_loss': -s[0] / n, 'entropy': s[1] / n,
                'value_loss': s[2] / n * self.value_loss_coef, 'adjusted': int(s[3])}

    # ---- train step -------------------------------------------------------------------
    def fused_train_step(self, events=None):
        rec = (lambda i: events[i].record()) if events else (lambda i: None)  # noqa: E731
        rec(0)
        slot = self._acer_rollout()
        rec(1)
        self.buffer_current_size += 1
        self._acer_update(*self._slot_views(slot))
        if self.replay_ratio > 0 and self.buffer_current_size >= self.buffers[0].initial_size:
            n_replay = self._replay_count
            if n_replay is None or self.redraw_replays:
                # the reference's train_step is a tf.function: range(np.random.poisson(...))
                # runs once, at trace time, so ONE draw fixes the replay count of the whole
                # run (acer/agent.py:376-380); redraw_replays=True draws every step instead
                n_replay = np.random.poisson(self.replay_ratio)
                if self.distributed:  # every rank must run the same number of all-reduces
                    t = torch.tensor([n_replay], dtype=torch.int64, device=self.device)
                    dist.broadcast(t, 0)
                    n_replay = int(t.item())
                self._replay_count = n_replay
            for _ in range(n_replay):
                self._acer_update(*self._gather(self.sample_slots()))
        rec(2)
        self.steps += self.n_envs * self.n_steps
        self._queue_episode_stats(self.b_done, self.b_epret)

    def train_step(self):
        self.fused_train_step()
