"""On-policy actor-critic train step for models run through the layer executor (the
CNN actor-critic of xagents/{a2c,ppo}/models/cnn-actor-critic.cfg, config C4) -- the
counterpart of the fused MLP kernels for any .cfg actor-critic.

Rollout (A2C.get_batch, xagents/a2c/agent.py:96-139), per step t:
    CNN forward of obs[t] (uint8 frames, scaled in the GEMM loader)   xa_gemm x layers
    Categorical sample / log-prob / entropy (Philox uniforms)          xa_categorical
    (Box action spaces: MultivariateNormalDiag(loc) sample / log-prob  xa_diag_gaussian)
    value -> values[:, t]                                              xa_copy_block
    env step: reward / done rows, obs[t+1] = the pre-reset obs (the
    terminal-obs feed-through of a2c/agent.py:132-136)                 xa_replay_env_step
then V(get_states()) and GAE / n-step returns (xa_gae / xa_nstep_returns).
Update (PPO.run_ppo_epochs ppo/agent.py:157-191, A2C.train_step a2c/agent.py:190-218):
every epoch's shuffle drawn and uploaded at once, the advantage statistics of every
minibatch in one launch (xa_minibatch_adv_sums) [+ ONE all-reduce of them per train step],
then per minibatch gather (xa_ring_gather) -> forward -> xa_ac_head_grad -> backward
[-> bucketed RCCL all-reduce of the gradient: the dense layers' slice is issued as soon as
its weight gradient is final, overlapping the conv backward] -> tf.clip_by_global_norm +
Keras Adam (xa_clip_adam).
Layouts: frames time-major [T+1, N, ...] (each step's batch is contiguous for the
GEMMs); per-step scalars env-major [N, T] (concat_step_batches order, base.py:549-564).
"""
import ctypes

import numpy as np
import torch

from xagents_amd import kernels
from xagents_amd._lib import (XA_DIST_DIAG_GAUSSIAN, XA_LOSS_PPO, XA_RETURNS_GAE,
                              XaHeadGradArgs, XaReplayStepArgs, call, stream)
from xagents_amd.layers import LayerExecutor


class ExecutorActorCritic:
    """Mixin for A2C / PPO when the model is not the fused actor-critic MLP."""

    CHUNK = 4096

    def _setup_executor_path(self):
        env = self.envs
        if not hasattr(env, 'fill_step_args'):
            raise NotImplementedError('the executor on-policy path needs a transition-replay '
                                      'device env (create_envs for Atari / BipedalWalker ids)')
        if len(self.model.outputs) != 2:
            raise NotImplementedError('actor-critic models need [logits, value] outputs')
        N, T = self.n_envs, self.n_steps
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs_buf = torch.zeros((T + 1, N) + env.obs_shape,
                                   dtype=env.state.dtype, device=dev)
        # Box action spaces: MultivariateNormalDiag(loc = actor output), f32 action rows
        self.gaussian = getattr(self, 'distribution_type', 'Categorical') != 'Categorical'
        A = self.n_actions
        if self.gaussian:
            self.b_act = torch.zeros(N, T, A, dtype=torch.float32, device=dev)
        else:
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
        self.rng_seed = (int(seed) * 1000003 + self.rank * 7919 + 17) % 2**64
        self.ex_roll = LayerExecutor(self.model, N)
        self.ex_roll.keep_hidden = False  # forward only
        self._sa = XaReplayStepArgs()
        env.fill_step_args(self._sa)
        self._sa.ring_states = None
        B = N * T
        mb = getattr(self, 'mini_batch_size', B)
        self.mb = mb
        self.n_mb = (B + mb - 1) // mb
        # the update minibatch runs in chunks of <= 4096 samples (each chunk keeps its own
        # activations; GEMM index ranges stay 32-bit), gradients accumulate over chunks
        self.chunk = min(mb, self.CHUNK)
        self.ex_chunks = [LayerExecutor(self.model, min(self.chunk, mb - c0))
                          for c0 in range(0, mb, self.chunk)]
        ex0 = self.ex_chunks[0]
        for ex in self.ex_chunks[1:]:  # backward buffers are used one chunk at a time
            ex.workspace, ex.dcol = ex0.workspace, ex0.dcol
            ex.douts = [None if d is None else d0[:ex.B] for d, d0 in zip(ex.douts, ex0.douts)]
        self.mb_logits = torch.zeros(mb, self.n_actions, **f32)
        self.mb_value = torch.zeros(mb, 1, **f32)
        self.mb_obs = torch.zeros((mb,) + env.obs_shape, dtype=env.state.dtype, device=dev)
        self.mb_act = (torch.zeros(mb, A, dtype=torch.float32, device=dev) if self.gaussian
                       else torch.zeros(mb, dtype=torch.int32, device=dev))
        self.mb_logp, self.mb_val = torch.zeros(mb, **f32), torch.zeros(mb, **f32)
        self.mb_ret = torch.zeros(mb, **f32)
        self.dlogits = torch.zeros(mb, self.n_actions, **f32)
        self.dvalue = torch.zeros(mb, 1, **f32)
        self.head_loss = torch.zeros(3, **f32)
        E = getattr(self, 'ppo_epochs', 1)
        # [sum adv, sum adv^2, count] of every (epoch, minibatch) of a train step
        self.adv_sums = torch.zeros(E * self.n_mb, 3, dtype=torch.float64, device=dev)
        self.grad = torch.zeros(self.model.n_params, **f32)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        # every epoch's shuffled sample slots of a train step, uploaded in one copy
        self._slots_obs = torch.zeros(E * B, dtype=torch.int64, device=dev)
        self._slots_flat = torch.zeros(E * B, dtype=torch.int64, device=dev)
        self._exec_uniforms = None
        # data parallel: all-reduce buckets of at least this many bytes, issued while the
        # backward of the earlier layers runs (XA_BUCKET_MB, default 4)
        import os
        self.bucket_floats = int(float(os.environ.get('XA_BUCKET_MB', '4')) * (1 << 20)) // 4
        if self.distributed:
            torch.distributed.broadcast(self.model.theta, 0)

    # ---- rollout ------------------------------------------------------------------
    def _executor_rollout(self):
        N, T = self.n_envs, self.n_steps
        env = self.envs
        a = self._sa
        self.obs_buf[0].copy_(env.state)
        call('xa_copy_block', env.done.data_ptr(), 1, self.b_done.data_ptr(), T + 1, N, 1,
             stream())
        ob = env.obs_bytes
        for t in range(T):
            logits, value = self.ex_roll.forward(self.obs_buf[t])
            A = self.n_actions
            if self.gaussian:
                call('xa_diag_gaussian', logits.data_ptr(), A, N, A, None,
                     self.rng_counter.data_ptr(), self.rng_seed, t, None, T * A,
                     self.b_act.data_ptr() + 4 * t * A, self.b_logp.data_ptr() + 4 * t,
                     self.b_ent.data_ptr() + 4 * t, T, stream())
            else:
                u = self._exec_uniforms
                call('xa_categorical', logits.data_ptr(), A, N, A,
                     None if u is None else u.data_ptr() + 4 * t * N,
                     self.rng_counter.data_ptr(), self.rng_seed, t, None,
                     self.b_act.data_ptr() + 4 * t, self.b_logp.data_ptr() + 4 * t,
                     self.b_ent.data_ptr() + 4 * t, T, stream())
            call('xa_copy_block', value.data_ptr(), 1, self.b_val.data_ptr() + 4 * t, T, N, 1,
                 stream())
            a.out_new_states = self.obs_buf.data_ptr() + (t + 1) * N * ob
            a.out_rewards = self.b_rew.data_ptr() + 4 * t
            a.out_dones = self.b_dstep.data_ptr() + 4 * t
            a.done_epret = self.b_epret.data_ptr() + 4 * t
            a.out_ld = T  # env-major [N, T] rows
            if hasattr(env, 'pre_step'):
                # raw-frame env (AtariWrapper.step) / dynamics env (env.step with step t's
                # actions: env-major rows of b_act, stride T A) into the one-step record
                if self.gaussian:
                    env.pre_step(self.b_act.data_ptr() + 4 * t * A, T * A)
                else:
                    env.pre_step(self.b_act.data_ptr() + 4 * t, T)
            call('xa_replay_env_step', ctypes.byref(a), stream())
        # dones[:, t + 1] = done of step t (dones[:, 0] is the carried-in flag)
        call('xa_copy_block', self.b_dstep.data_ptr(), T, self.b_done.data_ptr() + 4, T + 1, N,
             T, stream())
        value = self.ex_roll.forward(env.state)[1]
        call('xa_copy_block', value.data_ptr(), 1, self.next_val.data_ptr(), 1, N, 1, stream())
        if self.return_kind == XA_RETURNS_GAE:
            kernels.gae(self.b_rew, self.b_val, self.b_done, self.next_val, self.gamma,
                        self.lam, out=self.b_ret)
        else:
            kernels.nstep_returns(self.b_rew, self.b_done, self.next_val, self.gamma,
                                  out=self.b_ret)
        kernels.counter_bump(self.rng_counter)

    # ---- update ---------------------------------------------------------------------
    def _upload_slots(self, flat_idx):
        """flat env-major sample indices i = env T + t -> frame slots t N + env."""
        N, T = self.n_envs, self.n_steps
        idx = np.asarray(flat_idx, np.int64)
        obs_slots = (idx % T) * N + idx // T
        self._slots_obs[:idx.size].copy_(torch.from_numpy(obs_slots))
        self._slots_flat[:idx.size].copy_(torch.from_numpy(idx))
        return idx.size

    def _gather_minibatch(self, n, off=0):
        """Gather the n samples whose slots start at slot row `off`."""
        so = self._slots_obs.data_ptr() + 8 * off
        sf = self._slots_flat.data_ptr() + 8 * off
        call('xa_ring_gather', self.obs_buf.data_ptr(), self.mb_obs.data_ptr(), so, n,
             self.envs.obs_bytes, stream())
        act_bytes = 4 * self.n_actions if self.gaussian else 4
        for src, dst, nb in ((self.b_act, self.mb_act, act_bytes), (self.b_logp, self.mb_logp, 4),
                             (self.b_val, self.mb_val, 4), (self.b_ret, self.mb_ret, 4)):
            call('xa_ring_gather', src.data_ptr(), dst.data_ptr(), sf, n, nb, stream())

    def _minibatch_step(self, n, k=None):
        """One optimizer step on the gathered minibatch of n samples. k: its row of
        adv_sums (the train step's precomputed, all-reduced advantage statistics); None
        computes them from the minibatch itself (all-reduced in place when data
        parallel)."""
        A = self.n_actions
        for j, ex in enumerate(self.ex_chunks):
            c0 = j * self.chunk
            if c0 >= n:
                break
            lg, vl = ex.forward(self.mb_obs[c0:c0 + ex.B])
            rows = min(ex.B, n - c0)
            call('xa_copy_block', lg.data_ptr(), A, self.mb_logits.data_ptr() + 4 * c0 * A, A,
                 rows, A, stream())
            call('xa_copy_block', vl.data_ptr(), 1, self.mb_value.data_ptr() + 4 * c0, 1, rows,
                 1, stream())
        logits, value = self.mb_logits, self.mb_value
        h = XaHeadGradArgs()
        h.n, h.n_actions, h.loss_kind = n, self.n_actions, self.loss_kind
        h.logits, h.ld_logits = logits.data_ptr(), self.n_actions
        h.values, h.ld_values = value.data_ptr(), 1
        if self.gaussian:
            h.dist_kind, h.actions = XA_DIST_DIAG_GAUSSIAN, None
            h.actions_f, h.ld_actions = self.mb_act.data_ptr(), A
        else:
            h.actions = self.mb_act.data_ptr()
        h.old_logp = self.mb_logp.data_ptr()
        h.old_values, h.returns = self.mb_val.data_ptr(), self.mb_ret.data_ptr()
        h.clip_norm = float(getattr(self, 'clip_norm', 0.0))
        h.entropy_coef, h.value_coef = float(self.entropy_coef), float(self.value_loss_coef)
        h.adv_eps = float(getattr(self, 'advantage_epsilon', 0.0))
        h.dlogits, h.dvalues, h.loss = (self.dlogits.data_ptr(), self.dvalue.data_ptr(),
                                        self.head_loss.data_ptr())
        h.stats_mode = 0
        if self.loss_kind == XA_LOSS_PPO and k is not None:
            h.stats_mode, h.adv_stats = 2, self.adv_sums[k].data_ptr()
        elif self.distributed and self.loss_kind == XA_LOSS_PPO:
            sums = self.adv_sums[0]
            h.adv_stats = sums.data_ptr()
            h.stats_mode = 1
            call('xa_ac_head_grad', ctypes.byref(h), stream())
            torch.distributed.all_reduce(sums)
            h.stats_mode = 2
        call('xa_ac_head_grad', ctypes.byref(h), stream())
        works = []
        n_chunks = sum(1 for j in range(len(self.ex_chunks)) if j * self.chunk < n)
        hook = self._bucket_hook(works) if self.distributed else None
        for j, ex in enumerate(self.ex_chunks[:n_chunks]):
            c0 = j * self.chunk
            rows = min(ex.B, n - c0)
            ex.backward([self.dlogits[c0:c0 + rows], self.dvalue[c0:c0 + rows]], self.grad,
                        batch=rows, accumulate=j > 0,
                        on_grad=hook if j == n_chunks - 1 else None)
        if self.distributed:
            # the slice no bucket has taken yet (the first layers), then wait for the
            # buckets in flight: the optimizer reads the whole all-reduced gradient
            if self._bucket_hi > 0:
                torch.distributed.all_reduce(self.grad[:self._bucket_hi])
            for w in works:
                w.wait()
        opt = self.model.optimizer
        call('xa_adam_step_bump', opt.iterations.data_ptr(), stream())
        kernels.clip_adam(self.model.theta, opt.m, opt.v, self.grad, opt.iterations,
                          opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                          clip_norm=self.grad_norm, grad_scale=1.0 / self.world_size,
                          workspace=self.adam_ws)

    def _bucket_hook(self, works):
        """Backward hook of the last chunk (LayerExecutor.backward on_grad): layers finish
        in reverse parameter order, so once layer l's weight gradient is queued the slice
        grad[w0_l:] is final; every slice of at least bucket_floats goes into an async
        all-reduce right away (on RCCL's stream, behind the launches that wrote it) while
        the compute stream goes on with the earlier layers' backward. For the CNN
        actor-critic the first bucket is the dense layers' 77 MB, in flight during the dense
        input gradient and the conv backward."""
        self._bucket_hi = self.model.n_params

        def hook(w0):
            if self._bucket_hi - w0 >= self.bucket_floats:
                works.append(torch.distributed.all_reduce(self.grad[w0:self._bucket_hi],
                                                          async_op=True))
                self._bucket_hi = w0
        return hook

    def _shuffles(self):
        """Every epoch's permutation of the env-major batch (get_mini_batches,
        ppo/agent.py:139-155): numpy's global RNG, one np.random.permutation per epoch in
        epoch order; or the parity-mode permutations of set_minibatch_permutation."""
        B = self.n_envs * self.n_steps
        host = getattr(self, '_host_perm', None)
        if host is not None:
            return host.cpu().numpy().astype(np.int64).reshape(-1)
        return np.concatenate([np.random.permutation(B) for _ in range(self.ppo_epochs)])

    def _executor_update(self):
        B = self.n_envs * self.n_steps
        if self.loss_kind == XA_LOSS_PPO:
            # all epochs' shuffles at once, then contiguous minibatch slices of each; the
            # advantage statistics of all E x M minibatches in one launch and (data
            # parallel) one all-reduce, instead of one blocking collective per minibatch
            E = self.ppo_epochs
            if self._slots_obs.numel() < E * B or self.adv_sums.shape[0] < E * self.n_mb:
                # ppo_epochs raised after construction
                dev = self.device
                self._slots_obs = torch.zeros(E * B, dtype=torch.int64, device=dev)
                self._slots_flat = torch.zeros(E * B, dtype=torch.int64, device=dev)
                self.adv_sums = torch.zeros(E * self.n_mb, 3, dtype=torch.float64, device=dev)
            self._upload_slots(self._shuffles())
            call('xa_minibatch_adv_sums', self.b_ret.data_ptr(), self.b_val.data_ptr(),
                 self._slots_flat.data_ptr(), B, self.mb, self.ppo_epochs,
                 self.adv_sums.data_ptr(), stream())
            if self.distributed:
                torch.distributed.all_reduce(self.adv_sums)
            k = 0
            for e in range(self.ppo_epochs):
                for m in range(self.n_mb):
                    n = min(self.mb, B - m * self.mb)
                    self._gather_minibatch(n, e * B + m * self.mb)
                    self._minibatch_step(n, k)
                    k += 1
        else:
            n = self._upload_slots(np.arange(B))
            self._gather_minibatch(n)
            self._minibatch_step(n)

    def _executor_train_step(self):
        self._executor_rollout()
        self._executor_update()
        self.steps += self.n_envs * self.n_steps
        self._queue_episode_stats(self.b_done, self.b_epret)

