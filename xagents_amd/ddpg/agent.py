"""DDPG with the xagents class surface (xagents/ddpg/agent.py:7-166) on the device path.

Per gradient step (ddpg/agent.py:129-147), all launches on device:
    concat_buffer_samples   host index draw (np.random.randint per RB2, the reference's
                            stream) -> xa_ring_gather
    update_critic_weights   target_actor(s') -> [s', a'] -> target_critic -> y;
                            critic([s, a]) -> xa_critic_td_grad -> backward -> Keras Adam
    update_actor_weights    actor(s) -> critic([s, pi(s)]) -> d(-mean Q)/d input ->
                            actor backward -> Keras Adam           (every policy_delay)
    sync_target_models      xa_polyak (1 - tau) target + tau online (every policy_delay)
The MLPs run on xa_gemm through the layer executor (xagents_amd/layers.py).
"""
import ctypes

import numpy as np
import torch

from xagents_amd import kernels
from xagents_amd._lib import call, stream
from xagents_amd.base import OffPolicy
from xagents_amd.envs import Box
from xagents_amd.layers import LayerExecutor


class DDPG(OffPolicy):
    """Continuous control with deep reinforcement learning https://arxiv.org/abs/1509.02971"""

    def __init__(
        self,
        envs,
        actor_model,
        critic_model,
        buffers,
        gradient_steps=None,
        tau=0.05,
        step_noise_coef=0.1,
        huber_delta=None,
        **kwargs,
    ):
        super(DDPG, self).__init__(envs, actor_model, buffers, **kwargs)
        # opt-in Huber-TD critic loss (BASELINE north_star; the reference uses MSE,
        # ddpg/agent.py:126, td3/agent.py:102-104): None keeps the reference's MSE
        self.huber_delta = huber_delta
        self.assert_valid_env(envs[0], Box)
        self.actor = actor_model
        self.critic = critic_model
        self.policy_delay = 1
        self.gradient_steps = gradient_steps
        self.tau = tau
        self.step_noise_coef = step_noise_coef
        self.episode_steps = np.zeros(self.n_envs, np.float32)
        self.output_models.append(self.critic)
        self.target_actor = self.actor.clone()
        self.target_critic = self.critic.clone()
        self.model_groups = [(self.actor, self.target_actor), (self.critic, self.target_critic)]
        self.batch_dtypes = 5 * ['float32']
        self._setup_device()

    # ---- device state ----------------------------------------------------------
    def _setup_device(self):
        S = int(np.prod(self.envs.obs_shape))
        A = self.n_actions
        self._setup_offpolicy((A,), np.float32)
        B = self.n_envs * self.replay.k
        self.batch_size, self.S, self.A = B, S, A
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.s, self.s2 = torch.zeros(B, S, **f32), torch.zeros(B, S, **f32)
        self.a = torch.zeros(B, A, **f32)
        self.r, self.d = torch.zeros(B, **f32), torch.zeros(B, **f32)
        self.sa, self.s2a2 = torch.zeros(B, S + A, **f32), torch.zeros(B, S + A, **f32)
        self.spa, self.dspa = torch.zeros(B, S + A, **f32), torch.zeros(B, S + A, **f32)
        self.da = torch.zeros(B, A, **f32)
        self.dv1, self.dv2 = torch.zeros(B, 1, **f32), torch.zeros(B, 1, **f32)
        self.critic_loss = torch.zeros(B, **f32)
        self.dq_actor = torch.full((B, 1), -1.0 / B, **f32)  # d(-mean Q)/dQ
        self.noise = torch.zeros(B, A, **f32)
        self.ta_smooth = torch.zeros(B, A, **f32)
        self.step_actions = torch.zeros(self.n_envs, A, **f32)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        self.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        seed = self.seed if self.seed is not None else int(np.random.SeedSequence().entropy % 2**63)
        self.rng_seed = (int(seed) * 2654435761 + 97) % 2**64
        self.ex_step = LayerExecutor(self.actor, self.n_envs)
        self.ex_actor = LayerExecutor(self.actor, B)
        self.ex_target_actor = LayerExecutor(self.target_actor, B)
        self.ex_critic = LayerExecutor(self.critic, B)
        self.ex_critic_pi = LayerExecutor(self.critic, B)
        self.ex_target_critic = LayerExecutor(self.target_critic, B)
        self.g_actor = torch.zeros(self.actor.n_params, **f32)
        self.g_critic = torch.zeros(self.critic.n_params, **f32)
        self._sync_params(self.actor, self.critic, self.target_actor, self.target_critic)

    def _concat(self, left, right, out):
        B = self.batch_size
        call('xa_copy_block', left.data_ptr(), left.shape[1], out.data_ptr(), out.shape[1], B,
             left.shape[1], stream())
        call('xa_copy_block', right.data_ptr(), right.shape[1], out.data_ptr() + 4 * left.shape[1],
             out.shape[1], B, right.shape[1], stream())

    def _adam(self, model, grad, mean=False):
        opt = model.optimizer
        scale = self._reduce_grad(grad, mean=mean)
        call('xa_adam_step_bump', opt.iterations.data_ptr(), stream())
        kernels.clip_adam(model.theta, opt.m, opt.v, grad, opt.iterations, opt.learning_rate,
                          opt.beta_1, opt.beta_2, opt.epsilon, clip_norm=0.0,
                          grad_scale=scale, workspace=self.adam_ws)

    def _noisy(self, x, sigma, noise_clip, out, noise_out=None):
        rows, cols = x.shape
        call('xa_noisy_actions', x.data_ptr(), cols, rows, cols, kernels._f32(sigma),
             kernels._f32(noise_clip), kernels._f32(-1.0), kernels._f32(1.0),
             self.rng_counter.data_ptr(), self.rng_seed, out.data_ptr(), out.shape[1],
             noise_out.data_ptr() if noise_out is not None else None, stream())
        kernels.counter_bump(self.rng_counter)

    # ---- reference surface ---------------------------------------------------------
    def get_step_actions(self):
        """clip(actor(s) + N(0, step_noise_coef), -1, 1) (ddpg/agent.py:60-71): one launch
        (xa_td3_act: actor forward, tanh, the noise and the clip, the counter bump) when the
        actor is the 3-layer .cfg MLP; otherwise the layer executor + xa_noisy_actions."""
        fa = self._fused_act_args()
        if fa is not None:
            fa.states = self.envs.state.data_ptr()
            call('xa_td3_act', ctypes.byref(fa), stream())
            return self.step_actions
        a = self.ex_step.forward(self.envs.state)[0]
        self._noisy(a, self.step_noise_coef, float('inf'), self.step_actions)
        return self.step_actions

    def _device_checks(self):
        """A fused launch whose grid barrier timed out (its workgroups were not all resident
        within 10 s) set the status word and left the step unfinished: fail loudly."""
        st = self.__dict__.get('_fused_status')
        if st is not None and int(st.item()) != 0:
            raise RuntimeError('xa_td3_update / xa_td3_act: a grid barrier timed out (the '
                               'persistent launch needs every workgroup resident); the '
                               'gradient step state is invalid')

    def _step_noise(self):
        """(sigma, counter bump) of the exploration step: DDPG draws N(0, step_noise_coef)."""
        return self.step_noise_coef, 1

    def _fused_act_args(self):
        """xa_td3_act's launch arguments (built once), or None (other actor shapes, an env
        batch over 256 or a non-contiguous f32 state)."""
        if '_fused_act' in self.__dict__:
            return self.__dict__['_fused_act']
        import os
        from xagents_amd import _lib
        from xagents_amd._lib import XaTd3ActArgs
        fa = None
        st = getattr(self.envs, 'state', None)
        if (os.environ.get('XA_TD3_FUSED', '1') != '0' and self._fused_ok() and
                isinstance(st, torch.Tensor) and st.dtype == torch.float32 and st.dim() == 2 and
                st.is_contiguous() and st.shape[1] == self.S and st.shape[0] <= 256):
            fa = XaTd3ActArgs()
            n, S, A = st.shape[0], self.S, self.A
            H1, H2 = self.actor.layers[0].units, self.actor.layers[1].units
            fa.n, fa.obs_dim, fa.act_dim, fa.h1, fa.h2 = n, S, A, H1, H2
            fa.states, fa.theta = st.data_ptr(), self.actor.theta.data_ptr()
            sigma, bump = self._step_noise()
            fa.sigma = kernels._f32(sigma)
            fa.noise_clip = float('inf')
            fa.lo, fa.hi = kernels._f32(-1.0), kernels._f32(1.0)
            fa.rng_counter, fa.seed, fa.bump = self.rng_counter.data_ptr(), self.rng_seed, bump
            fa.out, fa.ld_out = self.step_actions.data_ptr(), self.step_actions.shape[1]
            fa.noise_out = None
            nbytes = _lib.load().xa_td3_act_workspace_bytes(n, S, A, H1, H2)
            self._fused_act_ws = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
            fa.workspace, fa.workspace_bytes = self._fused_act_ws.data_ptr(), nbytes
            fa.n_blocks = int(os.environ.get('XA_TD3_ACT_BLOCKS', '0')) or self._shared_blocks()
            if '_fused_status' not in self.__dict__:
                self._fused_status = torch.zeros(1, dtype=torch.int32, device=self.device)
            fa.status = self._fused_status.data_ptr()
        self.__dict__['_fused_act'] = fa
        return fa

    def _play_actions(self):
        """play(): the actor's output without exploration noise (self.actor(states),
        xagents/base.py:639-640)."""
        return self.ex_step.forward(self.envs.state)[0]

    def sync_target_models(self):
        """target = (1 - tau) target + tau online, every model group (ddpg/agent.py:73-85)."""
        for model, target in self.model_groups:
            call('xa_polyak', model.theta.data_ptr(), target.theta.data_ptr(), model.n_params,
                 kernels._f32(self.tau), stream())

    def _target_inputs(self):
        ta = self.ex_target_actor.forward(self.s2)[0]
        self._concat(self.s2, ta, self.s2a2)

    def update_critic_weights(self, states=None, actions=None, new_states=None, dones=None,
                              rewards=None):
        """ddpg/agent.py:104-127 on the gathered batch."""
        self._target_inputs()
        tv = self.ex_target_critic.forward(self.s2a2)[0]
        self._concat(self.s, self.a, self.sa)
        v = self.ex_critic.forward(self.sa)[0]
        call('xa_critic_td_grad', v.data_ptr(), None, tv.data_ptr(), None, self.r.data_ptr(),
             self.d.data_ptr(), self.batch_size, kernels._f32(self.gamma),
             kernels._f32(self.huber_delta or 0.0), self.dv1.data_ptr(), None,
             self.critic_loss.data_ptr(), stream())
        self.ex_critic.backward([self.dv1], self.g_critic)
        self._adam(self.critic, self.g_critic)

    def update_actor_weights(self, states=None):
        """-mean(critic([s, actor(s)])) minimized over the actor (ddpg/agent.py:87-102)."""
        pa = self.ex_actor.forward(self.s)[0]
        self._concat(self.s, pa, self.spa)
        self.ex_critic_pi.forward(self.spa)
        self.ex_critic_pi.backward([self.dq_actor], None, dinput=self.dspa)
        call('xa_copy_block', self.dspa.data_ptr() + 4 * self.S, self.S + self.A,
             self.da.data_ptr(), self.A, self.batch_size, self.A, stream())
        self.ex_actor.backward([self.da], self.g_actor)
        self._adam(self.actor, self.g_actor, mean=True)

    def concat_buffer_samples(self):
        slots = self.replay.upload_slots(self.replay.sample_slots())
        self.replay.gather(slots, self.s, self.a, self.r, self.d, self.s2)
        return [self.s, self.a, self.r, self.d, self.s2]

    def update_weights(self, gradient_steps):
        """ddpg/agent.py:129-147. The sample indices come from the host RNG exactly as
        before. The device work of a gradient step (gather, critic update; actor update and
        Polyak sync) is ONE persistent launch (xa_td3_update, csrc/td3_update.hip) when the
        models are the 3-layer .cfg MLPs and the run is one process; otherwise the layer
        executor's ~40-90 launches, captured once per phase and replayed as hipGraphs."""
        fused = self._fused_args()
        for gradient_step in range(int(gradient_steps)):
            policy = gradient_step % self.policy_delay == 0
            if fused is not None and not self.distributed and self._staged_slots_ok():
                # the launch reads the sampled slots from one of two mapped pinned buffers
                # (no upload copy); one captured graph per (phase, buffer)
                i = self._stage_fused_slots(self.replay.sample_slots())
                fused.slots = self._fslots['dev'][i]
                if self._fused_graph():
                    self._run_phase(('fused_actor' if policy else 'fused') + f'@{i}',
                                    lambda p=policy: self._fused_step(p))
                else:
                    self._fused_step(policy)
                self._fslots['ev'][i].record()
                continue
            self.replay.upload_slots(self.replay.sample_slots())
            if fused is not None and self.distributed:
                self._fused_dp_step(policy)
                continue
            if fused is not None:
                fused.slots = self.replay.slots.data_ptr()
                self._run_phase('fused_actor' if policy else 'fused',
                                lambda p=policy: self._fused_step(p))
                continue
            self._run_phase('critic', self._critic_phase)
            if policy:
                self._run_phase('actor', self._actor_phase)

    # ---- the fused gradient step (xa_td3_update) -------------------------------------
    def _staged_slots_ok(self):
        """(XA_TD3_STAGED_SLOTS=0: the upload copy into the device slot buffer instead)"""
        if '_sslots' not in self.__dict__:
            import os
            self._sslots = os.environ.get('XA_TD3_STAGED_SLOTS', '1') != '0' and \
                torch.device(self.device).type == 'cuda'
        return self._sslots

    def _fused_graph(self):
        """Launch the one-kernel gradient step directly (default) or replay it from a captured
        hipGraph (XA_TD3_GRAPH=1): a replay adds its own submission latency in front of the
        kernel (C5 gradient step 0.128 -> 0.121 ms launched directly,
        profiles/r06p_td3_graph_ab.txt)."""
        if '_fgraph' not in self.__dict__:
            import os
            self._fgraph = os.environ.get('XA_TD3_GRAPH', '0') == '1'
        return self._fgraph

    def _stage_fused_slots(self, slots):
        """The gradient step's sample slots into one of two mapped pinned buffers, which the
        fused launch reads over the host link (each workgroup once, into its LDS slot
        table), replacing the host -> device copy launch. Alternates buffers; the launch
        that read this buffer two gradient steps ago must have finished (its event).
        Returns the buffer index."""
        st = self.__dict__.get('_fslots')
        if st is None:
            bufs, devs = [], []
            for _ in range(2):
                t = torch.zeros(len(slots), dtype=torch.int64).pin_memory()
                dp = ctypes.c_void_p()
                call('xa_host_device_pointer', ctypes.c_void_p(t.data_ptr()), ctypes.byref(dp))
                bufs.append(t)
                devs.append(dp.value)
            st = self._fslots = {'buf': bufs, 'dev': devs, 'i': 0,
                                 'ev': [torch.cuda.Event(), torch.cuda.Event()], 'used': [False] * 2}
        i = st['i']
        if st['used'][i]:
            st['ev'][i].synchronize()
        st['buf'][i].numpy()[:] = slots
        st['used'][i] = True
        st['i'] = i ^ 1
        return i

    def _shared_blocks(self):
        """Grid of the persistent TD3 launches (0 = the kernel's default, one workgroup per
        CU up to 256). Ranks sharing one GPU each take 3/4 of their share of
        the CUs, so every rank's launch is resident at once and the grid barriers cannot
        wait on a workgroup that is queued behind another rank's spinning grid."""
        share = getattr(self, '_ranks_share', 1)
        if share <= 1:
            return 0
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        return max(16, min(256, cus) // share * 3 // 4)

    def _fused_ok(self):
        import os
        if os.environ.get('XA_TD3_FUSED', '1') == '0':
            return False
        if self.replay.obs_t != torch.float32 or self.replay.act_t != torch.float32:
            return False
        if len(self.envs.obs_shape) != 1:
            return False
        models = [self.actor, self.critic] + ([self.critic2] if hasattr(self, 'critic2') else [])
        want = {id(self.actor): ['relu', 'relu', 'tanh']}
        h = None
        for m in models:
            ls = m.layers
            if len(ls) != 3 or any(l.kind != 'dense' for l in ls) or list(m.outputs) != [2]:
                return False
            acts = [l.activation or 'linear' for l in ls]
            if acts != want.get(id(m), ['relu', 'relu', 'linear']):
                return False
            if any(l.input_index != i - 1 for i, l in enumerate(ls)):
                return False
            dims = (ls[0].units, ls[1].units)
            if h is not None and dims != h:
                return False
            h = dims
        S, A = self.S, self.A
        if self.actor.layers[2].units != A or self.critic.layers[2].units != 1:
            return False
        if self.actor.layers[0].in_features != S or self.critic.layers[0].in_features != S + A:
            return False
        B = self.batch_size
        return (B <= 256 and max(h) <= 416 and h[0] % 4 == 0 and h[1] % 4 == 0 and S + A <= 64
                and A <= 4 and h[1] * A <= 2048 and B * A <= 1024)

    def _fused_args(self):
        """The launch arguments of xa_td3_update (built once), or None when the fused step
        does not apply (other model shapes). Data parallel runs it in stages with the
        gradient all-reduces between them (_fused_dp_step)."""
        if '_fused' in self.__dict__:
            return self.__dict__['_fused']
        from xagents_amd import _lib
        from xagents_amd._lib import XaTd3UpdateArgs
        fused = None
        if self._fused_ok():
            a = XaTd3UpdateArgs()
            B, S, A = self.batch_size, self.S, self.A
            H1, H2 = self.actor.layers[0].units, self.actor.layers[1].units
            a.batch, a.obs_dim, a.act_dim, a.h1, a.h2 = B, S, A, H1, H2
            twin = hasattr(self, 'critic2')
            a.twin = a.smooth = int(twin)
            a.gamma = kernels._f32(self.gamma)
            a.tau = kernels._f32(self.tau)
            a.noise_sigma = kernels._f32(getattr(self, 'policy_noise_coef', 0.0))
            a.noise_clip = kernels._f32(getattr(self, 'noise_clip', 0.0))
            a.huber_delta = kernels._f32(self.huber_delta or 0.0)
            r = self.replay
            a.ring_states, a.ring_new_states = r.states.data_ptr(), r.new_states.data_ptr()
            a.ring_actions = r.actions.data_ptr()
            a.ring_rewards, a.ring_dones = r.rewards.data_ptr(), r.dones.data_ptr()
            a.slots = r.slots.data_ptr()
            a.rng_counter, a.seed = self.rng_counter.data_ptr(), self.rng_seed

            def net(model, target=False):
                n = type(a.actor)()
                n.theta = model.theta.data_ptr()
                if not target:
                    opt = model.optimizer
                    n.m, n.v, n.step = opt.m.data_ptr(), opt.v.data_ptr(), opt.iterations.data_ptr()
                    n.lr, n.beta1 = opt.learning_rate, opt.beta_1
                    n.beta2, n.eps = opt.beta_2, opt.epsilon
                return n
            a.actor, a.critic1 = net(self.actor), net(self.critic)
            a.target_actor, a.target_critic1 = net(self.target_actor, True), net(self.target_critic, True)
            if twin:
                a.critic2, a.target_critic2 = net(self.critic2), net(self.target_critic2, True)
            a.out_s, a.out_a, a.out_r = self.s.data_ptr(), self.a.data_ptr(), self.r.data_ptr()
            a.out_d, a.out_s2 = self.d.data_ptr(), self.s2.data_ptr()
            a.noise_out = self.noise.data_ptr()
            a.dv1, a.dv2 = self.dv1.data_ptr(), self.dv2.data_ptr()
            a.loss_out = self.critic_loss.data_ptr()
            a.g_actor, a.g_critic1 = self.g_actor.data_ptr(), self.g_critic.data_ptr()
            if twin:
                a.g_critic2 = self.g_critic2.data_ptr()
            nbytes = _lib.load().xa_td3_update_workspace_bytes(B, S, A, H1, H2)
            self._fused_ws = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
            if '_fused_status' not in self.__dict__:
                self._fused_status = torch.zeros(1, dtype=torch.int32, device=self.device)
            a.workspace, a.workspace_bytes = self._fused_ws.data_ptr(), nbytes
            import os
            a.n_blocks = int(os.environ.get('XA_TD3_BLOCKS', '0')) or self._shared_blocks()
            a.status = self._fused_status.data_ptr()
            a.stage = 0
            # data parallel: the critics' losses are batch sums (Keras MSE + minimize), the
            # actor's a batch mean, so Adam takes the rank sum of the critics' gradients as
            # it is and the actor's over world (the executor path's _reduce_grad scales)
            a.critic_grad_scale = 1.0
            a.actor_grad_scale = kernels._f32(1.0 / self.world_size)
            fused = a
        self.__dict__['_fused'] = fused
        return fused

    # (bench) a list to collect (policy step, [(start, end) events of its launches]) of
    # eager fused gradient steps
    fused_timing = None

    def _fused_step(self, policy):
        a = self._fused
        a.actor_update = int(policy)
        self._fused_launch(a)
        self._fused_timing_row(policy)

    def _fused_launch(self, a):
        """One xa_td3_update launch (event-timed into self._launch_events when the bench
        collects fused_timing)."""
        ev = None
        if self.fused_timing is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        call('xa_td3_update', ctypes.byref(a), stream())
        if ev is not None:
            ev[1].record()
            self.__dict__.setdefault('_launch_events', []).append(ev)

    def _fused_timing_row(self, policy):
        """(bench) file this gradient step's launch events: (policy, [(start, end), ...])."""
        if self.fused_timing is not None:
            self.fused_timing.append((bool(policy), self.__dict__.pop('_launch_events', [])))

    def _fused_dp_step(self, policy):
        """One data-parallel gradient step on the fused kernel: stage 1 (critics' raw
        gradients) -> all-reduce of both critics' gradients (one flat buffer) -> stage 2
        (critics' Adam [+ Polyak]; on policy steps the actor's raw gradient through the
        updated critic 1) -> all-reduce of the actor's gradient -> stage 3 (actor Adam +
        Polyak). Three launches and one or two collectives instead of the executor's ~90
        launches (ddpg/agent.py:129-147 on the union of the ranks' batches)."""
        import torch.distributed as dist
        a = self._fused
        a.actor_update = int(policy)
        try:
            a.stage = 1
            self._fused_launch(a)
            dist.all_reduce(self._g_critics_flat())
            a.stage = 2
            self._fused_launch(a)
            if policy:
                dist.all_reduce(self.g_actor)
                a.stage = 3
                self._fused_launch(a)
        finally:
            a.stage = 0
        self._fused_timing_row(policy)

    def _g_critics_flat(self):
        """The buffer holding every critic's raw gradient (one all-reduce per step)."""
        return self.g_critic

    def fused_step_flops(self, policy=True):
        """Algorithmic FLOPs of one fused gradient step (2 M N K per GEMM): the forwards of
        the target actor, the critics and the target critics, the critics' weight and input
        gradients; on policy steps the actor forward, critic 1 forward on [s, pi(s)] and its
        input gradient, the actor's weight and input gradients."""
        B, S, A = self.batch_size, self.S, self.A
        H1, H2 = self.actor.layers[0].units, self.actor.layers[1].units
        C = S + A
        mm = lambda i, o: 2 * B * i * o  # noqa: E731
        mlp = lambda i, o: mm(i, H1) + mm(H1, H2) + mm(H2, o)  # noqa: E731
        nc = 2 if hasattr(self, 'critic2') else 1
        f = mlp(S, A) + 2 * nc * mlp(C, 1)                    # target actor, critics, targets
        f += nc * (mlp(C, 1) + mm(H1, H2) + mm(H2, 1))         # critics: dW + dX
        if policy:
            f += mlp(S, A) + mm(C, H1) + mm(H1, H2)              # actor, critic 1 on [s, pi]
            f += mm(H2, 1) + mm(H1, H2) + mm(H1, A)              # d(-mean Q) / d pi
            f += mlp(S, A) + mm(H1, H2) + mm(H2, A)              # actor: dW + dX
        return f

    def _critic_phase(self):
        self.replay.gather(self.replay.slots, self.s, self.a, self.r, self.d, self.s2)
        self.update_critic_weights()

    def _actor_phase(self):
        self.update_actor_weights()
        self.sync_target_models()

    def _run_phase(self, name, fn):
        """Eager once, then captured and replayed. Data-parallel steps stay eager (their
        gradient all-reduce is a torch collective)."""
        graphs = self.__dict__.setdefault('_graphs', {})
        warm = self.__dict__.setdefault('_warm', set())
        if not getattr(self, 'use_graph', True) or self.distributed:
            fn()
        elif name in graphs:
            graphs[name].replay()
        elif name in warm:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            graphs[name] = g
            g.replay()
        else:
            fn()
            warm.add(name)

    def _on_lr_change(self):
        self.__dict__['_graphs'] = {}  # the learning rates are baked into the launches
        self.__dict__['_warm'] = set()
        self.__dict__.pop('_fused', None)  # (and into the fused step's arguments)

    def _setup_step_stage(self):
        """The [done row | episode-return row] the captured env step writes: a mapped pinned
        host buffer the kernel stores into and the host reads after one event (default), or
        (XA_TD3_HOST_STAGE=0) a device buffer copied into the statistics rows and read back
        with a D2H copy each step."""
        import os
        self._stage_host = os.environ.get('XA_TD3_HOST_STAGE', '1') != '0' and \
            torch.device(self.device).type == 'cuda'
        if self._stage_host:
            self._stage = torch.zeros(2, self.n_envs, dtype=torch.float32).pin_memory()
            dp = ctypes.c_void_p()
            call('xa_host_device_pointer', ctypes.c_void_p(self._stage.data_ptr()), ctypes.byref(dp))
            self._stage_ptrs = (dp.value, dp.value + 4 * self.n_envs)
            self._stage_ev = torch.cuda.Event()
            self._stage_rows = 0
        else:
            self._stage = torch.zeros(2, self.n_envs, dtype=torch.float32, device=self.device)
            self._stage_ptrs = (self._stage[0].data_ptr(), self._stage[1].data_ptr())
        self._stage_done, self._stage_epret = self._stage[0], self._stage[1]
        # the env step's two launches launched directly, or (XA_TD3_STEP_GRAPH=1) replayed
        # from a hipGraph
        # (direct by default: C5 0.1069 -> 0.1047 ms per step, profiles/r06r_td3_step_graph_ab.txt)
        self._step_graph = os.environ.get('XA_TD3_STEP_GRAPH', '0') == '1'

    def _fold_step_row(self, d, e):
        """One step's episode statistics (host rows), env order as step_envs; the device
        status word is checked every _STATS_ROWS steps (as the statistics flush does)."""
        for i in np.nonzero(d)[0]:
            if self.history_checkpoint:
                self.update_history(float(e[i]))
            self.total_rewards.append(float(e[i]))
            self.games += 1
            self.done_envs += 1
        self._stage_rows += 1
        if self._stage_rows == self._STATS_ROWS:
            self._stage_rows = 0
            self._device_checks()

    def _step_phase(self):
        """get_step_actions + one xa_replay_env_step (ring append) writing the step's
        done / episode-return row into fixed staging rows (graph-capturable)."""
        actions = self.get_step_actions()
        a = self._step_args
        self.replay.fill_step_args(a, actions)
        a.out_dones, a.done_epret = self._stage_ptrs
        call('xa_replay_env_step', ctypes.byref(a), stream())

    def train_step(self):
        """ddpg/agent.py:149-166: step every env, then for each env that finished an
        episode run gradient_steps (or that env's episode length) gradient steps.
        The env phase is one hipGraph replay (a few small launches at batch n_envs);
        envs with a host-side pre_step (raw-frame Atari) stay on the eager path."""
        if hasattr(self.envs, 'pre_step'):
            actions = self.get_step_actions()
            row = self._st_row
            self._env_step(actions)
            self.steps += self.n_envs
            dones = self._host_row_dones(row)
        else:
            if not hasattr(self, '_stage'):
                self._setup_step_stage()
            if self._step_graph:
                self._run_phase('step', self._step_phase)
            else:
                self._step_phase()
            if self._stage_host:
                # the step's rows land in mapped host memory: one event wait, no copies
                self._stage_ev.record()
                self._stage_ev.synchronize()
                dones = self._stage[0].numpy().copy()
                self._fold_step_row(dones, self._stage[1].numpy())
            else:
                r = self._st_row
                self._st[r].copy_(self._stage)  # both rows in one copy
                self._st_row += 1
                if self._st_row == self._STATS_ROWS:
                    self._flush_offpolicy_stats()
                dones = self._stage_done.cpu().numpy()
            self.replay.appended()
            self.steps += self.n_envs
        if self.distributed:
            # every rank runs the gradient steps of the union of the ranks' finished
            # episodes, in global (rank-major) env order -- what one process stepping all
            # envs would run (ddpg/agent.py:157-166) -- so every rank issues the same
            # sequence of gradient all-reduces
            all_dones = self._all_gather_host(dones)
            all_steps = self._all_gather_host(self.episode_steps)
        else:
            all_dones, all_steps = dones, self.episode_steps
        for idx in np.nonzero(all_dones)[0]:
            steps = self.gradient_steps or all_steps[idx]
            self.update_weights(steps)
        self.episode_steps = (self.episode_steps + 1.0) * (1.0 - dones)

    def _host_row_dones(self, row):
        """The done flags of the step just taken (the reference returns them from the
        numpy step_envs; here one small synchronous copy of the step's stats row)."""
        return self._st_done[row].cpu().numpy()
