"""PPO with the xagents class surface (xagents/ppo/agent.py:7-225) on the fused
MI355X path.

train_step = one hipGraph replay of:
    xa_mlp_rollout (n_steps x [forward, sample, env step, store] + GAE)
    xa_ppo_update  (every optimizer step of the train step in ONE persistent launch:
                   shuffle, adv normalisation, fwd + clipped PPO loss + bwd, in-launch
                   gradient reduction, clip + Keras Adam; data parallel over the peer
                   path: the advantage sums and gradient slices are exchanged between the
                   ranks inside the same launch)
    chain (XA_PPO_UPDATE=chain, or data parallel without the peer path, i.e. RCCL only):
                   xa_ppo_minibatches (shuffle-gather, adv sums) -> [all_reduce]
                   ppo_epochs x mini_batches x:
                       xa_ac_grad (prologue: the previous step's clip + Adam; fwd + loss +
                       bwd -> partial rows) -> xa_grad_reduce -> [all_reduce]
                   -> xa_clip_adam
    xa_counter_bump (inside xa_ppo_update's last block on the persistent path)
Multi-GPU: every rank owns n_envs envs (weak scaling); the minibatch of a step is the
union of the ranks' local minibatches, advantage normalisation and the loss mean use
the global statistics/count, so the update equals a single-GPU update on the union.
"""
import os

import numpy as np
import torch

from xagents_amd import _lib, kernels
from xagents_amd._lib import XA_RETURNS_GAE, XaPpoUpdateArgs, XaShuffle
from xagents_amd.comm import PeerBlocks, ranks_per_device
from xagents_amd.a2c.agent import A2C


class PPO(A2C):
    """Proximal Policy Optimization Algorithms https://arxiv.org/abs/1707.06347"""

    loss_kind = kernels.XA_LOSS_PPO
    return_kind = XA_RETURNS_GAE

    def __init__(
        self,
        envs,
        model,
        lam=0.95,
        ppo_epochs=4,
        mini_batches=4,
        advantage_epsilon=1e-8,
        clip_norm=0.1,
        **kwargs,
    ):
        self.lam = lam
        self.ppo_epochs = ppo_epochs
        self.mini_batches = mini_batches
        self.advantage_epsilon = advantage_epsilon
        self.clip_norm = clip_norm
        n_envs = len(envs)
        n_steps = kwargs.get('n_steps', 1)
        self.batch_size = n_envs * n_steps
        self.mini_batch_size = self.batch_size // self.mini_batches
        assert (
            self.mini_batch_size > 0
        ), f'Invalid batch size to mini-batch size ratio {self.batch_size}: {self.mini_batches}'
        super(PPO, self).__init__(envs, model, **kwargs)

    def _setup_update(self):
        # a re-plan (a peer timeout dropping to the chain, a new permutation source) starts
        # with no statistics stored by an update launch: fold what earlier launches stored,
        # and only `_setup_fused_stats` (persistent mode) turns the fused slots back on
        # (a chain step must not fold the last persistent launch's slot again)
        if getattr(self, '_stats_fused', False):
            self._drain_episode_stats()
        self._stats_fused = False
        # optimizer step placement of the chain: 'prologue' (next minibatch's xa_ac_grad
        # recomputes it in every block) or 'kernel' (a standalone xa_clip_adam launch)
        self._opt_kernel = os.environ.get('XA_PPO_OPT', 'prologue') == 'kernel'
        B, MB, E = self.batch_size, self.mini_batch_size, self.ppo_epochs
        # range(0, B, MB) slicing: a ragged last minibatch when MB does not divide B
        # (xagents/ppo/agent.py:152)
        self.n_mb = (B + MB - 1) // MB
        dev = self.device
        self.shuffle = XaShuffle()
        perm = getattr(self, '_host_perm', None)
        self.shuffle.perm = None if perm is None else perm.data_ptr()
        self.shuffle.seed = self.rng_seed ^ 0x9E3779B97F4A7C15
        self.shuffle.rng_counter = self.rng_counter.data_ptr()
        self._tail_bump, self._tail_nobump = self._adam_tail(True), self._adam_tail(False)
        # one process: every optimizer step of the train step in ONE persistent launch
        # (xa_ppo_update); data parallel (a cross-rank exchange per step) or
        # XA_PPO_UPDATE=chain: the per-minibatch launch chain below
        # data parallel: the persistent launch exchanges the advantage sums and the
        # gradient slices between ranks itself, over IPC-mapped exchange blocks (needs the
        # peer path: ranks of one node); otherwise (RCCL only) the chain below
        self.update_mode = 'chain'
        dp_ok = not self.distributed or (getattr(self, 'peer', None) is not None and
                                         self.world_size <= 16)
        if os.environ.get('XA_PPO_UPDATE', 'persistent') == 'persistent' and dp_ok and \
                E * self.n_mb <= 128:
            obs_dim, A = self.model.obs_dim, self.n_actions
            G = kernels.ppo_update_blocks(obs_dim, A, MB)
            # (measurement knob: fewer workgroups, more tiles each -- fewer gradient rows to
            # exchange per optimizer step)
            g_cap = int(os.environ.get('XA_PPO_MAX_BLOCKS', '0'))
            if G > 0 and g_cap > 0:
                G = min(G, g_cap)
            if G > 0 and self.distributed:
                # every rank's workgroups must be resident together: ranks sharing a GPU
                # split its capacity
                # (collective: computed once, so a later re-setup stays rank-local)
                if getattr(self, '_ranks_share', None) is None:
                    self._ranks_share = ranks_per_device()
                share = self._ranks_share
                if share > 1:
                    G = min(G, kernels.ppo_update_blocks(obs_dim, A, 1 << 24) // share)
            if G > 0:
                self._setup_persistent(G)
                return
        self.device_status = None
        nb = kernels.ac_grad_blocks(MB)
        self.partials = torch.zeros(nb, self.model.n_params, dtype=torch.float32, device=dev)
        self.loss_partials = torch.zeros(nb, 4, dtype=torch.float32, device=dev)
        self.adv_stats = torch.zeros(kernels.adv_stats_size(B, MB, E), dtype=torch.float64,
                                     device=dev)
        # every minibatch of the train step materialised up front (ppo/agent.py:139-155)
        obs_dim = self.model.obs_dim
        f32 = dict(dtype=torch.float32, device=dev)
        self.mb_obs = torch.zeros(E * B, obs_dim, **f32)
        self.mb_act = torch.zeros(E * B, dtype=torch.int32, device=dev)
        self.mb_logp = torch.zeros(E * B, **f32)
        self.mb_val = torch.zeros(E * B, **f32)
        self.mb_ret = torch.zeros(E * B, **f32)
        mb = kernels.XaMinibatchArgs()
        mb.batch, mb.mb_size, mb.epochs, mb.obs_dim = B, MB, E, obs_dim
        mb.shuffle = self.shuffle
        mb.returns, mb.values = self.b_ret.data_ptr(), self.b_val.data_ptr()
        mb.obs, mb.actions, mb.old_logp = (self.b_obs.data_ptr(), self.b_act.data_ptr(),
                                           self.b_logp.data_ptr())
        mb.stats = self.adv_stats.data_ptr()
        mb.mb_obs, mb.mb_actions, mb.mb_old_logp = (self.mb_obs.data_ptr(),
                                                    self.mb_act.data_ptr(),
                                                    self.mb_logp.data_ptr())
        mb.mb_values, mb.mb_returns = self.mb_val.data_ptr(), self.mb_ret.data_ptr()
        self._mbargs = mb
        # minibatch k applies minibatch k-1's optimizer step in its prologue, reading
        # theta/m/v from slot (k-1)%2 and writing slot k%2 (slot 0 = the model's)
        opt = self.model.optimizer
        slots = [(self.model.theta, opt.m, opt.v), (self.theta_alt, self.m_alt, self.v_alt)]
        self._slots = slots
        adam = kernels.adam_struct(opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                                   clip_norm=self.grad_norm)
        self._gargs_list = []
        for e in range(E):
            for m in range(self.n_mb):
                k = len(self._gargs_list)
                g = self._grad_args(MB, nb, self.partials, self.loss_partials)
                g.epoch, g.mb_index = e, m
                g.gathered = 1
                g.obs, g.actions = self.mb_obs.data_ptr(), self.mb_act.data_ptr()
                g.old_logp, g.old_values = self.mb_logp.data_ptr(), self.mb_val.data_ptr()
                g.returns = self.mb_ret.data_ptr()
                count = min(MB, B - m * MB)
                g.adv_stats = self.adv_stats.data_ptr()
                g.adv_count = float(count * self.world_size)
                g.adv_in = None
                g.loss_scale = 1.0 / (count * self.world_size)
                src = slots[(k - 1) % 2] if k else slots[0]
                if self._opt_kernel:
                    src = slots[0]
                g.theta = src[0].data_ptr()
                if k and not self._opt_kernel:
                    dst = slots[k % 2]
                    g.pend_grad = self.grad.data_ptr()
                    g.pend_m, g.pend_v = src[1].data_ptr(), src[2].data_ptr()
                    g.theta_out, g.m_out, g.v_out = (x.data_ptr() for x in dst)
                    g.adam_step = opt.iterations.data_ptr()
                    g.adam = adam
                self._gargs_list.append(g)
        self._final_src = slots[0 if self._opt_kernel else (len(self._gargs_list) - 1) % 2]

    def _setup_persistent(self, n_blocks):
        """Arguments of the persistent update (xa_ppo_update): the rollout buffers in place,
        theta / Adam moments / iterations of the model in place, a workspace for the
        in-launch gradient exchange and a device status word (checked with the episode
        statistics)."""
        B, MB, E = self.batch_size, self.mini_batch_size, self.ppo_epochs
        dev, opt = self.device, self.model.optimizer
        obs_dim, A = self.model.obs_dim, self.n_actions
        nbytes = kernels.ppo_update_workspace_bytes(obs_dim, A, B, MB, E, n_blocks)
        # zeroed once: a re-setup with the same shapes (a learning-rate change) keeps the
        # workspace and with it the launch generation, which data-parallel ranks must share
        key = (B, MB, E, n_blocks)
        if getattr(self, 'update_ws', None) is None or getattr(self, '_ws_key', None) != key:
            self.update_ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
            self._ws_key = key
            self._upd_launches = 0  # the launch number the zeroed workspace starts from
        # the status word rides in the packed episode-statistics buffer (one D2H copy)
        self.device_status = self._stats_status
        self.device_status.zero_()
        u = XaPpoUpdateArgs()
        u.obs_dim, u.n_actions = obs_dim, A
        u.batch, u.mb_size, u.epochs = B, MB, E
        u.shuffle = self.shuffle
        u.obs, u.actions = self.b_obs.data_ptr(), self.b_act.data_ptr()
        u.old_logp, u.old_values = self.b_logp.data_ptr(), self.b_val.data_ptr()
        u.returns = self.b_ret.data_ptr()
        u.clip_norm, u.entropy_coef = float(self.clip_norm), float(self.entropy_coef)
        u.value_coef, u.adv_eps = float(self.value_loss_coef), float(self.advantage_epsilon)
        u.theta, u.adam_m, u.adam_v = (self.model.theta.data_ptr(), opt.m.data_ptr(),
                                       opt.v.data_ptr())
        u.adam_step = opt.iterations.data_ptr()
        u.adam = kernels.adam_struct(opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                                     clip_norm=self.grad_norm)
        u.workspace, u.workspace_bytes = self.update_ws.data_ptr(), nbytes
        u.loss_out = u.grad_out = None
        u.status = self.device_status.data_ptr()
        u.n_blocks = n_blocks
        # the Philox counter bump that ends a train step runs in the launch's last block
        u.bump_counter = int(bool(self.shuffle.rng_counter))
        u.dp_world, u.dp_rank = 1, 0
        # XCD-local placement of small grids (xa_ppo_update): automatic in one process; data
        # parallel only when every rank owns its GPU (ranks sharing one could strand each
        # other's XCD elections). XA_PPO_PLACE=spread|local overrides.
        # The election needs G free CU slots on ONE XCD (at G = 32 with one block per CU:
        # all 8 x 32 CUs idle), so it assumes the update owns the GPU while it runs: a
        # kernel overlapping it on another stream could hold a CU on every XCD and stall
        # every spinning block until the abort. The opt-in side-stream statistics copy
        # (XA_STATS_SIDE_STREAM=1) can overlap the update, so it forces the spread grid.
        place = os.environ.get('XA_PPO_PLACE', 'auto')
        if getattr(self, 'stats_side_stream', False) and place != 'local':
            place = 'spread'
        if place == 'spread':
            u.placement = _lib.XA_PPO_PLACE_SPREAD
        elif place == 'local' or (self.distributed and getattr(self, '_ranks_share', 1) == 1):
            u.placement = _lib.XA_PPO_PLACE_LOCAL
        else:
            u.placement = _lib.XA_PPO_PLACE_AUTO
        if self.distributed:
            if getattr(self, 'dp_blocks', None) is None or self._dp_blocks_key != (B, MB, E,
                                                                                  n_blocks):
                nbytes = _lib.load().xa_ppo_update_dp_block_bytes(obs_dim, A, B, MB, E,
                                                                  n_blocks, self.world_size)
                self.dp_blocks = PeerBlocks(nbytes)
                self._dp_blocks_key = (B, MB, E, n_blocks)
            u.dp_world, u.dp_rank = self.world_size, self.rank
            for r, ptr in enumerate(self.dp_blocks.pointers):
                u.dp_blocks[r] = ptr
        self._setup_fused_stats(u)
        self._uargs = u
        self.update_mode = 'persistent'
        self.update_blocks = n_blocks

    def _setup_fused_stats(self, u):
        """The train step's episode statistics (done flags, running returns, the status word:
        the packed buffer a2c/agent.py lays out) leave the device inside the update launch,
        into XA_PPO_STATS_SLOTS mapped pinned host slots chosen by the launch number -- no
        xa_copy_to_host launch per train step, and several train steps per graph replay. Off with XA_STATS_IN_UPDATE=0 or the opt-in
        side-stream copy."""
        import ctypes
        from xagents_amd._lib import call
        u.stats_words = 0
        self._stats_fused = False
        if os.environ.get('XA_STATS_IN_UPDATE', '1') == '0' or \
                getattr(self, 'stats_side_stream', False):
            return
        nd, sd, oe, se, os_ = self._stats_views
        nw = os_ + 1  # through the status word
        if getattr(self, '_fused_host', None) is None or self._fused_host[0].numel() != nw + 1:
            self._fused_host = [torch.zeros(nw + 1, dtype=torch.float32).pin_memory()
                                for _ in range(_lib.XA_PPO_STATS_SLOTS)]
            self._fused_done = [h[:nd].view(sd) for h in self._fused_host]
            self._fused_epret = [h[oe:oe + se[0] * se[1]].view(se) for h in self._fused_host]
            self._fused_host_status = [h[os_:os_ + 1].view(torch.int32)
                                       for h in self._fused_host]
            self._fused_gen = [h[nw:nw + 1].view(torch.int32) for h in self._fused_host]
            self._fused_dev = []
            for h in self._fused_host:
                dp = ctypes.c_void_p()
                call('xa_host_device_pointer', ctypes.c_void_p(h.data_ptr()), ctypes.byref(dp))
                self._fused_dev.append(dp.value)
        u.stats_src = self._stats_pack.data_ptr()
        for i, dp in enumerate(self._fused_dev):
            u.stats_dst[i] = dp
        u.stats_words = nw
        self._stats_fused = True

    def set_minibatch_permutation(self, perm):
        """Parity mode: the fused update takes every epoch's shuffle from `perm`, an
        [ppo_epochs, batch] int32 device tensor of permutations of the env-major batch
        (what tf.random.shuffle produced in the reference, ppo/agent.py:149-151), instead
        of the device Feistel shuffle; None restores the device shuffle. The tensor is read
        at every train step (update it in place for a new draw)."""
        if perm is not None:
            assert perm.dtype == torch.int32 and perm.is_contiguous() and \
                tuple(perm.shape) == (self.ppo_epochs, self.batch_size), \
                f'Expected an int32 [{self.ppo_epochs}, {self.batch_size}] permutation tensor'
        self._host_perm = perm
        if not self.executor_path:
            self._setup_update()
        self._graph = None

    def _update_impl(self):
        self._update()
        if not (self.update_mode == 'persistent' and self._uargs.bump_counter):
            kernels.counter_bump(self.rng_counter)

    def _timed_kernels(self):
        if self.update_mode == 'persistent':
            return {'rollout': 1, 'ppo_update': 1}
        return {'rollout': 1, 'ac_grad': len(self._gargs_list)}

    def _update(self):
        if self.update_mode == 'persistent':
            self._kernel_event('ppo_update', 0, 0)
            kernels.ppo_update(self._uargs)
            self._kernel_event('ppo_update', 0, 1)
            if not torch.cuda.is_current_stream_capturing():
                self._upd_launches += 1  # (a captured launch counts at its replays)
            return
        kernels.minibatches(self._mbargs)
        self._all_reduce(self.adv_stats)
        last = len(self._gargs_list) - 1
        for i, g in enumerate(self._gargs_list):
            self._kernel_event('ac_grad', i, 0)
            kernels.ac_grad(g)
            self._kernel_event('ac_grad', i, 1)
            self._reduce_gradients(self.partials)
            if self._opt_kernel and i < last:
                self._optimizer_step()  # standalone clip + Adam launch
        self._optimizer_step(self._final_src)

    # ---- reference-level pieces --------------------------------------------
    def calculate_returns(self, rewards, dones, values=None, selected_critic_logits=None,
                          selected_importance=None):
        """GAE from time-major rewards [T,N], dones [T+1,N], values [T,N]
        (xagents/ppo/agent.py:48-94); bootstraps on V(get_states())."""
        next_values = self.get_model_outputs(self.get_states(), self.output_models)[2]
        f = lambda x: torch.as_tensor(x, dtype=torch.float32,  # noqa: E731
                                      device=self.device).reshape(x.shape[0], -1).t().contiguous()
        ret = kernels.gae(f(rewards), f(values), f(dones), next_values.contiguous(), self.gamma,
                          self.lam)
        return ret.t()

    def get_batch(self):
        """Fused rollout + GAE; returns env-major flat [states, actions, returns, values,
        log_probs] exactly as concat_step_batches lays them out
        (xagents/ppo/agent.py:193-213, xagents/base.py:549-564)."""
        a = self._rargs
        self._sync_stats_copy()
        kernels.rollout(a)
        kernels.counter_bump(self.rng_counter)
        self.steps += self.n_envs * self.n_steps
        self._queue_episode_stats(self.b_done, self.b_epret)
        B = self.batch_size
        return [self.b_obs.reshape(B, -1), self.b_act.reshape(B).float(),
                self.b_ret.reshape(B), self.b_val.reshape(B), self.b_logp.reshape(B)]

    def get_mini_batches(self, *args):
        """Per epoch: reshuffle, then contiguous minibatch slices
        (xagents/ppo/agent.py:139-155)."""
        mini_batches = []
        indices = torch.arange(self.batch_size, device=self.device)
        for _ in range(self.ppo_epochs):
            indices = indices[torch.randperm(self.batch_size, device=self.device)]
            for i in range(0, self.batch_size, self.mini_batch_size):
                batch_indices = indices[i: i + self.mini_batch_size]
                mini_batches.append([item[batch_indices] for item in args])
        return mini_batches

    def update_gradients(self, states, actions, old_values, returns, old_log_probs, advantages):
        """One clipped-PPO Adam step on a given minibatch (xagents/ppo/agent.py:96-137)."""
        n = states.shape[0]
        dev = self.device
        c = lambda x, dt=torch.float32: torch.as_tensor(  # noqa: E731
            x, device=dev).to(dt).reshape(n, -1).squeeze(-1).contiguous()
        obs = torch.as_tensor(states, device=dev).float().reshape(n, -1).contiguous()
        act, oldv, ret = c(actions, torch.int32), c(old_values), c(returns)
        oldlp, adv = c(old_log_probs), c(advantages)
        nb = kernels.ac_grad_blocks(n)
        partials = torch.zeros(nb, self.model.n_params, dtype=torch.float32, device=dev)
        lossp = torch.zeros(nb, 4, dtype=torch.float32, device=dev)
        g = self._grad_args(n, nb, partials, lossp)
        g.batch = n
        g.epoch = g.mb_index = 0
        ident = torch.arange(n, dtype=torch.int32, device=dev)
        sh = XaShuffle()
        sh.perm, sh.seed, sh.rng_counter = ident.data_ptr(), 0, None
        g.shuffle = sh
        g.obs, g.actions, g.old_logp = obs.data_ptr(), act.data_ptr(), oldlp.data_ptr()
        g.old_values, g.returns, g.adv_in = oldv.data_ptr(), ret.data_ptr(), adv.data_ptr()
        g.adv_stats, g.adv_count = None, 0.0
        g.loss_scale = 1.0 / (n * self.world_size)
        kernels.ac_grad(g)
        self._apply_gradients(partials)
        lp = lossp.sum(0)
        return {'pg_loss': lp[0] / lp[3], 'value_loss': 0.5 * lp[1] / lp[3],
                'entropy': lp[2] / lp[3]}

    def run_ppo_epochs(self, states, actions, returns, old_values, old_log_probs):
        """Minibatch loop with per-minibatch advantage normalisation
        (xagents/ppo/agent.py:157-191)."""
        for states_mb, actions_mb, returns_mb, old_values_mb, old_log_probs_mb in (
                self.get_mini_batches(states, actions, returns, old_values, old_log_probs)):
            adv = returns_mb - old_values_mb
            adv = (adv - adv.mean()) / (adv.std(unbiased=False) + self.advantage_epsilon)
            self.update_gradients(states_mb, actions_mb, old_values_mb, returns_mb,
                                  old_log_probs_mb, adv)

    def train_step(self):
        hooks = ('get_batch', 'calculate_returns', 'update_gradients', 'run_ppo_epochs',
                 'get_mini_batches')
        if any(getattr(type(self), h) is not getattr(PPO, h) for h in hooks):
            # a subclass overrode a reference hook: compose the pieces instead of
            # the fused graph so the override is honoured
            self.run_ppo_epochs(*self.get_batch())
            return
        self.fused_train_step()
