"""A2C with the xagents class surface (xagents/a2c/agent.py:9-218) on the fused
MI355X path.

train_step = one hipGraph replay of:
    xa_mlp_rollout (n_steps x [forward, sample, env step, store] + n-step returns)
    xa_ac_grad (A2C loss, full batch) -> xa_grad_reduce -> [RCCL all_reduce]
    -> xa_clip_adam (tf.clip_by_global_norm + Keras Adam) -> xa_counter_bump
"""
import ctypes
import os
import warnings

import numpy as np
import torch
import torch.distributed as dist

from xagents_amd import kernels
from xagents_amd.comm import maybe_peer_all_reduce
from xagents_amd._lib import (XA_RETURNS_GAE, XA_RETURNS_NONE, XA_RETURNS_NSTEP,
                              XaAcGradArgs, XaRolloutArgs, XaShuffle)
from xagents_amd.base import OnPolicy
from xagents_amd.envs import Discrete
from xagents_amd.onpolicy_executor import ExecutorActorCritic


class A2C(ExecutorActorCritic, OnPolicy):
    """Asynchronous Methods for Deep Reinforcement Learning
    https://arxiv.org/abs/1602.01783"""

    loss_kind = kernels.XA_LOSS_A2C
    return_kind = XA_RETURNS_NSTEP

    def __init__(
        self,
        envs,
        model,
        entropy_coef=0.01,
        value_loss_coef=0.5,
        grad_norm=0.5,
        use_graph=True,
        data_parallel=None,
        **kwargs,
    ):
        # data_parallel: None = data parallel over the default process group when one is
        # initialised; False = a single-process agent even inside a process group
        self.data_parallel = data_parallel
        super(A2C, self).__init__(envs, model, **kwargs)
        self.entropy_coef = entropy_coef
        self.value_loss_coef = value_loss_coef
        self.grad_norm = grad_norm
        # the reference counts Keras' InputLayer in model.layers
        assert (
            len(model.layers) + 1 > 2
        ), f'Expected a model that has at least 3 layers, got {len(model.layers) + 1}'
        activations = [layer.activation for layer in model.layers[-2:]]
        # A2C.get_distribution (a2c/agent.py:54-63): Categorical(probs) after a softmax
        # output layer (its log-prob is the log-softmax of the layer's pre-activation,
        # which the executor returns), Categorical(logits) otherwise, and
        # MultivariateNormalDiag(loc = actor output) for Box action spaces
        self.output_is_softmax = 'softmax' in activations
        self.distribution_type = (
            'Categorical' if isinstance(self.envs[0].action_space, Discrete)
            else 'MultivariateNormalDiag')
        self.use_graph = use_graph
        self._graph = None
        # the Categorical actor-critic MLP of the fused kernels' shapes runs fused; any other
        # .cfg actor-critic (the CNN, a softmax actor, a Gaussian policy, other sizes) on the
        # layer executor (xagents_amd/onpolicy_executor.py)
        self.executor_path = not (
            getattr(model, 'fused_kind', None) == 'actor_critic_mlp'
            and self.distribution_type == 'Categorical'
            and (getattr(model, 'obs_dim', None), self.n_actions) in kernels.FUSED_MLP_SHAPES)
        if self.executor_path:
            self._detect_distributed()
            self._setup_executor_path()
        else:
            self._setup_device()

    # ---- device state ------------------------------------------------------
    def _detect_distributed(self):
        dp = getattr(self, 'data_parallel', None)
        self.distributed = (dist.is_available() and dist.is_initialized() and dp is not False)
        self.world_size = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0

    def _setup_device(self):
        self._detect_distributed()
        N, T, obs = self.n_envs, self.n_steps, self.model.obs_dim
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.b_obs = torch.zeros(N, T, obs, **f32)
        self.b_act = torch.zeros(N, T, dtype=torch.int32, device=dev)
        self.b_logp = torch.zeros(N, T, **f32)
        self.b_val = torch.zeros(N, T, **f32)
        self.b_ent = torch.zeros(N, T, **f32)
        self.b_rew = torch.zeros(N, T, **f32)
        # done flags, running episode returns and a device status word in ONE buffer, so
        # the per-step episode statistics leave the device in one D2H copy
        al = lambda x: (x + 63) // 64 * 64  # noqa: E731  (256-B aligned views)
        o_ep = al(N * (T + 1))
        o_st = o_ep + al(N * T)
        self._stats_pack = torch.zeros(o_st + 64, **f32)
        self.b_done = self._stats_pack[:N * (T + 1)].view(N, T + 1)
        self.b_epret = self._stats_pack[o_ep:o_ep + N * T].view(N, T)
        self._stats_status = self._stats_pack[o_st:o_st + 1].view(torch.int32)
        self._stats_views = (N * (T + 1), (N, T + 1), o_ep, (N, T), o_st)
        self.b_ret = torch.zeros(N, T, **f32)
        self.next_val = torch.zeros(N, **f32)
        self.rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self._rollout_ev = None
        # Episode statistics leave the device after every train step. On the launch stream
        # (default) they cost ~4 us per copy; on a side stream behind the rollout they
        # overlap the update (C2: 0.43 -> 0.41 ms per step), but the first copies of a
        # process's side stream stall the host ~7 ms twice at a random early step
        # (tools/diag_bench_steps.py), which a 20-step timed loop cannot absorb.
        self.stats_side_stream = os.environ.get('XA_STATS_SIDE_STREAM', '0') == '1'
        seed = self.seed if self.seed is not None else int(np.random.SeedSequence().entropy % 2**63)
        self.rng_seed = (int(seed) * 1000003 + self.rank * 7919 + 17) % 2**64
        P = self.model.n_params
        self.grad = torch.zeros(P, **f32)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        # last-block election counter of the fused optimizer tails (self-resetting)
        self.arrivals = torch.zeros(1, dtype=torch.int32, device=dev)
        # second (ping-pong) slot of theta / Adam moments for PPO's prologue optimizer step
        self.theta_alt = torch.zeros(P, **f32)
        self.m_alt = torch.zeros(P, **f32)
        self.v_alt = torch.zeros(P, **f32)
        if self.distributed:
            dist.broadcast(self.model.theta, 0)
        # small exchanges (gradient, advantage sums) over IPC peer blocks; RCCL otherwise
        self.peer = maybe_peer_all_reduce(self.world_size)
        a = XaRolloutArgs()
        a.n_envs, a.n_steps, a.obs_dim, a.n_actions = N, T, obs, self.n_actions
        a.theta = self.model.theta.data_ptr()
        self.envs.fill_rollout_args(a)
        a.uniforms = None
        a.seed = self.rng_seed
        a.rng_counter = self.rng_counter.data_ptr()
        a.obs_out, a.act_out = self.b_obs.data_ptr(), self.b_act.data_ptr()
        a.logp_out, a.val_out = self.b_logp.data_ptr(), self.b_val.data_ptr()
        a.ent_out, a.rew_out = self.b_ent.data_ptr(), self.b_rew.data_ptr()
        a.done_out, a.epret_out = self.b_done.data_ptr(), self.b_epret.data_ptr()
        a.next_val, a.ret_out = self.next_val.data_ptr(), self.b_ret.data_ptr()
        a.return_kind = self.return_kind
        a.gamma = float(np.float32(self.gamma))
        a.gamma_lam = kernels.gamma_lam_f32(self.gamma, getattr(self, 'lam', 0.0))
        self._rargs = a
        self._setup_update()

    def set_rollout_uniforms(self, uniforms):
        """Parity mode: the fused rollout samples every action by inverse CDF from these
        [n_envs, n_steps] f32 device uniforms (held, not copied) instead of the Philox
        stream; None restores Philox. On the layer-executor path (Categorical actors) the
        uniforms are copied time-major once, so each step's xa_categorical reads a row."""
        if uniforms is not None:
            assert uniforms.dtype == torch.float32 and uniforms.is_contiguous() and \
                tuple(uniforms.shape) == (self.n_envs, self.n_steps), \
                f'Expected f32 [{self.n_envs}, {self.n_steps}] uniforms'
        if self.executor_path:
            if self.gaussian:
                raise NotImplementedError('rollout uniforms drive Categorical sampling only')
            self._exec_uniforms = None if uniforms is None else uniforms.t().contiguous()
            return
        self._rollout_uniforms = uniforms
        self._rargs.uniforms = None if uniforms is None else uniforms.data_ptr()
        self._graph = None

    def _grad_args(self, mb_size, n_blocks, partials, loss_partials):
        g = XaAcGradArgs()
        g.obs_dim, g.n_actions = self.model.obs_dim, self.n_actions
        g.loss_kind = self.loss_kind
        g.theta = self.model.theta.data_ptr()
        g.batch = self.n_envs * self.n_steps
        g.mb_size = mb_size
        g.obs, g.actions = self.b_obs.data_ptr(), self.b_act.data_ptr()
        g.old_logp, g.old_values = self.b_logp.data_ptr(), self.b_val.data_ptr()
        g.returns = self.b_ret.data_ptr()
        g.clip_norm = float(getattr(self, 'clip_norm', 0.0))
        g.entropy_coef = float(self.entropy_coef)
        g.value_coef = float(self.value_loss_coef)
        g.adv_eps = float(getattr(self, 'advantage_epsilon', 0.0))
        g.n_blocks = n_blocks
        g.partials = partials.data_ptr()
        g.loss_partials = loss_partials.data_ptr()
        return g

    def _setup_update(self):
        self._tail_bump, self._tail_nobump = self._adam_tail(True), self._adam_tail(False)
        B = self.n_envs * self.n_steps
        nb = kernels.ac_grad_blocks(B)
        self.partials = torch.zeros(nb, self.model.n_params, dtype=torch.float32,
                                    device=self.device)
        self.loss_partials = torch.zeros(nb, 4, dtype=torch.float32, device=self.device)
        g = self._grad_args(B, nb, self.partials, self.loss_partials)
        g.epoch = g.mb_index = 0
        g.loss_scale = 1.0 / (B * self.world_size)
        self._gargs = g

    # ---- the fused train step ----------------------------------------------
    def _all_reduce(self, t):
        if not self.distributed:
            return
        peer = getattr(self, 'peer', None)
        if peer is not None and peer.fits(t):
            peer.all_reduce(t)
        else:
            dist.all_reduce(t)

    def check_peer_all_reduce(self):
        """After warm-up: if any rank's peer exchange timed out, every rank drops it,
        re-broadcasts rank 0's parameters and re-captures the step on RCCL.
        Returns the transport in use."""
        peer = getattr(self, 'peer', None)
        if peer is None:
            return 'rccl' if self.distributed else 'none'
        if peer.healthy_everywhere():
            return 'peer-ipc'
        warnings.warn('peer all-reduce timed out on some rank; falling back to RCCL')
        self.peer = None
        opt = self.model.optimizer
        for t in (self.model.theta, opt.m, opt.v, opt.iterations):
            dist.broadcast(t, 0)
        self._graph = None
        if not self.executor_path:
            # PPO's persistent update exchanges through IPC blocks too: re-plan the update
            # without the peer path (the per-minibatch chain over RCCL)
            self._setup_update()
        return 'rccl'

    def _adam_tail(self, bump):
        opt = self.model.optimizer
        return kernels.adam_tail(self.model.theta, opt.m, opt.v, opt.iterations, self.arrivals,
                                 opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                                 clip_norm=self.grad_norm, bump=bump)

    def _reduce_gradients(self, partials):
        """Partial rows -> gradient (Adam step += 1) -> [all-reduce]."""
        kernels.grad_reduce(partials, self.grad, self.model.optimizer.iterations)
        self._all_reduce(self.grad)

    def _optimizer_step(self, src=None):
        """Clip + Keras Adam of self.grad applied to slot `src` = (theta, m, v), result
        in the canonical slot (model.theta, optimizer.m, optimizer.v)."""
        opt = self.model.optimizer
        src = src or (self.model.theta, opt.m, opt.v)
        kernels.clip_adam(*src, self.grad, opt.iterations, opt.learning_rate, opt.beta_1,
                          opt.beta_2, opt.epsilon, clip_norm=self.grad_norm,
                          workspace=self.adam_ws, out=(self.model.theta, opt.m, opt.v))

    def _apply_gradients(self, partials):
        """Partial rows -> gradient -> [all-reduce] -> clip + Keras Adam (t += 1) for one
        optimizer step (A2C, PPO.update_gradients). One launch on one GPU (the reduce's
        last block runs the optimizer); with data parallelism the peer exchange carries
        the optimizer tail, RCCL is followed by xa_clip_adam."""
        opt = self.model.optimizer
        if not self.distributed:
            kernels.grad_reduce_adam(partials, self.grad, self._tail_bump)
            return
        kernels.grad_reduce(partials, self.grad, opt.iterations)
        peer = getattr(self, 'peer', None)
        if peer is not None and peer.fits(self.grad):
            peer.all_reduce(self.grad, tail=self._tail_nobump)
        else:
            dist.all_reduce(self.grad)
            self._optimizer_step()

    def _update(self):
        self._kernel_event('ac_grad', 0, 0)
        kernels.ac_grad(self._gargs)
        self._kernel_event('ac_grad', 0, 1)
        self._apply_gradients(self.partials)

    def _rollout_impl(self):
        self._kernel_event('rollout', 0, 0)
        kernels.rollout(self._rargs)
        self._kernel_event('rollout', 0, 1)

    # ---- per-kernel timing (bench): HIP event pairs around the rollout launch and
    # every xa_ac_grad launch of an eagerly launched train step (ROCm torch refuses
    # external events inside graph capture, so captured steps record none) --------
    def timed_train_step(self):
        """One eager train step with events around the hot launches; returns
        {name: [ms per launch]} for _timed_kernels() (synchronizes)."""
        ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        self._kernel_events = {name: [(ev(), ev()) for _ in range(n)]
                               for name, n in self._timed_kernels().items()}
        try:
            # park the stream on a spin kernel so the host enqueues the whole step behind
            # it: the event pairs then bracket GPU execution, not host launch gaps
            self._sync_stats_copy()
            torch.cuda._sleep(20_000_000)
            self._step_impl()
            self.steps += self.n_envs * self.n_steps
            self._queue_episode_stats(self.b_done, self.b_epret)
            torch.cuda.synchronize()
            return {k: [a.elapsed_time(b) for a, b in v] for k, v in self._kernel_events.items()}
        finally:
            self._kernel_events = None

    def _timed_kernels(self):
        """Event-bracketed launches of one eager train step: name -> count."""
        return {'rollout': 1, 'ac_grad': 1}

    def _kernel_event(self, name, i, j):
        evs = getattr(self, '_kernel_events', None)
        if evs is not None:
            evs[name][i][j].record()

    def _update_impl(self):
        self._update()
        kernels.counter_bump(self.rng_counter)

    def _step_impl(self):
        self._rollout_impl()
        self._update_impl()

    def _capture(self):
        """Capture the rollout, the update, and the two back to back as hipGraphs (a
        train step replays the combined graph; the per-phase graphs serve the event-timed
        pass, so the update can be timed on its own). Data-parallel steps are
        captured when every exchange goes through the peer kernel or through RCCL (the
        nccl backend's all-reduce is graph-capturable: tests/test_gpu_rccl_capture.py);
        a gloo collective cannot be captured, so gloo steps without the peer path run
        eagerly (as does any step whose capture raises). A multi-rank RCCL collective
        replayed from a hipGraph has only been tested at world size 1, so RCCL steps of
        W > 1 ranks stay eager unless XA_CAPTURE_RCCL=1; and in data-parallel runs the
        capture-or-eager outcome is agreed collectively (every rank captures, then a MIN
        all-reduce of the success flags), so no rank replays a graph while another runs
        the step eagerly."""
        rccl_only = self.distributed and getattr(self, 'peer', None) is None
        if rccl_only and (dist.get_backend() != 'nccl' or (
                self.world_size > 1 and os.environ.get('XA_CAPTURE_RCCL', '0') != '1')):
            self.use_graph = False
            self._graph = None
            return
        ok = True
        try:
            graphs = []
            # rollout, update, and both back to back: a train step replays the third (one
            # graph launch per train step), the per-phase event pass the first two; with the
            # persistent update (every exchange and the statistics copy inside its launch)
            # further graphs hold graph_steps() train steps back to back, then half as
            # many, ... down to 2 (fused_train_steps: one replay per group of steps, the
            # largest group that fits what is left)
            seqs = [(self._rollout_impl,), (self._update_impl,),
                    (self._rollout_impl, self._update_impl)]
            S = self.graph_steps()
            sizes, s = [], S
            while s > 1:
                sizes.append(s)
                seqs.append((self._rollout_impl, self._update_impl) * s)
                s //= 2
            self._graph_S = S
            self._graph_sizes = sizes
            for fns in seqs:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for fn in fns:
                        fn()
                graphs.append(g)
            self._graph = graphs
        except Exception as exc:  # collectives that refuse capture -> eager launches
            warnings.warn(f'hipGraph capture failed ({exc}); running the train step eagerly')
            ok = False
        if self.distributed:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            if dist.get_backend() == 'nccl':
                flag = flag.to(self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(int(flag.item()))
            if not ok and self._graph is not None:
                warnings.warn('hipGraph capture failed on another rank; running eagerly')
        if not ok:
            self.use_graph = False
            self._graph = None

    def _on_lr_change(self):
        self._graph = None
        if not self.executor_path:
            self._setup_update()  # the learning rate is baked into the optimizer tails

    def fused_train_step(self, events=None):
        """One train step. `events` = (start, mid, end) torch.cuda.Events recorded
        around the rollout and the update on the replay stream (bench timing)."""
        rec = (lambda i: events[i].record()) if events else (lambda i: None)  # noqa: E731
        if self.executor_path:
            rec(0)
            self._executor_rollout()
            rec(1)
            self._executor_update()
            rec(2)
            self.steps += self.n_envs * self.n_steps
            self._queue_episode_stats(self.b_done, self.b_epret)
            return
        self._sync_stats_copy()
        if self._rollout_ev is None and self.stats_side_stream:
            self._rollout_ev = torch.cuda.Event()
        if self.use_graph and self._graph is not None and not events and \
                not self.stats_side_stream:
            self._graph[2].replay()
            self._count_update_replay()
        elif self.use_graph and self._graph is not None:
            rec(0)
            self._graph[0].replay()
            if self.stats_side_stream:
                self._rollout_ev.record()
            rec(1)
            self._graph[1].replay()
            self._count_update_replay()
            rec(2)
        else:
            rec(0)
            self._rollout_impl()
            if self.stats_side_stream:
                self._rollout_ev.record()
            rec(1)
            self._update_impl()
            rec(2)
            if self.use_graph:
                self._capture()
        self.steps += self.n_envs * self.n_steps
        # opt-in: the statistics copy overlaps the update (side stream behind the rollout)
        self._queue_episode_stats(self.b_done, self.b_epret,
                                  after=self._rollout_ev if self.stats_side_stream else None)
        self._maybe_check_peer()

    def graph_steps(self):
        """Train steps per replay of the multi-step graph (XA_GRAPH_STEPS, at most
        BaseAgent.FUSED_GROUP_MAX; 1 = none): only with the persistent update, whose launch
        stores each step's episode statistics into a host slot of its own."""
        if self.executor_path or getattr(self, 'update_mode', None) != 'persistent' or \
                not getattr(self, '_stats_fused', False) or self.stats_side_stream:
            return 1
        # default 8 steps per replay (16 envs 0.1453 -> 0.1435 ms per step,
        # profiles/r06t_graph_steps_ab.txt; 256 envs 0.2553 -> 0.2515 ms once the host's
        # statistics fold was vectorised, profiles/r06zh_c2_graph_steps_ab.txt)
        return max(1, min(int(os.environ.get('XA_GRAPH_STEPS', 8)), self.FUSED_GROUP_MAX))

    def fused_train_steps(self, n):
        """n train steps: groups of graph_steps() steps as one replay of the multi-step
        hipGraph (the kernel sequence of the single-step replays back to back, so the same
        arithmetic; one graph launch and one completion event per group), the rest one
        step at a time. The host bookkeeping of every step (step count, statistics fold,
        peer health check) runs after its group."""
        while n > 0:
            g = self._graph if self.use_graph else None
            sizes = getattr(self, '_graph_sizes', []) if g is not None and len(g) > 3 else []
            j = next((j for j, s in enumerate(sizes) if s <= n), None)
            if j is None:
                self.fused_train_step()
                n -= 1
                continue
            S = sizes[j]
            self._sync_stats_copy()
            g[3 + j].replay()
            for i in range(S):
                self._count_update_replay()
                self.steps += self.n_envs * self.n_steps
                self._queue_episode_stats(self.b_done, self.b_epret, group_end=i == S - 1)
                self._maybe_check_peer()
            n -= S

    def _count_update_replay(self):
        """A graph replay that ran the persistent update: one more launch number (the
        in-launch statistics slots, PPO._setup_fused_stats)."""
        if getattr(self, '_stats_fused', False) and self.update_mode == 'persistent':
            self._upd_launches += 1

    # every rank reaches the same train-step count, so this collective check lines up
    PEER_CHECK_STEPS = 64

    def _maybe_check_peer(self):
        """A timed-out peer exchange leaves a sticky error after which every exchange
        returns local values: check every PEER_CHECK_STEPS train steps (a collective on a
        schedule identical on all ranks) and, if any rank failed, fall back to RCCL after
        re-broadcasting rank 0's parameters and optimizer state (check_peer_all_reduce)."""
        if not self.distributed or getattr(self, 'peer', None) is None:
            return
        self._fused_steps = getattr(self, '_fused_steps', 0) + 1
        every = int(os.environ.get('XA_PEER_CHECK_STEPS', self.PEER_CHECK_STEPS))
        if self._fused_steps % every == 0:
            self.check_peer_all_reduce()

    def np_train_step(self):
        """Batching and returns (xagents/a2c/agent.py:173-186): get_batch ->
        calculate_returns -> concat_step_batches; env-major flat [states, returns,
        actions, critic_output]."""
        (states, rewards, actions, critic_output, dones, log_probs, entropies,
         actor_output) = self.get_batch()
        returns = self.calculate_returns(rewards, dones)
        return self.concat_step_batches(states, returns, actions, critic_output)

    def update_gradients(self, states, returns, actions, old_values):
        """The A2C loss of a batch (xagents/a2c/agent.py:188-218): adv = R - V_old,
        -mean(adv logp) - entropy_coef mean(H) + value_loss_coef mean((v - R)^2),
        tf.clip_by_global_norm, Keras Adam -- xa_ac_grad + the reduce's optimizer tail."""
        n = states.shape[0]
        dev = self.device
        c = lambda x, dt=torch.float32: torch.as_tensor(  # noqa: E731
            x, device=dev).to(dt).reshape(n, -1).squeeze(-1).contiguous()
        obs = torch.as_tensor(states, device=dev).float().reshape(n, -1).contiguous()
        act, ret, oldv = c(actions, torch.int32), c(returns), c(old_values)
        nb = kernels.ac_grad_blocks(n)
        partials = torch.zeros(nb, self.model.n_params, dtype=torch.float32, device=dev)
        lossp = torch.zeros(nb, 4, dtype=torch.float32, device=dev)
        g = self._grad_args(n, nb, partials, lossp)
        g.loss_kind = kernels.XA_LOSS_A2C
        g.batch = n
        g.epoch = g.mb_index = 0
        g.obs, g.actions = obs.data_ptr(), act.data_ptr()
        g.old_values, g.returns = oldv.data_ptr(), ret.data_ptr()
        g.old_logp = None
        g.adv_stats, g.adv_count, g.adv_in = None, 0.0, None
        g.loss_scale = 1.0 / (n * self.world_size)
        kernels.ac_grad(g)
        self._apply_gradients(partials)
        lp = lossp.sum(0)
        return {'pg_loss': lp[0] / lp[3], 'value_loss': lp[1] / lp[3],
                'entropy': lp[2] / lp[3]}

    _A2C_HOOKS = ('get_batch', 'calculate_returns', 'np_train_step', 'update_gradients')

    def train_step(self):
        if type(self).loss_kind == kernels.XA_LOSS_A2C and any(
                getattr(type(self), h) is not getattr(A2C, h) for h in self._A2C_HOOKS):
            # a subclass overrode a reference hook: compose the pieces (the reference's
            # np_train_step + gradient step) so the override is honoured
            self.update_gradients(*self.np_train_step())
            return
        self.fused_train_step()

    def _play_chunk(self):
        """play(): one rollout of n_steps with the actor's Categorical / Gaussian samples
        (the reference's play samples through get_model_outputs, a2c/agent.py:65-94);
        env 0's rewards and step dones. The rollout's episode statistics are not queued."""
        self._sync_stats_copy()
        if self.executor_path:
            self._executor_rollout()
        else:
            kernels.rollout(self._rargs)
            kernels.counter_bump(self.rng_counter)
        return self.b_rew[0].cpu().numpy(), self.b_done[0, 1:].cpu().numpy()

    # ---- reference-level pieces (composable, not used by the fused step) -----
    def get_model_outputs(self, inputs, models, training=True, actions=None):
        """[actions, log probs, critic output, entropy, actor output]
        (xagents/a2c/agent.py:65-94); sampling uses torch's generator for u."""
        model = models[0] if isinstance(models, (list, tuple)) else models
        obs = torch.as_tensor(inputs, dtype=torch.float32, device=self.device)
        obs = obs.reshape(-1, model.obs_dim).contiguous()
        uniforms = None
        if actions is None:
            uniforms = torch.rand(obs.shape[0], device=self.device)
        else:
            actions = torch.as_tensor(actions, device=self.device).to(torch.int32).reshape(-1)
        act, logp, value, ent, logits = kernels.mlp_forward(
            model.theta, obs, self.n_actions, actions=actions, uniforms=uniforms,
            want_logits=True)
        return act, logp, value, ent, logits

    def get_batch(self, return_kind=XA_RETURNS_NONE):
        """Run one fused rollout; returns time-major views
        [states, rewards, actions, critic_output, dones, log_probs, entropies, None]
        shaped like the reference's per-step lists (xagents/a2c/agent.py:96-139)."""
        a = self._rargs
        saved = a.return_kind
        a.return_kind = return_kind
        try:
            self._sync_stats_copy()
            kernels.rollout(a)
            kernels.counter_bump(self.rng_counter)
        finally:
            a.return_kind = saved
        self.steps += self.n_envs * self.n_steps
        self._queue_episode_stats(self.b_done, self.b_epret)
        tm = lambda x: x.transpose(0, 1)  # noqa: E731
        return [tm(self.b_obs), tm(self.b_rew), tm(self.b_act), tm(self.b_val),
                tm(self.b_done), tm(self.b_logp), tm(self.b_ent), None]

    def calculate_returns(self, rewards, dones, values=None, selected_critic_logits=None,
                          selected_importance=None):
        """n-step returns from time-major rewards [T,N], dones [T+1,N]
        (xagents/a2c/agent.py:141-171); bootstraps on V(get_states())."""
        next_values = self.get_model_outputs(self.get_states(), self.output_models)[2]
        r = torch.as_tensor(rewards, dtype=torch.float32, device=self.device).t().contiguous()
        d = torch.as_tensor(dones, dtype=torch.float32, device=self.device).t().contiguous()
        return kernels.nstep_returns(r, d, next_values.contiguous(), self.gamma).t()
