"""DQN / double DQN with the xagents class surface (xagents/dqn/agent.py:8-209) on the
device path.

train_step (dqn/agent.py:182-197), all on device except the reference's host RNG draws:
    get_actions          np.random.random() < epsilon ? np.random.randint(0, A, n)
                         : tf.argmax(Q(states / 255))         -> xa_gemm CNN + xa_dqn_act
    step_envs(store)     xa_replay_env_step (env step fused with the replay append)
    concat_buffer_samples  host index draw (random.sample / np.random.randint, the
                         reference's streams) -> xa_ring_gather, env-major batch
    get_targets          Q(s), [Q(s')], Qt(s') (one online pass over [s; s'] when double)
                         -> xa_dqn_td_grad (TD target, MSE gradient of the batch sum)
    update_gradients     CNN backward (xa_gemm / xa_conv1d_input_grad) -> Keras Adam
                         (no gradient clipping, optimizer.minimize): the 37632 x 512 dense
                         layer's step inside its weight-gradient GEMM (xa_gemm_adam, no
                         gradient round trip), the other layers' via xa_clip_adam
at_step_end: hard target copy when steps % target_sync_steps == 0 (xa_polyak, tau 1).
"""
import os

import numpy as np
import torch

from xagents_amd import kernels
from xagents_amd._lib import call, stream
from xagents_amd.base import OffPolicy
from xagents_amd.envs import Discrete
from xagents_amd.layers import LayerExecutor, adam_apply


class DQN(OffPolicy):
    """Playing Atari with Deep Reinforcement Learning https://arxiv.org/abs/1312.5602"""

    def __init__(
        self,
        envs,
        model,
        buffers,
        double=False,
        epsilon_start=1.0,
        epsilon_end=0.02,
        epsilon_decay_steps=150000,
        target_sync_steps=1000,
        huber_delta=None,
        **kwargs,
    ):
        super(DQN, self).__init__(envs, model, buffers, **kwargs)
        # opt-in Huber-TD loss (BASELINE north_star; the reference uses MSE,
        # dqn/agent.py:170): None keeps the reference's MSE
        self.huber_delta = huber_delta
        self.assert_valid_env(envs[0], Discrete)
        self.target_model = self.model.clone()
        self.double = double
        self.epsilon_start = self.epsilon = epsilon_start
        self.epsilon_end = epsilon_end
        self.epsilon_decay_steps = epsilon_decay_steps
        self.target_sync_steps = target_sync_steps
        self.batch_dtypes = ['uint8', 'int64', 'float64', 'bool', 'uint8']
        self._setup_device()

    def _setup_device(self):
        self._setup_offpolicy((), np.int32)
        k = self.replay.k
        if self.n_envs * k > 1 and k == 1:
            # ReplayBuffer1.get_sample returns the raw tuple for k == 1 and
            # concat_buffer_samples then fails (buffers.py:96-98, base.py:363-367)
            raise ValueError('zero-dimensional arrays cannot be concatenated')
        B = self.n_envs * k
        self.batch_size = B
        dev = self.device
        obs = self.envs.obs_shape
        self.xb = torch.zeros((2 * B,) + obs, dtype=self.replay.obs_t, device=dev)
        self.b_act = torch.zeros(B, dtype=torch.int32, device=dev)
        self.b_rew = torch.zeros(B, dtype=torch.float32, device=dev)
        self.b_done = torch.zeros(B, dtype=torch.float32, device=dev)
        self.dq = torch.zeros(B, self.n_actions, dtype=torch.float32, device=dev)
        self.td_loss = torch.zeros(B, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.model.n_params, dtype=torch.float32, device=dev)
        self.adam_ws = torch.zeros(1024, dtype=torch.float64, device=dev)
        self.actions = torch.zeros(self.n_envs, dtype=torch.int32, device=dev)
        self._rand_actions = torch.zeros(self.n_envs, dtype=torch.int32, device=dev)
        self.ex_online = LayerExecutor(self.model, 2 * B if self.double else B)
        self.ex_target = LayerExecutor(self.target_model, B)
        self.ex_act = LayerExecutor(self.model, self.n_envs)
        # forward-only executors skip the conv stack's hidden activations
        self.ex_target.keep_hidden = self.ex_act.keep_hidden = False
        self._sync_params(self.model, self.target_model)

    # ---- reference surface ---------------------------------------------------
    def update_epsilon(self):
        """dqn/agent.py:86-95"""
        self.epsilon = max(
            self.epsilon_end, self.epsilon_start - self.steps / self.epsilon_decay_steps)

    def sync_target_model(self):
        """dqn/agent.py:97-105"""
        if self.steps % self.target_sync_steps == 0:
            call('xa_polyak', self.model.theta.data_ptr(), self.target_model.theta.data_ptr(),
                 self.model.n_params, kernels._f32(1.0), stream())

    def get_model_outputs(self, inputs, models, training=True):
        """[argmax Q, Q] (dqn/agent.py:70-84) for a device batch of states."""
        model = models[0] if isinstance(models, (list, tuple)) else models
        x = torch.as_tensor(inputs, device=self.device).contiguous()
        ex = LayerExecutor(model, x.shape[0])
        q = ex.forward(x)[0].clone()
        act = torch.empty(x.shape[0], dtype=torch.int32, device=self.device)
        call('xa_dqn_act', q.data_ptr(), x.shape[0], self.n_actions, None, 0, act.data_ptr(),
             stream())
        return act, q

    def get_actions(self):
        """Epsilon-greedy, all envs random or all greedy (dqn/agent.py:107-116)."""
        if np.random.random() < self.epsilon:
            r = np.random.randint(0, self.n_actions, self.n_envs)
            self._rand_actions.copy_(torch.from_numpy(r.astype(np.int32)))
            call('xa_dqn_act', None, self.n_envs, self.n_actions,
                 self._rand_actions.data_ptr(), 1, self.actions.data_ptr(), stream())
        elif self._head_fused():
            # greedy: the argmax rides in the Q head's launch (xa_dqn_head mode 0)
            self.ex_act.forward(self.envs.state, head=self._head_args('act'))
        else:
            q = self.ex_act.forward(self.envs.state)[0]
            call('xa_dqn_act', q.data_ptr(), self.n_envs, self.n_actions, None, 0,
                 self.actions.data_ptr(), stream())
        return self.actions

    def _head_fused(self):
        """The Q head (last layer: dense, <= 8 actions, linear, K <= 4096) can run as
        xa_dqn_head (XA_DQN_FUSED_HEAD=0: separate xa_dqn_act / xa_dqn_td_grad launches)."""
        if '_hf' not in self.__dict__:
            import os
            ls = self.model.layers
            last = ls[-1]
            self._hf = (os.environ.get('XA_DQN_FUSED_HEAD', '1') != '0' and
                        last.kind == 'dense' and last.units <= 8 and
                        last.in_features <= 4096 and last.activation in (None, 'linear') and
                        list(self.model.outputs) == [len(ls) - 1])
        return self._hf

    def _head_args(self, kind):
        """XaDqnHeadArgs of the acting head (argmax into self.actions) or of the target
        head (TD target + MSE / Huber gradient of the sampled batch, t += 1)."""
        cache = self.__dict__.setdefault('_head_cache', {})
        if kind not in cache:
            from xagents_amd._lib import XaDqnHeadArgs
            h = XaDqnHeadArgs()
            if kind == 'act':
                h.mode, h.actions = 0, self.actions.data_ptr()
            else:
                B = self.batch_size
                q_all = self.ex_online.outs[-1]
                h.mode = 1
                h.q = q_all.data_ptr()
                h.q_next_online = q_all[B:].data_ptr() if self.double else None
                h.act, h.rewards = self.b_act.data_ptr(), self.b_rew.data_ptr()
                h.dones = self.b_done.data_ptr()
                h.gamma = kernels._f32(self.gamma)
                h.huber = kernels._f32(self.huber_delta or 0.0)
                h.dq, h.loss = self.dq.data_ptr(), self.td_loss.data_ptr()
                h.adam_step = self.model.optimizer.iterations.data_ptr()
            cache[kind] = h
        return cache[kind]

    def _play_actions(self):
        """play(): greedy argmax Q for every env (get_model_outputs(...)[0],
        xagents/base.py:641-644 with dqn/agent.py:70-84)."""
        q = self.ex_act.forward(self.envs.state)[0]
        call('xa_dqn_act', q.data_ptr(), self.n_envs, self.n_actions, None, 0,
             self.actions.data_ptr(), stream())
        return self.actions

    def concat_buffer_samples(self):
        """One sampled batch gathered from the device rings in the reference's index
        order: [states, actions, rewards, dones, new_states] (base.py:344-368)."""
        slots = self.replay.upload_slots(self.replay.sample_slots())
        B = self.batch_size
        self.replay.gather(slots, self.xb[:B], self.b_act, self.b_rew, self.b_done,
                           self.xb[B:])
        return [self.xb[:B], self.b_act, self.b_rew, self.b_done, self.xb[B:]]

    def _td_grad(self):
        """TD targets + loss gradient; the same launch bumps the optimizer's t (the update's
        Adam reads it after the backward)."""
        B = self.batch_size
        q_all = self.ex_online.forward(self.xb if self.double else self.xb[:B])[0]
        if self._head_fused():
            # the TD target and its gradient ride in the target head's launch (mode 1)
            self.ex_target.forward(self.xb[B:], head=self._head_args('td'))
            return
        q_next_t = self.ex_target.forward(self.xb[B:])[0]
        q_next_o = q_all[B:].data_ptr() if self.double else None
        call('xa_dqn_td_grad', q_all.data_ptr(), q_next_t.data_ptr(), q_next_o,
             self.b_act.data_ptr(), self.b_rew.data_ptr(), self.b_done.data_ptr(), B,
             self.n_actions, kernels._f32(self.gamma), kernels._f32(self.huber_delta or 0.0),
             self.dq.data_ptr(), self.td_loss.data_ptr(),
             self.model.optimizer.iterations.data_ptr(), stream())

    # the raw gradient of the dense layers whose Adam step runs inside their weight-gradient
    # GEMM is written to self.grad only on request (the raw-gradient parity tests)
    write_raw_grad = False

    def _fused_adam_layers(self):
        """Dense layers (the 37632 x 512 one of the NatureCNN cfg) whose Keras Adam step runs
        in the weight-gradient GEMM's epilogue (xa_gemm_adam): the reference's DQN update has
        no gradient clip (dqn/agent.py:158-171), so a layer's step needs only its own
        gradient. Not when data parallel (the gradient is all-reduced before Adam)."""
        if '_fused_adam' not in self.__dict__:
            import os
            ex, layers = self.ex_online, self.model.layers
            fl = [] if self.distributed or os.environ.get('XA_DQN_FUSED_ADAM', '1') == '0' else [
                i for i, l in enumerate(layers)
                if l.kind == 'dense' and l.in_features * l.units >= (1 << 20) and
                ex.adam_fusable(i, self.batch_size)]
            # the parameter ranges the remaining Adam launches cover
            rest, lo = [], 0
            for i in fl:
                w0, b0 = ex.offsets[i]
                if w0 > lo:
                    rest.append((lo, w0))
                lo = b0 + layers[i].units
            if lo < self.model.n_params:
                rest.append((lo, self.model.n_params))
            self._fused_adam = (fl, rest)
        return self._fused_adam

    def _apply(self):
        opt = self.model.optimizer
        fl, rest = self._fused_adam_layers()
        if fl:
            # t += 1 happened in _td_grad (the fused epilogues read it); the dense layers'
            # Adam runs inside the backward, the rest of the parameters in one launch per range
            th, m, v = self.model.theta, opt.m, opt.v
            ex = self.ex_online
            spec = {i: (adam_apply(th, m, v, opt.iterations, opt, ex.offsets[i][0]),
                        self.write_raw_grad) for i in fl}
            rest = list(rest)
            stack_end = ex.offsets[2][1] + ex.layers[2].filters if ex.stack else None
            if ex.stack and ex._stack_bwd_ok() and (0, stack_end) in rest and \
                    os.environ.get('XA_STACK_ADAM', '1') != '0':
                # the conv stack's Adam inside its backward's reduce launch, with the one
                # other range (the Q head's, final by then) folded into the same launch
                rest.remove((0, stack_end))
                tail = None
                later = [r for r in rest if r[0] >= stack_end]
                if later:
                    lo, hi = later[0]
                    rest.remove(later[0])
                    tail = (adam_apply(th, m, v, opt.iterations, opt, lo),
                            self.grad.data_ptr() + 4 * lo, hi - lo)
                spec['stack'] = (adam_apply(th, m, v, opt.iterations, opt, 0),
                                 self.write_raw_grad, tail)
            ex.backward([self.dq], self.grad, batch=self.batch_size, adam=spec)
            for lo, hi in rest:
                kernels.clip_adam(th[lo:hi], m[lo:hi], v[lo:hi], self.grad[lo:hi],
                                  opt.iterations, opt.learning_rate, opt.beta_1, opt.beta_2,
                                  opt.epsilon, clip_norm=0.0, workspace=self.adam_ws)
            return
        self.ex_online.backward([self.dq], self.grad, batch=self.batch_size)
        scale = self._reduce_grad(self.grad)
        kernels.clip_adam(self.model.theta, opt.m, opt.v, self.grad, opt.iterations,
                          opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                          clip_norm=0.0, grad_scale=scale, workspace=self.adam_ws)

    def get_targets(self, states, actions, rewards, dones, new_states):
        """TD targets y [B, A] (dqn/agent.py:118-156)."""
        q = self.get_model_outputs(states, self.model)[1]
        qt = self.get_model_outputs(new_states, self.target_model)[1]
        if self.double:
            a_next = self.get_model_outputs(new_states, self.model)[0].long()
            v = qt.gather(1, a_next[:, None])[:, 0]
        else:
            v = qt.max(1).values
        d = torch.as_tensor(dones, device=self.device).bool()
        v = torch.where(d, torch.zeros_like(v), v)
        y = q.clone()
        upd = v * np.float32(self.gamma) + torch.as_tensor(rewards, device=self.device).float()
        idx = torch.as_tensor(actions, device=self.device).long()
        y[torch.arange(y.shape[0], device=self.device), idx] = upd
        return y

    def update_gradients(self, x, y):
        """MSE(y, Q(x)) minimized with Keras Adam (dqn/agent.py:158-171)."""
        x = torch.as_tensor(x, device=self.device).contiguous()
        y = torch.as_tensor(y, device=self.device, dtype=torch.float32).contiguous()
        ex = LayerExecutor(self.model, x.shape[0])
        q = ex.forward(x)[0]
        dq = torch.empty_like(q)
        call('xa_mse_grad', q.data_ptr(), y.data_ptr(), x.shape[0], self.n_actions,
             dq.data_ptr(), None, stream())
        ex.backward([dq], self.grad)
        opt = self.model.optimizer
        call('xa_adam_step_bump', opt.iterations.data_ptr(), stream())
        kernels.clip_adam(self.model.theta, opt.m, opt.v, self.grad, opt.iterations,
                          opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                          clip_norm=0.0, workspace=self.adam_ws)

    def at_step_start(self):
        self.update_epsilon()

    def train_step(self):
        """dqn/agent.py:182-197"""
        hooks = ('get_targets', 'update_gradients', 'concat_buffer_samples', 'get_actions')
        if any(getattr(type(self), h) is not getattr(DQN, h) for h in hooks):
            actions = self.get_actions()
            self._env_step(actions.to(torch.int32).contiguous())
            self.steps += self.n_envs
            batch = self.concat_buffer_samples()
            self.update_gradients(batch[0], self.get_targets(*batch))
            return
        self.get_actions()
        self._env_step(self.actions)
        self.steps += self.n_envs
        # host index draw in the reference's order, then the device learner phase (its
        # gather reads the staged slots from mapped pinned memory: no upload launch;
        # XA_PINNED_SLOTS=0: the upload copy)
        if self._pinned_slots():
            self.replay.stage_slots(self.replay.sample_slots())
            self._run_learn()
            if self.replay._stage_open:  # (graph replay: no event inside the capture)
                self.replay.stage_consumed()
        else:
            self.replay.upload_slots(self.replay.sample_slots())
            self._run_learn()

    def _pinned_slots(self):
        if '_pslots' not in self.__dict__:
            self._pslots = os.environ.get('XA_PINNED_SLOTS', '1') != '0' and \
                torch.device(self.device).type == 'cuda'
        return self._pslots

    def _stage_early(self):
        """Record the staged slots' completion event right behind the gather (default;
        XA_DQN_STAGE_EARLY=0: behind the whole learner phase, for A/B)."""
        if '_se_on' not in self.__dict__:
            self._se_on = os.environ.get('XA_DQN_STAGE_EARLY', '1') != '0'
        return self._se_on

    def _learn_phase(self):
        """gather the sampled batch -> TD gradient -> CNN backward -> Keras Adam."""
        B = self.batch_size
        r = self.replay
        src = (r.stage_ptr(), r.slots.numel()) if self._pinned_slots() else r.slots
        r.gather(src, self.xb[:B], self.b_act, self.b_rew, self.b_done, self.xb[B:])
        if self._pinned_slots() and self._stage_early() and \
                not torch.cuda.is_current_stream_capturing():
            # the gather is the staged slots' only reader: the next step's stage_slots waits
            # for it alone, not for the whole learner phase, so the host enqueues the next
            # acting launches while this backward runs (no idle gap between steps)
            r.stage_consumed()
        self._td_grad()
        self._apply()

    def _run_learn(self):
        """Eager once, then captured and replayed as a hipGraph (the sample slots live in a
        fixed device buffer); data-parallel steps stay eager (torch collective)."""
        if not getattr(self, 'use_graph', True) or self.distributed or not self._learn_graph():
            self._learn_phase()
        elif getattr(self, '_lgraph', None) is not None:
            self._lgraph.replay()
        elif getattr(self, '_lwarm', False):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._learn_phase()
            self._lgraph = g
            g.replay()
        else:
            self._learn_phase()
            self._lwarm = True

    def _learn_graph(self):
        """Launch the learner phase directly (default: between the eager acting launches a
        graph replay adds its own transition latency; C3 0.4886 -> 0.4840 ms per step,
        profiles/r06zb_dqn_learn_graph_ab.txt) or replay it from a hipGraph
        (XA_DQN_LEARN_GRAPH=1)."""
        if '_lg_on' not in self.__dict__:
            self._lg_on = os.environ.get('XA_DQN_LEARN_GRAPH', '0') == '1'
        return self._lg_on

    def _on_lr_change(self):
        self._lgraph = None  # the learning rate is baked into the Adam launch
        self._lwarm = False

    def at_step_end(self):
        self.sync_target_model()
