"""BaseAgent / OnPolicy / OffPolicy with the reference's class surface
(xagents/base.py:22-751). The host-side bookkeeping (metrics, checkpoints, early
stopping, history) is kept in Python as in the reference; env stepping, batching
and math go to libxagents_hip.so through the subclasses.

Differences forced by the device design (documented in DESIGN.md):
* `envs` is a device vector env (xagents_amd.envs) rather than a list of gym envs;
  it supports len(), envs[0].observation_space / action_space.
* Episode statistics of a fused rollout are copied back asynchronously and folded
  into total_rewards / games / done_envs in the reference's step-major, env-minor
  order at the next train_step (one train_step of lag), so the host never stalls
  the device between steps.
"""
import os
import random
from abc import ABC
from collections import deque
from contextlib import nullcontext as _nullcontext
from datetime import timedelta
from pathlib import Path
from time import perf_counter

import numpy as np
import torch
import torch.distributed as dist

from xagents_amd.envs import Box, Discrete
from xagents_amd.utils.common import write_from_dict


class BaseAgent(ABC):
    def __init__(
        self,
        envs,
        model,
        checkpoints=None,
        reward_buffer_size=100,
        n_steps=1,
        gamma=0.99,
        display_precision=2,
        seed=None,
        log_frequency=None,
        history_checkpoint=None,
        plateau_reduce_factor=0.9,
        plateau_reduce_patience=10,
        early_stop_patience=3,
        divergence_monitoring_steps=None,
        quiet=False,
        trial=None,
    ):
        assert envs, 'No environments given'
        self.n_envs = len(envs)
        self.envs = envs
        self.model = model
        self.checkpoints = checkpoints
        self.total_rewards = deque(maxlen=reward_buffer_size)
        self.n_steps = n_steps
        self.gamma = gamma
        self.display_precision = display_precision
        self.seed = seed
        self.output_models = [self.model]
        self.log_frequency = log_frequency or self.n_envs
        # the agent package (xagents/base.py:88); a user subclass defined outside the
        # package (the reference would fail here) takes its nearest agent base class's id
        self.id = next((c.__module__.split('.')[1] for c in type(self).__mro__
                        if c.__module__.startswith('xagents_amd.')), self.__module__)
        self.history_checkpoint = history_checkpoint
        self.plateau_reduce_factor = plateau_reduce_factor
        self.plateau_reduce_patience = plateau_reduce_patience
        self.early_stop_patience = early_stop_patience
        self.divergence_monitoring_steps = divergence_monitoring_steps
        self.quiet = quiet
        self.trial = trial
        self.reported_rewards = 0
        self.plateau_count = 0
        self.early_stop_count = 0
        self.target_reward = None
        self.max_steps = None
        self.input_shape = self.envs[0].observation_space.shape
        self.n_actions = None
        self.best_reward = -float('inf')
        self.mean_reward = -float('inf')
        self.device = getattr(envs, 'device', torch.device('cuda'))
        self.dones = [False] * self.n_envs
        self.steps = 0
        self.frame_speed = 0
        self.last_reset_step = 0
        self.training_start_time = None
        self.last_reset_time = None
        self.games = 0
        self.episode_rewards = np.zeros(self.n_envs)
        self.done_envs = 0
        self.supported_action_spaces = Box, Discrete
        self._pending_stats = None
        if seed:
            self.set_seeds(seed)
        self.reset_envs()
        self.set_action_count()
        self.img_inputs = len(self.input_shape) >= 2
        self.display_titles = (
            'time',
            'steps',
            'games',
            'speed',
            'mean reward',
            'best reward',
        )

    # ---- reference surface (host bookkeeping) -----------------------------
    def assert_valid_env(self, env, valid_type):
        assert isinstance(env.action_space, valid_type), (
            f'Invalid environment: {env.spec.id}. {self.__class__.__name__} supports '
            f'environments with a {valid_type} action space only, got {env.action_space}'
        )

    def display_message(self, *args, **kwargs):
        if not self.quiet:
            print(*args, **kwargs)

    def set_seeds(self, seed):
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.envs.seed(seed)
        os.environ['PYTHONHASHSEED'] = f'{seed}'
        random.seed(seed)

    def reset_envs(self):
        self.envs.reset()

    @property
    def states(self):
        """Per-env view of the current (post-reset) observations, as the reference's list
        (LazyFrames for Atari frames, xagents/base.py:105-113); the device path reads
        self.envs.state directly."""
        from xagents_amd.utils.common import DeviceStates
        return DeviceStates(self.envs.state)

    def set_action_count(self):
        action_space = self.envs[0].action_space
        assert (
            type(action_space) in self.supported_action_spaces
        ), f'Expected one of {self.supported_action_spaces}, got {action_space}'
        if isinstance(action_space, Discrete):
            self.n_actions = action_space.n
        if isinstance(action_space, Box):
            self.n_actions = action_space.shape[0]

    def check_checkpoints(self):
        n_models = len(self.output_models)
        n_checkpoints = len(self.checkpoints)
        assert n_models == n_checkpoints, (
            f'Expected {n_models} checkpoints for {n_models} '
            f'given output models, got {n_checkpoints}'
        )

    def checkpoint(self):
        if self.mean_reward > self.best_reward:
            self.plateau_count = 0
            self.early_stop_count = 0
            self.display_message(
                f'Best reward updated: {self.best_reward} -> {self.mean_reward}'
            )
            if self.checkpoints:
                # a persistent launch that failed (device status word) left the weights
                # invalid: raise before any of them reaches a checkpoint file
                checks = getattr(self, '_device_checks', None)
                if checks is not None:
                    checks()
                for model, checkpoint in zip(self.output_models, self.checkpoints):
                    model.save_weights(checkpoint)
        self.best_reward = max(self.mean_reward, self.best_reward)

    def display_metrics(self):
        display_values = (
            timedelta(seconds=perf_counter() - self.training_start_time),
            self.steps,
            self.games,
            f'{round(self.frame_speed)} steps/s',
            self.mean_reward,
            self.best_reward,
        )
        display = (
            f'{title}: {value}'
            for title, value in zip(self.display_titles, display_values)
        )
        self.display_message(', '.join(display))

    def update_metrics(self):
        self.checkpoint()
        if (
            self.divergence_monitoring_steps
            and self.steps >= self.divergence_monitoring_steps
            and self.mean_reward <= self.best_reward
        ):
            self.plateau_count += 1
        if self.plateau_count >= self.plateau_reduce_patience:
            current_lr, new_lr = None, None
            pending = getattr(self, '_pending_lr', None)
            for model in self.output_models:
                current_lr = model.optimizer.learning_rate
                if pending is not None and model is self.output_models[-1]:
                    # data parallel: a reduction not applied yet (it waits for the next
                    # _dp_sync) compounds with this one, as the reference's would
                    current_lr = pending
                new_lr = current_lr * self.plateau_reduce_factor
            self.display_message(f'Learning rate reduced {current_lr} -> {new_lr}')
            if getattr(self, 'distributed', False):
                # data parallel: rank 0 decides, every rank applies it at the same train
                # step (_dp_sync), so learning rates and launch state stay identical
                if self.rank == 0:
                    self._pending_lr = new_lr
            else:
                # the reference only updates the LAST output model (xagents/base.py:277-284)
                self.output_models[-1].optimizer.learning_rate = new_lr
                self._on_lr_change()
            self.plateau_count = 0
            self.early_stop_count += 1
        self.frame_speed = (self.steps - self.last_reset_step) / (
            perf_counter() - self.last_reset_time
        )
        self.last_reset_step = self.steps
        self.mean_reward = np.around(
            np.mean(self.total_rewards), self.display_precision
        )

    def _on_lr_change(self):
        """Subclasses holding captured graphs re-capture them (lr is a kernel arg)."""

    # data parallel: the host decisions that must agree across ranks -- plateau learning-
    # rate reductions and stopping on the target reward / early-stop patience, which the
    # reference's one process takes from its own rewards -- are rank 0's, exchanged every
    # DP_SYNC_STEPS train steps of fit() and applied by every rank at the same step
    DP_SYNC_STEPS = 64

    def _dp_sync(self, stop_local):
        """One small collective (MAX over ranks): rank 0's pending learning rate and stop
        decision. Returns the agreed stop decision."""
        lr0 = getattr(self, '_pending_lr', None)
        t = torch.tensor([lr0 if (self.rank == 0 and lr0 is not None) else -1.0,
                          1.0 if (self.rank == 0 and stop_local) else 0.0], dtype=torch.float64)
        if dist.get_backend() != 'gloo':
            t = t.to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lr, stop = float(t[0].item()), bool(t[1].item() > 0)
        self._pending_lr = None
        if lr > 0:
            self.output_models[-1].optimizer.learning_rate = lr
            self._on_lr_change()
        return stop

    def _fit_done(self):
        """training_done(), collective in data-parallel runs: max_steps is identical on every
        rank (equal step counts); the reward-based decisions are rank 0's (_dp_sync)."""
        done = self.training_done()
        if not getattr(self, 'distributed', False):
            return done
        if self.max_steps and self.steps >= self.max_steps:
            return True
        self._fit_steps = getattr(self, '_fit_steps', 0) + 1
        every = int(os.environ.get('XA_DP_SYNC_STEPS', self.DP_SYNC_STEPS))
        if self._fit_steps % every:
            return False
        return self._dp_sync(done)

    def report_rewards(self):
        self.trial.report(np.mean(self.total_rewards), self.reported_rewards)
        self.reported_rewards += 1
        if self.trial.should_prune():
            import optuna

            raise optuna.exceptions.TrialPruned()

    def check_episodes(self):
        self._drain_episode_stats()
        if self.done_envs >= self.log_frequency:
            self.update_metrics()
            if self.trial:
                self.report_rewards()
            self.last_reset_time = perf_counter()
            self.display_metrics()
            self.done_envs = 0

    def training_done(self):
        if self.early_stop_count >= self.early_stop_patience:
            self.display_message('Early stopping')
            return True
        if self.target_reward and self.mean_reward >= self.target_reward:
            self.display_message(f'Reward achieved in {self.steps} steps')
            return True
        if self.max_steps and self.steps >= self.max_steps:
            self.display_message('Maximum steps exceeded')
            return True
        return False

    def concat_buffer_samples(self):
        """Concatenate per-env buffer samples (xagents/base.py:344-368)."""
        if hasattr(self, 'buffers'):
            batches = []
            for i in range(self.n_envs):
                batches.append(self.buffers[i].get_sample())
            dtypes = (
                self.batch_dtypes
                if hasattr(self, 'batch_dtypes')
                else [np.float32 for _ in range(len(batches[0]))]
            )
            if len(batches) > 1:
                return [
                    np.concatenate(item).astype(dtype)
                    for (item, dtype) in zip(zip(*batches), dtypes)
                ]
            return [item.astype(dtype) for (item, dtype) in zip(batches[0], dtypes)]

    def update_history(self, episode_reward):
        data = {
            'mean_reward': [self.mean_reward],
            'best_reward': [self.best_reward],
            'episode_reward': [episode_reward],
            'step': [self.steps],
            'time': [perf_counter() - self.training_start_time],
        }
        write_from_dict(data, self.history_checkpoint)

    def init_from_checkpoint(self):
        import pandas as pd

        previous_history = pd.read_parquet(self.history_checkpoint)
        expected_columns = {'time', 'mean_reward', 'best_reward', 'step', 'episode_reward'}
        assert (
            set(previous_history.columns) == expected_columns
        ), f'Expected the following columns: {expected_columns}, got {set(previous_history.columns)}'
        last_row = previous_history.loc[previous_history['time'].idxmax()]
        self.mean_reward = last_row['mean_reward']
        self.best_reward = previous_history['best_reward'].max()
        history_start_steps = last_row['step']
        history_start_time = last_row['time']
        self.training_start_time = perf_counter() - history_start_time
        self.last_reset_step = self.steps = int(history_start_steps)
        self.total_rewards.append(last_row['episode_reward'])
        self.games = previous_history.shape[0]

    def init_training(self, target_reward, max_steps, monitor_session):
        self.target_reward = target_reward
        self.max_steps = max_steps
        if monitor_session:
            import wandb

            wandb.init(name=monitor_session)
        if self.checkpoints:
            self.check_checkpoints()
        self.training_start_time = perf_counter()
        self.last_reset_time = perf_counter()
        if self.history_checkpoint and Path(self.history_checkpoint).exists():
            self.init_from_checkpoint()

    def train_step(self):
        raise NotImplementedError(
            f'train_step() should be implemented by {self.__class__.__name__} subclasses'
        )

    def get_model_outputs(self, inputs, models, training=True):
        if self.img_inputs:
            inputs = torch.as_tensor(inputs, device=self.device).float() / 255.0
        if not isinstance(models, (list, tuple)):
            return models(inputs, training=training)
        elif len(models) == 1:
            return models[0](inputs, training=training)
        return [sub_model(inputs, training=training) for sub_model in models]

    def at_step_start(self):
        pass

    def at_step_end(self):
        pass

    def get_states(self):
        """Most recent (post-reset) states, [n_envs, *obs] on device."""
        return self.envs.state

    def get_dones(self):
        return self.envs.done

    @staticmethod
    def concat_step_batches(*args):
        """Time-major [T, N, ...] -> env-major flat [N*T, ...] (xagents/base.py:549-564).

        Works on numpy arrays and torch tensors. The device rollout already stores its
        buffers env-major, so the fused path never needs this copy."""
        concatenated = []
        for arg in args:
            if len(arg.shape) == 1:
                arg = arg[..., None] if isinstance(arg, torch.Tensor) else np.expand_dims(arg, -1)
            if isinstance(arg, torch.Tensor):
                concatenated.append(arg.transpose(0, 1).reshape(-1, *arg.shape[2:]))
            else:
                concatenated.append(arg.swapaxes(0, 1).reshape(-1, *arg.shape[2:]))
        return concatenated

    # ---- device episode bookkeeping ----------------------------------------
    def _queue_episode_stats(self, done_out, epret_out, after=None, group_end=True):
        """Async D2H copy of one rollout's done flags [N,T+1] and running returns [N,T]
        (with the persistent update's status word). `after`: an event recorded on the
        launch stream right after the rollout -- the copy then runs on a side stream
        behind it, overlapping the update, and the next rollout waits for it
        (_sync_stats_copy). When the persistent update stores the statistics into its host
        slots itself (PPO._setup_fused_stats) there is nothing to launch: the step's slot is
        its launch number modulo XA_PPO_STATS_SLOTS, and the fold checks the number the
        launch wrote. Steps are folded in groups behind one completion event (`group_end`:
        the caller closes a group, e.g. after a hipGraph replay of several train steps;
        XA_STATS_EVERY groups single steps), at most half the slots per group, so that a
        slot is folded before a later launch reuses it."""
        if getattr(self, '_stats_fused', False) and after is None and \
                getattr(self, 'update_mode', None) == 'persistent' and \
                done_out.data_ptr() == self.b_done.data_ptr():
            if getattr(self, '_stats_queue', None) is None or \
                    getattr(self, '_stats_queue_kind', None) != 'fused':
                self._drain_episode_stats()
                self._stats_queue = []
                self._stats_queue_kind = 'fused'
                self._fused_events = [torch.cuda.Event() for _ in range(4)]
                self._fused_ev_i = 0
                self._fused_pending = []
            self._fused_pending.append(self._upd_launches - 1)
            self._pending_stats = (done_out, epret_out)
            every = min(int(os.environ.get('XA_STATS_EVERY', '1')), self.FUSED_GROUP_MAX)
            if group_end and len(self._fused_pending) >= every or \
                    len(self._fused_pending) >= self.FUSED_GROUP_MAX:
                self._close_fused_group()
            return
        if self._pending_stats is None or self._pending_stats[0].shape != done_out.shape or \
                getattr(self, '_stats_queue_kind', None) == 'fused':
            self._drain_episode_stats()
            self._host_done = [torch.empty(done_out.shape, dtype=done_out.dtype).pin_memory()
                               for _ in range(2)]
            self._host_epret = [torch.empty(epret_out.shape, dtype=epret_out.dtype).pin_memory()
                                for _ in range(2)]
            self._host_pack = None
            self._host_copy_args = {}  # xa_copy_to_host args keyed on the old buffers
            # one completion event per host slot, reused (a slot is re-recorded only after
            # its previous copy was folded): no event creation on the step path
            self._stats_events = [torch.cuda.Event(), torch.cuda.Event()]
            self._stats_slot = 0
            self._stats_queue = []
            self._stats_queue_kind = 'copy'
        slot = self._stats_slot
        side = None
        if after is not None:
            if getattr(self, '_stats_stream', None) is None:
                self._stats_stream = torch.cuda.Stream(device=done_out.device)
                self._stats_warm = False
            side = self._stats_stream
            side.wait_event(after)
        with torch.cuda.stream(side) if side is not None else _nullcontext():
            pack = getattr(self, '_stats_pack', None)
            # the statistics leave in ONE xa_copy_to_host launch (stores into the mapped
            # pinned buffers) instead of D2H DMA copies: 16 envs 0.2859 -> 0.2814 ms per
            # step (three segments), C2 0.419 -> 0.401 ms (the whole pack as one segment)
            if pack is not None and pack.numel() >= 65536 and \
                    done_out.data_ptr() == self.b_done.data_ptr():
                # done, episode returns and the status word in one copy (a2c/agent.py)
                if self._host_pack is None:
                    nd, sd, oe, se, os_ = self._stats_views
                    self._host_pack = [torch.zeros(pack.shape, dtype=pack.dtype).pin_memory()
                                       for _ in range(2)]
                    self._host_done = [h[:nd].view(sd) for h in self._host_pack]
                    self._host_epret = [h[oe:oe + se[0] * se[1]].view(se)
                                        for h in self._host_pack]
                    self._host_status = [h[os_:os_ + 1].view(torch.int32)
                                         for h in self._host_pack]
                if side is not None and not self._stats_warm:
                    # the first device-to-pinned-host copies of a side stream block the
                    # host for ~7 ms each (MI355X / ROCm 7.2, tools/diag_d2h_side.py): pay
                    # them here, once, not inside a later step
                    for _ in range(4):
                        for h in self._host_pack:
                            h.copy_(pack, non_blocking=True)
                    side.synchronize()
                    self._stats_warm = True
                if side is None:
                    self._copy_to_host([(pack, self._host_pack[slot])])
                else:
                    self._host_pack[slot].copy_(pack, non_blocking=True)
            else:
                segs = [(done_out, self._host_done[slot]), (epret_out, self._host_epret[slot])]
                status = getattr(self, 'device_status', None)
                if status is not None:
                    if getattr(self, '_host_status', None) is None:
                        self._host_status = [torch.zeros(status.shape, dtype=status.dtype)
                                             .pin_memory() for _ in range(2)]
                    segs.append((status, self._host_status[slot]))
                self._copy_to_host(segs)
            ev = self._stats_events[slot]
            ev.record()
        self._stats_guard = ev if side is not None else None
        self._stats_queue.append((slot, ev))
        self._stats_slot ^= 1
        self._pending_stats = (done_out, epret_out)
        # keep at most one rollout in flight: fold the previous one now
        while len(self._stats_queue) > 1:
            self._fold_item(self._stats_queue.pop(0))

    # steps folded behind one event: half the in-launch statistics slots (_lib.XA_PPO_STATS_SLOTS)
    FUSED_GROUP_MAX = 8

    def _close_fused_group(self):
        """One completion event behind the pending fused steps; fold the previous group
        (its slots are complete once its event is), so one group stays in flight."""
        if not getattr(self, '_fused_pending', None):
            return
        ev = self._fused_events[self._fused_ev_i % len(self._fused_events)]
        self._fused_ev_i += 1
        ev.record()
        self._stats_queue.append(('fused', ev, tuple(self._fused_pending)))
        self._fused_pending = []
        while len(self._stats_queue) > 1:
            self._fold_item(self._stats_queue.pop(0))

    def _fold_item(self, item):
        if item[0] == 'fused':
            _, ev, gens = item
            ev.synchronize()
            for gen in gens:
                self._fold_stats(None, None, gen)
        else:
            self._fold_stats(*item)

    def _copy_to_host(self, segs):
        """(device, pinned host) tensor pairs to the host in ONE xa_copy_to_host launch on
        the current stream (at 16 envs three D2H DMA copies cost ~14 us of stream time per
        train step; the launch stores the same words into the mapped host buffers)."""
        if not segs[0][0].is_cuda:
            for d, h in segs:
                h.copy_(d, non_blocking=True)
            return
        from xagents_amd._lib import XaHostCopyArgs, call, stream
        import ctypes
        key = tuple((d.data_ptr(), h.data_ptr(), d.numel() * d.element_size()) for d, h in segs)
        cache = self.__dict__.setdefault('_host_copy_args', {})
        a = cache.get(key)
        if a is None:
            a = XaHostCopyArgs()
            a.n_segments = len(segs)
            for i, (d, h) in enumerate(segs):
                assert d.is_contiguous() and h.is_contiguous() and h.is_pinned()
                dev = ctypes.c_void_p()
                call('xa_host_device_pointer', ctypes.c_void_p(h.data_ptr()), ctypes.byref(dev))
                a.src[i], a.dst[i] = d.data_ptr(), dev.value
                a.bytes[i] = d.numel() * d.element_size()
            cache[key] = a
        call('xa_copy_to_host', ctypes.byref(a), stream())

    def _sync_stats_copy(self):
        """The launch stream waits for a side-stream statistics copy still reading the
        rollout buffers (call before every rollout launch)."""
        ev = getattr(self, '_stats_guard', None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
            self._stats_guard = None

    def _fold_stats(self, slot, ev, gen=None):
        if ev is not None:
            ev.synchronize()
        if gen is not None:
            from xagents_amd._lib import XA_PPO_STATS_SLOTS
            slot = gen % XA_PPO_STATS_SLOTS
        if gen is None:
            host_done, host_epret, host_status = (self._host_done[slot], self._host_epret[slot],
                                                  getattr(self, '_host_status', None))
            host_status = host_status[slot] if host_status is not None else None
        else:
            # the update launch number `gen` stored this slot (checked: a launch the host
            # did not count would otherwise fold another step's statistics)
            host_done, host_epret, host_status = (self._fused_done[slot],
                                                  self._fused_epret[slot],
                                                  self._fused_host_status[slot])
            got = int(self._fused_gen[slot].item())
            # a launch that aborted (exchange timeout) may never have stored its slot: the
            # device status word names that cause, so it is checked before the slot's number
            if got != gen:
                status = getattr(self, 'device_status', None)
                if status is not None and int(status.max().item()):
                    raise RuntimeError(
                        f'{self.__class__.__name__}: an in-launch exchange of the persistent '
                        f'update timed out (device status word set); the parameters are '
                        f'invalid')
                raise RuntimeError(f'{self.__class__.__name__}: episode statistics slot {slot} '
                                   f'holds update launch {got}, expected {gen}')
        if getattr(self, 'device_status', None) is not None and host_status is not None and \
                int(host_status.max()):
            raise RuntimeError(
                f'{self.__class__.__name__}: an in-launch exchange of the persistent update '
                f'timed out (device status word set); the parameters are invalid')
        done = host_done.numpy()[:, 1:]
        epret = host_epret.numpy()
        t_idx, env_idx = np.nonzero(done.T)  # step-major, env-minor like step_envs
        finished = epret[env_idx, t_idx]
        if self.history_checkpoint:
            for ret in finished:
                self.update_history(ret)
        # (one extend, not a Python append per finished episode: at 256 envs ~1,300 episodes
        # end per train step, and the fold is host time on every step)
        self.total_rewards.extend(finished.astype(np.float64).tolist())
        self.games += len(finished)
        self.done_envs += len(finished)
        self.episode_rewards = epret[:, -1] * (1.0 - done[:, -1])
        self.dones = (done[:, -1] != 0).tolist()

    def _drain_episode_stats(self):
        if getattr(self, '_fused_pending', None):
            self._close_fused_group()
        while getattr(self, '_stats_queue', None):
            self._fold_item(self._stats_queue.pop(0))
        # a side-stream copy reads the status word before the step's update ends: the
        # last update's status is read here
        status = getattr(self, 'device_status', None)
        if status is not None and (getattr(self, '_stats_stream', None) is not None or
                                   getattr(self, '_stats_fused', False)) and \
                int(status.max().item()):
            raise RuntimeError(
                f'{self.__class__.__name__}: an in-launch exchange of the persistent update '
                f'timed out (device status word set); the parameters are invalid')

    def fit(
        self,
        target_reward=None,
        max_steps=None,
        monitor_session=None,
    ):
        assert (
            target_reward or max_steps
        ), '`target_reward` or `max_steps` should be specified when fit() is called'
        self.init_training(target_reward, max_steps, monitor_session)
        while True:
            self.check_episodes()
            if self._fit_done():
                break
            self.at_step_start()
            self.train_step()
            self.at_step_end()
        self._drain_episode_stats()

    def play(self, video_dir=None, render=False, frame_dir=None, frame_delay=0.0,
             max_steps=None, action_idx=0, frame_frequency=1):
        """Play one game of env 0 with the current policy (xagents/base.py:595-653): reset
        the envs, act with the agent's play policy (A2C / PPO: a Categorical sample of the
        actor, DQN: argmax Q, DDPG / TD3: the noise-free actor), stop at env 0's first done
        or after max_steps steps, display the total reward.

        The envs are device envs, stepped together in chunks (_play_chunk); env 0's
        rewards and dones are read back per chunk and the reference's per-step loop runs
        over them. Nothing is rendered: video_dir / render / frame_dir need gym's renderer
        and cv2, which this build has no counterpart of. Training counters (steps, games,
        total_rewards) are left untouched, as the reference's play leaves them. Returns the
        total reward (the reference returns None)."""
        if video_dir or render or frame_dir:
            raise NotImplementedError(
                'play(): device envs have no renderer (video_dir / render / frame_dir need '
                'gym and cv2)')
        del frame_delay, action_idx, frame_frequency  # rendering / multi-output options
        self.reset_envs()
        total_reward, steps = 0.0, 0
        while True:
            rewards, dones = self._play_chunk()
            for r, d in zip(rewards, dones):
                if max_steps and steps >= max_steps:
                    self.display_message(f'Maximum steps {max_steps} exceeded')
                    return total_reward
                total_reward += float(r)
                if d:
                    self.display_message(f'Total reward: {total_reward}')
                    return total_reward
                steps += 1

    def _play_chunk(self):
        """Step every env with the play policy for one or more steps; env 0's rewards and
        dones (host arrays, one entry per step, in step order)."""
        raise NotImplementedError(f'play() is not available for {type(self).__name__}')


class OnPolicy(BaseAgent, ABC):
    def __init__(self, envs, model, **kwargs):
        super(OnPolicy, self).__init__(envs, model, **kwargs)


class OffPolicy(BaseAgent, ABC):
    def __init__(
        self,
        envs,
        model,
        buffers,
        **kwargs,
    ):
        super(OffPolicy, self).__init__(envs, model, **kwargs)
        assert len(envs) == len(buffers), (
            f'Expected equal env and replay buffer sizes, got {self.n_envs} '
            f'and {len(buffers)}'
        )
        self.buffers = buffers

    # ---- device env stepping + replay append (step_envs(store_in_buffers=True)) ----
    _STATS_ROWS = 64

    def _setup_offpolicy(self, act_shape, act_dtype):
        """Device replay rings mirroring self.buffers, the fused env-step arguments and
        the per-step episode-stat rows copied back asynchronously."""
        import torch.distributed as dist
        from xagents_amd._lib import XaReplayStepArgs
        from xagents_amd.replay import DeviceReplay
        # data parallel over env shards: each rank samples its own buffers, gradients
        # are all-reduced (sum) and scaled by 1 / world before Adam
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        # ranks sharing one GPU (the multi-process tests) split its resident-workgroup
        # capacity for the persistent kernels (DDPG / TD3 fused step): collective, so once here
        self._ranks_share = 1
        if self.distributed and torch.device(self.device).type == 'cuda':
            from xagents_amd.comm import ranks_per_device
            self._ranks_share = ranks_per_device()
        env = self.envs
        self.replay = DeviceReplay(self.buffers, env.obs_shape, env.obs_dtype, act_shape,
                                   act_dtype, self.device)
        self._step_args = XaReplayStepArgs()
        env.fill_step_args(self._step_args)
        n, K = self.n_envs, self._STATS_ROWS
        # per step: [done row | episode-return row] (one copy per step fills both)
        self._st = torch.zeros(K, 2, n, dtype=torch.float32, device=self.device)
        self._st_done = self._st[:, 0]
        self._st_epret = self._st[:, 1]
        self._st_row = 0
        self._st_host = []

    def _env_step(self, actions, store=True):
        """One xa_replay_env_step: every env steps with `actions` (device) and, when
        `store`, appends its transition to its replay ring (xagents/base.py:388-426)."""
        from xagents_amd._lib import call, stream
        import ctypes
        a = self._step_args
        if store:
            self.replay.fill_step_args(a, actions)
        else:
            a.ring_states = None
            a.actions, a.act_bytes = actions.data_ptr(), self.replay.act_bytes
        r = self._st_row
        a.out_dones = self._st_done[r].data_ptr()
        a.done_epret = self._st_epret[r].data_ptr()
        pre_step = getattr(self.envs, 'pre_step', None)
        if pre_step is not None:
            # raw-frame env (AtariWrapper.step) / dynamics env (env.step with the actions)
            # into the one-step record
            pre_step(actions)
        call('xa_replay_env_step', ctypes.byref(a), stream())
        if store:
            self.replay.appended()
        self._st_row += 1
        if self._st_row == self._STATS_ROWS:
            self._flush_offpolicy_stats()

    def _play_actions(self):
        """Device actions of the play policy for every env (subclasses)."""
        raise NotImplementedError(f'play() is not available for {type(self).__name__}')

    def _play_chunk(self):
        """One xa_replay_env_step with the play policy's actions and no replay append;
        reward / done rows go to play-only buffers, so the training statistics rows and
        the rings are untouched."""
        from xagents_amd._lib import XaReplayStepArgs, call, stream
        import ctypes
        if getattr(self, '_play_args', None) is None:
            n = self.n_envs
            self._play_out = torch.zeros(3, n, dtype=torch.float32, device=self.device)
            a = XaReplayStepArgs()
            self.envs.fill_step_args(a)
            a.ring_states = None
            o = self._play_out
            a.out_rewards, a.out_dones = o[0].data_ptr(), o[1].data_ptr()
            a.done_epret = o[2].data_ptr()
            self._play_args = a
        a = self._play_args
        actions = self._play_actions()
        a.actions, a.act_bytes = actions.data_ptr(), self.replay.act_bytes
        pre_step = getattr(self.envs, 'pre_step', None)
        if pre_step is not None:
            pre_step(actions)
        call('xa_replay_env_step', ctypes.byref(a), stream())
        out = self._play_out[:2, 0].cpu().numpy()
        return out[:1], out[1:]

    def _device_checks(self):
        """Raise on an error a persistent launch reported through its device status word
        (subclasses; called with every statistics flush, so no extra sync per step)."""

    def _flush_offpolicy_stats(self):
        self._device_checks()
        rows = self._st_row
        if rows == 0:
            return
        h = torch.empty(rows, 2, self.n_envs).pin_memory()
        h.copy_(self._st[:rows], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._st_host.append((h[:, 0], h[:, 1], ev))
        self._st_row = 0
        while len(self._st_host) > 1:
            self._fold_offpolicy_stats(*self._st_host.pop(0))

    def _fold_offpolicy_stats(self, hd, he, ev):
        ev.synchronize()
        d, e = hd.numpy(), he.numpy()
        for t in range(d.shape[0]):  # step-major, env-minor like step_envs
            for i in np.nonzero(d[t])[0]:
                if self.history_checkpoint:
                    self.update_history(float(e[t, i]))
                self.total_rewards.append(float(e[t, i]))
                self.games += 1
                self.done_envs += 1

    def _drain_episode_stats(self):
        super()._drain_episode_stats()
        if hasattr(self, '_st_host'):
            self._flush_offpolicy_stats()
            while self._st_host:
                self._fold_offpolicy_stats(*self._st_host.pop(0))

    def _sync_params(self, *models):
        if self.distributed:
            import torch.distributed as dist
            for m in models:
                dist.broadcast(m.theta, 0)

    def _reduce_grad(self, grad, mean=False):
        """All-reduce (sum) a gradient over the data-parallel ranks; returns Adam's
        grad_scale so the step equals one process on the union of the ranks' batches:
        1 for losses summed over the batch (Keras MSE + minimize: DQN, the critics,
        dqn/agent.py:170-171, ddpg/agent.py:126-127), 1 / world for batch means (the
        actor's -mean Q, ddpg/agent.py:97-100) when every rank samples the same count."""
        if not self.distributed:
            return 1.0
        import torch.distributed as dist
        dist.all_reduce(grad)
        return 1.0 / self.world_size if mean else 1.0

    def _all_gather_host(self, arr):
        """Concatenation over the ranks (rank-major) of a small host array."""
        import torch.distributed as dist
        parts = [None] * self.world_size
        dist.all_gather_object(parts, np.asarray(arr))
        return np.concatenate(parts)

    def _fill_action_plan(self):
        """The random actions of fill_buffers in the reference's draw order: env 0's
        action_space.sample() calls until its buffer is full, then env 1's, ...
        (xagents/base.py:702-730); [max missing, n_envs, *act] plus each env's count."""
        space = self.envs[0].action_space
        need = [max(b.initial_size - b.current_size, 0) for b in self.buffers]
        seqs = [[np.asarray(space.sample()) for _ in range(k)] for k in need]
        width = max(need) if need else 0
        proto = np.asarray(space.sample()) if width else None
        plan = None
        if width:
            plan = np.zeros((width, self.n_envs) + proto.shape, proto.dtype)
            for i, seq in enumerate(seqs):
                if seq:
                    plan[:len(seq), i] = np.stack(seq)
        return plan, need

    def fill_buffers(self):
        """Random actions until each buffer holds initial_size transitions
        (xagents/base.py:702-730), then reset the envs. The actions are drawn env by env
        in the reference's order (_fill_action_plan); the device then steps every env
        together (an env that needed fewer than another takes action 0 on the extra
        steps, which leaves the draw order unchanged)."""
        total = sum(b.initial_size for b in self.buffers)
        plan, need = self._fill_action_plan()
        step = 0
        while min(b.current_size - b.initial_size for b in self.buffers) < 0:
            acts = torch.as_tensor(plan[min(step, len(plan) - 1)], device=self.device)
            acts = acts.to(self.replay.act_t).contiguous()
            self._env_step(acts)
            step += 1
            filled = sum(min(b.current_size, b.initial_size) for b in self.buffers)
            complete = round((filled / total) * 100, self.display_precision)
            self.display_message(
                f'\rFilling replay buffer ==> {complete}% | {filled}/{total}', end='')
        self.display_message('')
        self._drain_episode_stats()
        self.total_rewards.clear()
        self.games = self.done_envs = 0
        self.reset_envs()

    def fit(self, target_reward=None, max_steps=None, monitor_session=None):
        self.fill_buffers()
        super(OffPolicy, self).fit(target_reward, max_steps, monitor_session)
