"""Device replay rings behind the reference's per-env buffer objects.

The reference keeps one ReplayBuffer1 (deque + random.sample) or ReplayBuffer2 (numpy
rings) per env (xagents/utils/buffers.py:59-148, created by create_buffers,
xagents/utils/common.py:515-565). Here the transitions of all envs live in HBM rings
[n_envs, size, ...]; `xa_replay_env_step` appends one transition per env per step and
`xa_ring_gather` assembles a sampled batch in concat_buffer_samples order
(xagents/base.py:344-368: env-major, k samples per env).

The index semantics stay the reference's and are computed on the host, consuming the
same RNG streams in the same order:
* RB1: deque order (oldest first), `random.sample(deque, k)` -> positions, mapped to
  ring slots (start + pos) % size;
* RB2: write row current_size % size with current_size saturating at size (so every
  append after the ring fills lands on row 0, buffers.py:133-135), samples
  `np.random.randint(0, min(current_size, size), k)`.
The per-env buffer objects passed in keep their `current_size` attribute in step.
"""
import random

import numpy as np
import torch

from xagents_amd._lib import XA_RING_DEQUE, XA_RING_RB2, call, stream
from xagents_amd.utils.buffers import ReplayBuffer1, ReplayBuffer2


class DeviceReplay:
    def __init__(self, buffers, obs_shape, obs_dtype, act_shape, act_dtype, device):
        b0 = buffers[0]
        assert all(type(b) is type(b0) and b.size == b0.size and b.batch_size == b0.batch_size
                   for b in buffers), 'device replay needs identical per-env buffers'
        self.buffers = buffers
        self.kind = XA_RING_RB2 if isinstance(b0, ReplayBuffer2) else XA_RING_DEQUE
        if not isinstance(b0, (ReplayBuffer1, ReplayBuffer2)):
            raise TypeError(f'unsupported buffer type {type(b0).__name__}')
        self.n = len(buffers)
        self.cap = b0.size
        self.k = b0.batch_size
        self.device = device
        n, cap = self.n, self.cap
        tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.float32): torch.float32,
               np.dtype(np.int32): torch.int32}
        self.obs_t = tdt[np.dtype(obs_dtype)]
        self.act_t = tdt[np.dtype(act_dtype)]
        self.obs_shape, self.act_shape = tuple(obs_shape), tuple(act_shape)
        self.states = torch.zeros((n, cap) + self.obs_shape, dtype=self.obs_t, device=device)
        self.new_states = torch.zeros_like(self.states)
        self.actions = torch.zeros((n, cap) + self.act_shape, dtype=self.act_t, device=device)
        self.rewards = torch.zeros(n, cap, dtype=torch.float32, device=device)
        self.dones = torch.zeros(n, cap, dtype=torch.float32, device=device)
        self.count = torch.zeros(n, dtype=torch.int64, device=device)
        self.host_count = np.zeros(n, np.int64)
        self.obs_bytes = self.states[0, 0].numel() * self.states.element_size()
        self.act_bytes = max(self.actions[0, 0].numel(), 1) * self.actions.element_size()
        self._pinned = [torch.empty(n * self.k, dtype=torch.int64).pin_memory() for _ in range(2)]
        self._pin_ev = [None, None]
        self._pin_slot = 0
        self.slots = torch.zeros(n * self.k, dtype=torch.int64, device=device)

    # ---- append (device) + host mirror -----------------------------------------
    def fill_step_args(self, a, actions):
        a.actions, a.act_bytes = actions.data_ptr(), self.act_bytes
        a.capacity, a.ring_kind, a.ring_count = self.cap, self.kind, self.count.data_ptr()
        a.ring_states, a.ring_new_states = self.states.data_ptr(), self.new_states.data_ptr()
        a.ring_actions = self.actions.data_ptr()
        a.ring_rewards, a.ring_dones = self.rewards.data_ptr(), self.dones.data_ptr()

    def appended(self):
        """Mirror one append per env (the kernel's counter rule)."""
        if self.kind == XA_RING_RB2:
            self.host_count = np.minimum(self.host_count + 1, self.cap)
        else:
            self.host_count = self.host_count + 1
        size = np.minimum(self.host_count, self.cap)
        for b, s in zip(self.buffers, size):
            b.current_size = int(s)

    def reset_counts(self):
        self.count.zero_()
        self.host_count[:] = 0
        for b in self.buffers:
            b.current_size = 0

    # ---- sampling -------------------------------------------------------------
    def sample_slots(self):
        """Ring slots of one concat_buffer_samples batch (env-major), reference RNG."""
        out = np.empty(self.n * self.k, np.int64)
        if self.kind == XA_RING_RB2 and (self.host_count == self.host_count[0]).all():
            # equal sizes: one randint(0, size, n k) draws the same legacy-RNG values as the
            # reference's n sequential randint(0, size, k) calls (tests/test_host.py)
            size = min(int(self.host_count[0]), self.cap)
            idx = np.random.randint(0, size, self.n * self.k).astype(np.int64)
            return np.repeat(np.arange(self.n, dtype=np.int64) * self.cap, self.k) + idx
        for i in range(self.n):
            cnt = int(self.host_count[i])
            if self.kind == XA_RING_RB2:
                idx = np.random.randint(0, min(cnt, self.cap), self.k)
            else:
                length = min(cnt, self.cap)
                pos = np.asarray(random.sample(range(length), self.k), np.int64)
                idx = ((cnt - length) + pos) % self.cap
            out[i * self.k:(i + 1) * self.k] = i * self.cap + idx
        return out

    def upload_slots(self, slots):
        s = self._pin_slot
        if self._pin_ev[s] is not None:
            self._pin_ev[s].synchronize()
        self._pinned[s].numpy()[:] = slots
        self.slots.copy_(self._pinned[s], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pin_ev[s] = ev
        self._pin_slot ^= 1
        return self.slots

    def gather(self, slots, states, actions, rewards, dones, new_states):
        m = slots.numel()
        sp = slots.data_ptr()
        for ring, dst, nb in ((self.states, states, self.obs_bytes),
                              (self.new_states, new_states, self.obs_bytes),
                              (self.actions, actions, self.act_bytes),
                              (self.rewards, rewards, 4), (self.dones, dones, 4)):
            call('xa_ring_gather', ring.data_ptr(), dst.data_ptr(), sp, m, nb, stream())
