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
import ctypes
import math
import random

import numpy as np
import torch

from xagents_amd._lib import XA_RING_DEQUE, XA_RING_RB2, XaGatherArgs, call, stream
from xagents_amd.utils.buffers import ReplayBuffer1, ReplayBuffer2


def _sample_range(n, k, getrandbits):
    """random.sample(range(n), k) on the module RNG, drawn through getrandbits directly: the
    same algorithm, the same draws and the same results as CPython's Random.sample with
    _randbelow_with_getrandbits (Lib/random.py, 3.8-3.12: a pool of n items when n is at
    most the small-set size, else rejection against the selected set), minus the per-call
    overhead (C3's 32 per-env samples took ~100 us of host time per train step through
    random.sample; tests/test_host.py checks the identity and the RNG state after)."""
    if not 0 <= k <= n:
        raise ValueError('Sample larger than population or is negative')
    setsize = 21
    if k > 5:
        setsize += 4 ** math.ceil(math.log(k * 3, 4))
    out = []
    if n <= setsize:
        pool = list(range(n))
        for i in range(k):
            m = n - i
            b = m.bit_length()
            r = getrandbits(b)
            while r >= m:
                r = getrandbits(b)
            out.append(pool[r])
            pool[r] = pool[m - 1]
    else:
        b = n.bit_length()
        sel = set()
        for _ in range(k):
            r = getrandbits(b)
            while r >= n or r in sel:
                r = getrandbits(b)
            sel.add(r)
            out.append(r)
    return out


def _sample_ranges(lengths, k, getrandbits):
    """[random.sample(range(n), k) for n in lengths], flattened, as _sample_range draws them;
    the k = 2 set case (C3's per-env batch of 2) inline."""
    out = []
    if k == 2:
        for n in lengths:
            if n <= 21:
                out.extend(_sample_range(n, 2, getrandbits))
                continue
            b = n.bit_length()
            r0 = getrandbits(b)
            while r0 >= n:
                r0 = getrandbits(b)
            r1 = getrandbits(b)
            while r1 >= n or r1 == r0:
                r1 = getrandbits(b)
            out.append(r0)
            out.append(r1)
        return out
    for n in lengths:
        out.extend(_sample_range(n, k, getrandbits))
    return out


def _fast_sampler():
    """_sample_ranges bound to the module RNG when that RNG draws through getrandbits (the
    stock random.Random); None otherwise (callers then use random.sample)."""
    inst = random._inst
    rb = getattr(type(inst), '_randbelow', None)
    if rb is not getattr(random.Random, '_randbelow_with_getrandbits', object()):
        return None
    gb = inst.getrandbits
    return lambda lengths, k: _sample_ranges(lengths, k, gb)


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
        self._stage = None  # the staged (mapped pinned) slots, allocated on first use

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
        size = np.minimum(self.host_count, self.cap).tolist()  # Python ints in one call
        for b, s in zip(self.buffers, size):
            b.current_size = s

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
        if self.kind != XA_RING_RB2:
            cnt = self.host_count
            length = np.minimum(cnt, self.cap)
            fast = _fast_sampler()
            if fast:
                pos = np.asarray(fast(length.tolist(), self.k), np.int64)
            else:
                pos = np.asarray([q for n in length.tolist()
                                  for q in random.sample(range(n), self.k)], np.int64)
            idx = (np.repeat(cnt - length, self.k) + pos) % self.cap
            return np.repeat(np.arange(self.n, dtype=np.int64) * self.cap, self.k) + idx
        for i in range(self.n):
            cnt = int(self.host_count[i])
            idx = np.random.randint(0, min(cnt, self.cap), self.k)
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

    # ---- staged slots: the consuming launch reads them from mapped pinned memory ------
    def stage_ptr(self):
        """Device address of the mapped pinned buffer the staged slots live in (fixed for
        the buffer's life, so a captured hipGraph may read it)."""
        if self._stage is None:
            from xagents_amd._lib import call as _call
            self._stage = torch.zeros(self.n * self.k, dtype=torch.int64).pin_memory()
            dp = ctypes.c_void_p()
            _call('xa_host_device_pointer', ctypes.c_void_p(self._stage.data_ptr()),
                  ctypes.byref(dp))
            self._stage_dev = dp.value
            self._stage_ev = torch.cuda.Event()
            self._stage_open = False
        return self._stage_dev

    def stage_slots(self, slots):
        """The next batch's slots into the staged buffer (no upload copy: the gather reads
        them over the host link, 8 B per sampled item). The previous batch's consumer must
        have run: its completion event (stage_consumed) is waited for first; without one the
        whole stream is (safe, slower)."""
        self.stage_ptr()
        if self._stage_open:
            torch.cuda.current_stream().synchronize()
        else:
            self._stage_ev.synchronize()
        self._stage.numpy()[:] = slots
        self._stage_open = True
        return self._stage_dev

    def stage_consumed(self):
        """Call right after enqueueing the launch (or graph replay) that read the staged
        slots."""
        self._stage_ev.record()
        self._stage_open = False

    def gather(self, slots, states, actions, rewards, dones, new_states):
        """The five fields of one sampled batch in one xa_ring_gather_fields launch (the
        argument block is built once per destination set and reused). slots: a device
        int64 tensor, or an (address, count) pair (the staged slots)."""
        if isinstance(slots, tuple):
            sp, sn = slots
        else:
            sp, sn = slots.data_ptr(), slots.numel()
        key = (sp, sn, states.data_ptr(), actions.data_ptr(),
               rewards.data_ptr(), dones.data_ptr(), new_states.data_ptr())
        if getattr(self, '_gkey', None) != key:
            a = XaGatherArgs()
            fields = ((self.states, states, self.obs_bytes),
                      (self.new_states, new_states, self.obs_bytes),
                      (self.actions, actions, self.act_bytes),
                      (self.rewards, rewards, 4), (self.dones, dones, 4))
            for f, (ring, dst, nb) in enumerate(fields):
                a.field[f].ring, a.field[f].dst, a.field[f].item_bytes = \
                    ring.data_ptr(), dst.data_ptr(), nb
            a.n_fields, a.n_items, a.slots = len(fields), sn, sp
            self._gargs, self._gkey = a, key
        call('xa_ring_gather_fields', ctypes.byref(self._gargs), stream())
