"""Host replay buffers with the observable behaviour of xagents/utils/buffers.py.

Kept behaviours (pinned by tests/golden/buffers_*.npz, generated from the
reference module itself):
* size validation and its assertion messages (buffers.py:21-30);
* ReplayBuffer1: a bounded deque sampled with random.sample; a 1-element sample is
  returned as the stored tuple itself, not as per-field arrays (buffers.py:95-98);
* ReplayBuffer2: per-field numpy rings allocated lazily on the first append, write
  row = current_size % size with current_size saturating at size -- so after the
  ring fills every append lands on row 0 (buffers.py:128-135); samples draw
  np.random.randint(0, filled, batch) (buffers.py:145-148).
The device-resident replay rings used by the off-policy fused path follow the same
rules.
"""
import random
from collections import deque

import numpy as np

_SIZE_RULES = (
    (lambda s, i, b: i is None or i > 0, 'Buffer initial size should be > 0, got {i}'),
    (lambda s, i, b: s > 0, 'Buffer size should be > 0,  got {s}'),
    (lambda s, i, b: b > 0, 'Buffer batch size should be > 0, got {b}'),
    (lambda s, i, b: b <= s, 'Buffer batch size `{b}` should be <= size `{s}`'),
    (lambda s, i, b: not i or s >= i, 'Buffer initial size exceeds max size'),
)


class BaseBuffer:
    def __init__(self, size, initial_size=None, batch_size=32):
        for rule, message in _SIZE_RULES:
            assert rule(size, initial_size, batch_size), message.format(
                s=size, i=initial_size, b=batch_size)
        self.size = size
        self.initial_size = initial_size if initial_size else size
        self.batch_size = batch_size
        self.current_size = 0

    def _abstract(self, name):
        raise NotImplementedError(
            f'{name}() should be implemented by {type(self).__name__} subclasses')

    def append(self, *args):
        self._abstract('append')

    def get_sample(self):
        self._abstract('get_sample')


class ReplayBuffer1(BaseBuffer):
    """Transitions stored as tuples in a bounded deque."""

    def __init__(self, size, **kwargs):
        super().__init__(size, **kwargs)
        self.main_buffer = deque(maxlen=size)
        self.temp_buffer = []

    def append(self, *args):
        self.main_buffer.append(args)
        self.current_size = min(self.current_size + 1, self.size)

    def get_sample(self):
        picked = random.sample(self.main_buffer, self.batch_size)
        if self.batch_size == 1:
            return picked[0]
        fields = len(picked[0])
        return [np.array([row[f] for row in picked]) for f in range(fields)]


class ReplayBuffer2(BaseBuffer):
    """One preallocated numpy ring per transition field."""

    def __init__(self, size, slots, **kwargs):
        super().__init__(size, **kwargs)
        self.slots = [np.array([]) for _ in range(slots)]
        self.current_size = 0

    def _ensure_ring(self, field, value):
        if self.slots[field].shape[0] == 0:
            self.slots[field] = np.zeros((self.size,) + value.shape, value.dtype)

    def append(self, *args):
        row = self.current_size % self.size
        for field, value in enumerate(args):
            value = value if isinstance(value, np.ndarray) else np.array([value])
            self._ensure_ring(field, value)
            self.slots[field][row] = value.copy()
        self.current_size = min(self.current_size + 1, self.size)

    def get_sample(self):
        filled = min(self.current_size, self.size)
        rows = np.random.randint(0, filled, self.batch_size)
        return [ring[rows] for ring in self.slots]
