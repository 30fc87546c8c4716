"""Peer all-reduce for the data-parallel update's small exchanges.

Per optimizer step the update all-reduces the flat gradient (18.7 KB for the CartPole
actor-critic) and, per train step, the advantage sums (2 KB). At these sizes an RCCL
ring is latency: 2(W-1) dependent hops over xGMI. `PeerAllReduce` instead maps every
rank's IPC-exported, uncached HBM block into every process once; each exchange is one
kernel (`xa_peer_allreduce`, csrc/comm.hip) that pushes the local values into every
peer's block as 8-byte (word, epoch) pairs, polls its own block until all W ranks'
pairs carry the current epoch (so it waits for data, not for a separate flag) and
sums them in rank order, so all ranks get identical bits. Larger tensors (the CNN's
77 MB gradient) stay on RCCL, where bandwidth, not latency, is what matters.

Waits inside the kernel are bounded; a timeout leaves a sticky error that
`healthy_everywhere()` reads, and callers then fall back to `dist.all_reduce`.
"""
import ctypes
import os
import warnings

import torch
import torch.distributed as dist

from xagents_amd import _lib
from xagents_amd._lib import XA_DTYPE_F32, XA_DTYPE_F64, XaPeerAllReduceArgs, call

DEFAULT_SLOT_BYTES = 64 * 1024
CHUNK_BYTES = 4096  # payload bytes per workgroup of xa_peer_allreduce
REALTIME_HZ = 100_000_000  # s_memrealtime clock


class PeerAllReduce:
    """IPC peer blocks of one process group; `all_reduce(t)` is an in-place SUM."""

    def __init__(self, group=None, slot_bytes=DEFAULT_SLOT_BYTES, timeout_s=30.0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > _lib.XA_PEER_MAX:
            raise ValueError(f'peer all-reduce supports at most {_lib.XA_PEER_MAX} ranks')
        self.slot_bytes = (int(slot_bytes) + CHUNK_BYTES - 1) // CHUNK_BYTES * CHUNK_BYTES
        lib = _lib.load()
        self.device = torch.device('cuda', torch.cuda.current_device())
        self.state = torch.zeros(lib.xa_peer_state_words(self.slot_bytes), dtype=torch.int32,
                                 device=self.device)
        self._own = ctypes.c_void_p()
        self._opened = []
        call('xa_peer_block_alloc', lib.xa_peer_block_bytes(self.slot_bytes, self.world),
             ctypes.byref(self._own))
        handle = (ctypes.c_char * 64)()
        call('xa_peer_ipc_handle', self._own, handle)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle), group=group)
        args = XaPeerAllReduceArgs()
        args.rank, args.world = self.rank, self.world
        args.slot_bytes = self.slot_bytes
        args.state = self.state.data_ptr()
        args.timeout_ticks = int(timeout_s * REALTIME_HZ)
        for p, h in enumerate(handles):
            if p == self.rank:
                args.blocks[p] = self._own.value
                continue
            blk = ctypes.c_void_p()
            buf = (ctypes.c_char * 64).from_buffer_copy(h)
            call('xa_peer_ipc_open', buf, ctypes.byref(blk))
            self._opened.append(blk)
            args.blocks[p] = blk.value
        self._args = args
        # every rank has mapped every block before the first push
        dist.barrier(group=group)

    def fits(self, t):
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.float64)
                and t.numel() * t.element_size() <= self.slot_bytes
                and t.data_ptr() % 8 == 0 and t.device == self.device)

    def all_reduce(self, t, tail=None):
        """In-place SUM of `t` over the group, asynchronous on torch's current stream
        (capturable into a hipGraph: the epoch lives in device memory). `tail` (an
        XaAdamTail, f32 gradients) applies clip + Keras Adam to the sum in the same
        launch."""
        a = self._args
        a.has_tail = int(tail is not None)
        if tail is not None:
            a.tail = tail
        a.dtype = XA_DTYPE_F64 if t.dtype == torch.float64 else XA_DTYPE_F32
        a.count = t.numel()
        a.src = a.dst = t.data_ptr()
        call('xa_peer_allreduce', ctypes.byref(a), _lib.stream())
        return t

    def status(self):
        """(epoch of chunk 0, error) of this rank; synchronizes the device. error 0 =
        healthy, 1 + p = an exchange timed out waiting for rank p."""
        st = self.state.cpu()
        return int(st[1]), int(st[0])

    def healthy_everywhere(self):
        """True iff no rank's block holds a timeout error (collective over the group)."""
        err = torch.tensor([float(self.status()[1] != 0)], dtype=torch.float64,
                           device=self.device)
        if dist.get_backend(self.group) == 'gloo':
            err = err.cpu()
        dist.all_reduce(err, op=dist.ReduceOp.MAX, group=self.group)
        return float(err.item()) == 0.0

    def close(self):
        """Unmap the peers' blocks, then (after every rank did) free this rank's."""
        if self._own is None:
            return
        torch.cuda.synchronize()
        for blk in self._opened:
            call('xa_peer_ipc_close', blk)
        self._opened = []
        dist.barrier(group=self.group)
        call('xa_peer_block_free', self._own)
        self._own = None


class PeerBlocks:
    """One uncached HBM block per rank of the default group, IPC-mapped into every rank
    (the exchange memory of the data-parallel persistent PPO update, csrc/ppo_update.hip);
    `pointers[r]` is rank r's block as this process addresses it. Zeroed at allocation."""

    def __init__(self, nbytes, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._own = ctypes.c_void_p()
        self._opened = []
        call('xa_peer_block_alloc', int(nbytes), ctypes.byref(self._own))
        handle = (ctypes.c_char * 64)()
        call('xa_peer_ipc_handle', self._own, handle)
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(handle), group=group)
        self.pointers = []
        for p, h in enumerate(handles):
            if p == self.rank:
                self.pointers.append(self._own.value)
                continue
            blk = ctypes.c_void_p()
            call('xa_peer_ipc_open', (ctypes.c_char * 64).from_buffer_copy(h), ctypes.byref(blk))
            self._opened.append(blk)
            self.pointers.append(blk.value)
        dist.barrier(group=group)

    def close(self):
        if self._own is None:
            return
        torch.cuda.synchronize()
        for blk in self._opened:
            call('xa_peer_ipc_close', blk)
        self._opened = []
        dist.barrier(group=self.group)
        call('xa_peer_block_free', self._own)
        self._own = None


def ranks_per_device(group=None):
    """The largest number of ranks of the group that share one physical device (1 on a
    node with one process per GPU; > 1 when ranks share a GPU, as the tests do)."""
    import socket
    key = (socket.gethostname(), torch.cuda.current_device())
    keys = [None] * dist.get_world_size(group)
    dist.all_gather_object(keys, key, group=group)
    return max(keys.count(k) for k in keys)


def maybe_peer_all_reduce(world_size):
    """A PeerAllReduce for the default group when data-parallel on HIP devices and not
    disabled (XA_PEER_ALLREDUCE=0); None (use RCCL) if the IPC setup fails."""
    if world_size <= 1 or os.environ.get('XA_PEER_ALLREDUCE', '1') == '0':
        return None
    if not torch.cuda.is_available():
        return None
    try:
        return PeerAllReduce(timeout_s=float(os.environ.get('XA_PEER_TIMEOUT_S', '30')))
    except Exception as exc:  # IPC unavailable on this node: RCCL carries the exchange
        warnings.warn(f'peer all-reduce unavailable ({exc}); using RCCL all_reduce')
        return None
