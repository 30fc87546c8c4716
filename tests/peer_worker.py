"""Worker for tests/test_gpu_peer.py: W processes on ONE HIP device (the test box has one
GPU), a gloo process group for the handle exchange and the expected values.

Checks, per rank:
  1. eager xa_peer_allreduce of f32 (4675 = the CartPole gradient) and f64 (256 = the
     advantage sums) buffers equals the rank-ordered float64-free sum of every rank's
     input, bit for bit, over many epochs (both slots reused);
  2. the same inside a captured hipGraph replayed several times;
  3. a rank that skips an exchange makes the others time out: they set the sticky
     error, return without waiting, and healthy_everywhere() reports it on every rank.
Prints 'PEER OK <rank>' at the end.
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def expected_sum(local, world):
    """Rank-ordered sum of every rank's tensor, computed with the tensor's own dtype."""
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    acc = parts[0].clone()
    for p in range(1, world):
        acc += parts[p]
    return acc


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from xagents_amd.comm import PeerAllReduce

    peer = PeerAllReduce(timeout_s=20.0)
    dev = torch.device('cuda', 0)
    gen = torch.Generator().manual_seed(1234 + rank)

    # 1. eager, both dtypes, several epochs
    for it in range(12):
        for dtype, n in ((torch.float32, 4675), (torch.float64, 256), (torch.float32, 3)):
            host = torch.randn(n, generator=gen, dtype=dtype)
            want = expected_sum(host, world)
            t = host.to(dev)
            peer.all_reduce(t)
            got = t.cpu()
            assert torch.equal(got, want), f'rank {rank} it {it} {dtype} n={n}: mismatch'
    epoch, err = peer.status()
    assert err == 0 and epoch == 36, (epoch, err)  # every call touches chunk 0

    # 1b. with the optimizer tail: == the exchange followed by xa_clip_adam, bit for bit
    from xagents_amd import kernels
    P = 4675
    base = torch.randn(3, P, generator=torch.Generator().manual_seed(99))  # same on all ranks
    th, m, v = (x.to(dev) for x in (base[0], base[1] * 1e-3, base[2].abs() * 1e-5))
    th_r, m_r, v_r = th.clone(), m.clone(), v.clone()
    step = torch.tensor([3], dtype=torch.int32, device=dev)
    step_r = step.clone()
    arrivals = torch.zeros(1, dtype=torch.int32, device=dev)
    tail = kernels.adam_tail(th, m, v, step, arrivals, 7e-4, 0.9, 0.999, 1e-7, clip_norm=0.5,
                             bump=False)
    for it in range(3):
        host = torch.randn(P, generator=gen) * 1e-2
        want = expected_sum(host, world).to(dev)
        kernels.clip_adam(th_r, m_r, v_r, want, step_r, 7e-4, 0.9, 0.999, 1e-7, clip_norm=0.5)
        t = host.to(dev)
        peer.all_reduce(t, tail=tail)
        torch.cuda.synchronize()
        assert torch.equal(t, want), f'rank {rank} tail it {it}: sum mismatch'
        for a, b, name in ((th, th_r, 'theta'), (m, m_r, 'm'), (v, v_r, 'v')):
            assert torch.equal(a, b), f'rank {rank} tail it {it}: {name} mismatch'
        assert int(arrivals.item()) == 0

    # 2. captured into a graph, replayed
    buf = torch.zeros(4675, dtype=torch.float32, device=dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        peer.all_reduce(buf)  # warm-up launch outside capture
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        peer.all_reduce(buf)
    for it in range(8):
        host = torch.randn(4675, generator=gen)
        want = expected_sum(host, world)
        buf.copy_(host.to(dev))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(buf.cpu(), want), f'rank {rank} graph replay {it}: mismatch'
    assert peer.healthy_everywhere()

    if os.environ.get('PEER_TIMING') == '1':
        # latency of a graph of 16 back-to-back exchanges (ranks share one GPU here)
        g16 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g16):
            for _ in range(16):
                peer.all_reduce(buf)
        for _ in range(3):
            g16.replay()
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            g16.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f'PEER TIMING rank {rank} world {world}: '
              f'{e0.elapsed_time(e1) * 1e3 / (50 * 16):.2f} us per exchange', flush=True)
        assert peer.healthy_everywhere()

    # 3. timeout path: the last rank skips one exchange
    if world > 1:
        peer._args.timeout_ticks = int(0.3 * 1e8)
        x = torch.ones(64, device=dev)
        if rank != world - 1:
            peer.all_reduce(x)
        torch.cuda.synchronize()
        ok = peer.healthy_everywhere()
        assert not ok, 'a skipped exchange must surface as an error on every rank'
        if rank != world - 1:
            assert peer.status()[1] == 1 + (world - 1), peer.status()
            assert torch.equal(x.cpu(), torch.ones(64)), 'timed-out call must leave local values'
            # sticky: the next call returns at once with local values
            y = torch.full((8,), 2.0, device=dev)
            peer.all_reduce(y)
            assert torch.equal(y.cpu(), torch.full((8,), 2.0))
    peer.close()
    dist.destroy_process_group()
    print(f'PEER OK {rank}', flush=True)


if __name__ == '__main__':
    main()
