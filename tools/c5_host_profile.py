"""Host-side profile of the C5 train step (TD3 BipedalWalker-shaped, 64 envs, RB2, gradient
steps on finished episodes): the bench's agent, 10 warm-up steps, wall time per step with and
without a device sync each step, then cProfile over 60 steps (sorted by own time).
usage: python tools/c5_host_profile.py"""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    dev = torch.device('cuda')
    n = 64
    envs = create_envs('BipedalWalker-v3', n, device=dev, seed=55)
    kw = dict(seed=55, device=dev)
    actor = create_model(envs, 'td3', 'actor_model', **kw)
    critic = create_model(envs, 'td3', 'critic_model', **kw)
    bufs = create_buffers('td3', 1_000_000, 100, n, initial_size=n * 64)
    agent = TD3(envs, actor, critic, bufs, gradient_steps=1, seed=55, quiet=True)
    agent.fill_buffers()
    for _ in range(10):
        agent.train_step()
    torch.cuda.synchronize()
    for label, sync in (('no sync', False), ('sync per step', True)):
        t = time.perf_counter()
        for _ in range(60):
            agent.train_step()
            if sync:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print(f'{label}: {(time.perf_counter() - t) / 60 * 1e6:.1f} us per step', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(60):
        agent.train_step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(35)
    print(s.getvalue())


if __name__ == '__main__':
    main()
