"""C5 (TD3, 64 BipedalWalker-shaped envs, ReplayBuffer2) gradient steps alone, for a
rocprofv3 kernel trace of one gradient step's launches (tools/gpu_steps.sh profc5).

usage: python tools/td3_grad_steps.py [n_steps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch
    from xagents_amd import TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = 64
    np.random.seed(55)
    envs = create_envs('BipedalWalker-v3', n, device='cuda', seed=55)
    kw = dict(seed=55, device='cuda')
    actor = create_model(envs, 'td3', 'actor_model', **kw)
    critic = create_model(envs, 'td3', 'critic_model', **kw)
    bufs = create_buffers('td3', 1_000_000, 100, n, initial_size=n * 64)
    agent = TD3(envs, actor, critic, bufs, gradient_steps=1, seed=55, quiet=True)
    agent.fill_buffers()
    for _ in range(10):
        agent.update_weights(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        agent.update_weights(1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n_steps
    print(f'TD3 gradient step: {dt * 1e3:.4f} ms ({n_steps} steps, graph replay)', flush=True)


if __name__ == '__main__':
    main()
