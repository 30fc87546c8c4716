"""Host-side profile of the C3 train step (DQN Pong-shaped, 32 envs, double, RB1 1M): the
bench's agent, 10 warm-up steps, then cProfile over 30 steps (sorted by own time) and the
wall time per step with and without a device sync each step.
usage: python tools/c3_host_profile.py"""
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
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    dev = torch.device('cuda')
    n = 32
    envs = create_envs('PongNoFrameskip-v4', n, device=dev, seed=55)
    model = create_model(envs, 'dqn', 'model', seed=55, device=dev)
    bufs = create_buffers('dqn', 1_000_000, 64, n, initial_size=1_000_000)
    agent = DQN(envs, model, bufs, double=True, seed=55, quiet=True, epsilon_start=0.02,
                epsilon_end=0.02)
    agent.fill_buffers()

    def step():
        agent.at_step_start()
        agent.train_step()
        agent.at_step_end()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    for label, sync in (('no sync', False), ('sync per step', True)):
        t = time.perf_counter()
        for _ in range(30):
            step()
            if sync:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print(f'{label}: {(time.perf_counter() - t) / 30 * 1e6:.1f} us per step')
    # host time alone per phase (each followed by a sync, so only the host part differs)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(30)
    print(s.getvalue())


if __name__ == '__main__':
    main()
