"""ACER train-step breakdown on the bench workload (Pong-shaped, 16 envs x 20 steps):
rollout vs updates, HIP events on the launch stream, mean over 10 steps after 3 warm-ups."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import ACER
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    dev = torch.device('cuda')
    n = 16
    envs = create_envs('PongNoFrameskip-v4', n, device=dev, seed=55)
    model = create_model(envs, 'acer', 'model', seed=55, device=dev)
    agent = ACER(envs, model, create_buffers('acer', 64 * n, 1, n, initial_size=n), n_steps=20,
                 seed=55, quiet=True, grad_norm=10.0)
    np.random.seed(55)
    for _ in range(3):
        agent.train_step()
    tr, tu, nu = 0.0, 0.0, 0
    for _ in range(10):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        it0 = int(agent.model.optimizer.iterations.item())
        agent.fused_train_step(events=ev)
        torch.cuda.synchronize()
        tr += ev[0].elapsed_time(ev[1])
        tu += ev[1].elapsed_time(ev[2])
        nu += int(agent.model.optimizer.iterations.item()) - it0
    print(f'rollout {tr / 10:.3f} ms/step, updates {tu / 10:.3f} ms/step '
          f'({nu / 10:.2f} per step, {tu / nu:.3f} ms each)', flush=True)


if __name__ == '__main__':
    main()
