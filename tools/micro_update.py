"""Micro-timings of the PPO update kernels in isolation (back-to-back launches, HIP
events): launch floor, xa_grad_reduce, xa_ac_grad with / without the pending Adam."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def t_us(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    torch.cuda._sleep(20_000_000)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    from xagents_amd import PPO, kernels
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 256, t_rec=4096, seed=55, device='cuda')
    model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
    agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=False)
    agent.fused_train_step()
    torch.cuda.synchronize()
    ctr = agent.rng_counter
    print(f'launch floor (counter_bump): {t_us(lambda: kernels.counter_bump(ctr)):.2f} us')
    it = model.optimizer.iterations
    print(f'grad_reduce: {t_us(lambda: kernels.grad_reduce(agent.partials, agent.grad, it)):.2f} us')
    g0, g1 = agent._gargs_list[0], agent._gargs_list[1]
    print(f'ac_grad (no pending Adam): {t_us(lambda: kernels.ac_grad(g0)):.2f} us')
    print(f'ac_grad (pending Adam):    {t_us(lambda: kernels.ac_grad(g1)):.2f} us')
    print(f'minibatches: {t_us(lambda: kernels.minibatches(agent._mbargs), 50):.2f} us')
    print(f'rollout: {t_us(lambda: kernels.rollout(agent._rargs), 20):.2f} us')


if __name__ == '__main__':
    main()
