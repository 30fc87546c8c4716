"""Diagnostic: bench.bench_ppo's timed loop restated step for step, printing every step's
update / rollout event times, then run again, then compared with an eager replica."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def timed_loop(agent, steps, label):
    import torch
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    words = []
    for k in range(steps):
        agent.fused_train_step(events[k])
        if label.startswith('synced'):
            torch.cuda.synchronize()
            w = agent.update_ws[:512].cpu().view(torch.int32).numpy()
            words.append((w[0], w[1], 0, 0, 0, w[64]))
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps * 1e3
    up = [e[1].elapsed_time(e[2]) * 1e3 for e in events]
    ro = [e[0].elapsed_time(e[1]) * 1e3 for e in events]
    print(f'{label}: ms/step {el:.4f}; update us: ' + ' '.join(f'{x:.0f}' for x in up), flush=True)
    print(f'{label}: rollout us: ' + ' '.join(f'{x:.0f}' for x in ro), flush=True)
    c = agent.update_ws[:512].cpu().view(torch.int32).numpy()
    c64 = agent.update_ws[:64].cpu().view(torch.int64).numpy()
    print(f'  ctl count {c[0]} abort {c[1]} gen {c[64]}; ctl as u64: '
          + ' '.join(f'{int(x) & 0xffffffffffffffff:#x}' for x in c64), flush=True)
    for k, w in enumerate(words):
        print(f'  step {k:2d} update {up[k]:5.0f} us: cnt0 {w[0]} abort {w[1]} exit {w[2]} '
              f'abort_at_start {w[3]} steps_done {w[4]} gen {w[5]}', flush=True)


def main():
    import numpy as np
    import torch
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv, record_cartpole_replay
    from xagents_amd.utils.common import create_model
    n = 16
    rec = record_cartpole_replay(n, 4096, seed=55)
    envs = ReplayVecEnv('CartPole-v1', n, device='cuda', record=rec)
    model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=55, device='cuda')
    theta0 = model.theta.cpu().numpy().copy()
    agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=True)
    for _ in range(5):
        agent.train_step()
    agent.check_peer_all_reduce()
    torch.cuda.synchronize()
    timed_loop(agent, 20, 'synced #1')
    timed_loop(agent, 20, 'bench-like #2')
    for _ in range(3):
        agent.timed_train_step()
    timed_loop(agent, 20, 'after timed_train_step')
    agent._drain_episode_stats()
    # eager replica of all 68 steps
    envs2 = ReplayVecEnv('CartPole-v1', n, device='cuda', record=rec)
    model2 = create_model(envs2, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                          seed=55, device='cuda')
    assert np.array_equal(theta0, model2.theta.cpu().numpy())
    b = PPO(envs2, model2, n_steps=128, seed=55, quiet=True, use_graph=False)
    for _ in range(5 + 20 + 20 + 3 + 20):
        b.train_step()
    torch.cuda.synchronize()
    print('theta equal to the eager replica:',
          np.array_equal(agent.model.theta.cpu().numpy(), b.model.theta.cpu().numpy()),
          'iters', int(agent.model.optimizer.iterations.item()),
          int(b.model.optimizer.iterations.item()), 'status', int(agent.device_status.item()),
          flush=True)


if __name__ == '__main__':
    main()
