"""Where does a short timed loop lose time? Mirrors bench.py's 16-env PPO setup (warmup,
peer check, 20 timed steps) and prints the host time each fused_train_step call returns
at, then the total after the final synchronize."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv, record_cartpole_replay
    from xagents_amd.utils.common import create_model
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    record = record_cartpole_replay(n, 4096, seed=55)
    envs = ReplayVecEnv('CartPole-v1', n, device='cuda', record=record)
    model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=55, device='cuda')
    agent = PPO(envs, model, n_steps=128, seed=55, quiet=True)
    import gc
    slow = []

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            d = time.perf_counter() - t
            if d > 1e-3:
                slow.append((name, round(d * 1e3, 2)))
            return r
        return w
    for name in ('_fold_stats', '_sync_stats_copy', '_queue_episode_stats', '_maybe_check_peer'):
        setattr(agent, name, timed(name, getattr(agent, name)))
    gc.callbacks.append(lambda phase, info: slow.append(('gc', phase, info.get('generation'))))
    for _ in range(5):
        agent.train_step()
    agent.check_peer_all_reduce()
    torch.cuda.synchronize()
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = []
        for k in range(20):
            agent.fused_train_step()
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        tot = time.perf_counter() - t0
        print(f'rep {rep}: total {tot * 1e3:.3f} ms  host returns (ms): ' +
              ' '.join(f'{t * 1e3:.2f}' for t in ts))
        print('   slow calls / gc:', slow)
        slow.clear()


if __name__ == '__main__':
    main()
