"""A/B timing of how a PPO train step ships its episode statistics to the host (16 envs
by default): on a side stream overlapping the update vs on the launch stream, as one
packed copy vs three copies, or not at all. Prints ms per step."""
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
    steps = 300
    record = record_cartpole_replay(n, 4096, seed=55)
    envs = ReplayVecEnv('CartPole-v1', n, device='cuda', record=record)
    model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=55, device='cuda')
    agent = PPO(envs, model, n_steps=128, seed=55, quiet=True)
    pack = agent._stats_pack
    q = agent._queue_episode_stats

    def setv(side, packed):
        agent._drain_episode_stats()
        agent._stats_pack = pack if packed else None
        agent._host_pack = None
        agent._pending_stats = None
        if packed < 0:
            agent._queue_episode_stats = lambda *a, **k: None
        elif side:
            agent._queue_episode_stats = q
        else:
            agent._queue_episode_stats = lambda d, e, after=None: q(d, e)
        for _ in range(3):
            agent.train_step()
        torch.cuda.synchronize()

    def run():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            agent.fused_train_step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    res = {}
    cfgs = [('side packed', 1, 1), ('side 3-copies', 1, 0), ('main packed', 0, 1),
            ('main 3-copies', 0, 0), ('no stats copy', 0, -1)]
    for rep in range(3):
        for name, side, packed in cfgs[::1 - 2 * (rep % 2)]:
            setv(side, packed)
            res.setdefault(name, []).append(run())
    for k, v in res.items():
        print(f'{n} envs  {k:16s} ' + ' '.join(f'{x:.4f}' for x in v) + f'  min {min(v):.4f} ms')
    agent._queue_episode_stats = q
    agent._drain_episode_stats()


if __name__ == '__main__':
    main()
