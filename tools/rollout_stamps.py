"""Per-phase shader-clock stamps of the batched replay rollout (diagnostic build:
python tools/build_variant.py rstamp -DXA_STAMPS --src mlp_rollout): block 0 thread 0's
cycles in weight staging (8), its tiles (9), the barrier after them (10), the chunk pass
(11), its barrier (12), the episode-return scan (13), the state / returns tail (14), summed
over a launch and averaged over launches.
usage: XA_LIB=tools/diag_lib/libxa_rstamp.so python tools/rollout_stamps.py [n_envs ...]"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import _lib
    lib = _lib.load(os.environ['XA_LIB'])
    _lib._lib = lib
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    names = {8: 'prologue', 9: 'tiles (wave 0)', 10: 'tile barrier', 11: 'chunk pass',
             12: 'chunk barrier', 14: 'state + returns'}
    for n in [int(a) for a in sys.argv[1:]] or [16, 256]:
        envs = ReplayVecEnv('CartPole-v1', n, t_rec=4096, seed=55, device='cuda')
        model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
        agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=False)
        buf = (ctypes.c_ulonglong * 64)()
        for _ in range(3):
            agent.train_step()
        torch.cuda.synchronize()
        lib.xa_diag_read_stamps_rollout(buf)
        k = 20
        for _ in range(k):
            agent.train_step()
        torch.cuda.synchronize()
        lib.xa_diag_read_stamps_rollout(buf)
        st = np.array(buf[:64], np.float64) / k
        print(f'{n} envs: cycles per launch (block 0, thread 0)')
        for s, name in names.items():
            print(f'  slot {s:2d} {name:18s} {st[s]:10.0f}')
        print(f'  total {st[8:15].sum():10.0f}')
        print('  per-wave arrival at the first tile barrier (cycles from the wave start): ' +
              ' '.join(f'w{w}={st[32 + w]:.0f}' for w in range(8)))
        print('  bootstrap wave: start / end ' + ' '.join(f'{st[k]:.0f}' for k in (54, 55)))
        print('  return wave: start / LDS rows / chain / sync / stores / sync ' +
              ' '.join(f'{st[k]:.0f}' for k in range(48, 54)))
        print('  returns wave: start / deltas / chain / stores ' +
              ' '.join(f'{st[k]:.0f}' for k in range(56, 60)))


if __name__ == '__main__':
    main()
