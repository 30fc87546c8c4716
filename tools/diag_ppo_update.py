"""Diagnostic: per-phase cycle shares of the persistent PPO update (xa_ppo_update) from
s_memtime stamps in thread 0 of block 0, at 16 and 256 envs. Uses the -DXA_STAMPS build of
tools/diag_stamps.py. Shares are meaningful; absolute times include the stamps' cost."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tools'))

SLOTS = {30: 'phase 0: adv sums', 31: 'hop 0 signal', 32: 'param loads', 33: 'hop 0 wait',
         34: 'adv stats + loop top', 35: 'tile gather + barriers',
         50: ' tile: H1 (VALU tanh)', 51: ' tile: Z2 = H1 W2 (MFMA) + tanh',
         52: ' tile: heads + loss + dz', 53: ' tile: dA2 + head grads',
         54: ' tile: dW2, dH1 (MFMA)', 55: ' tile: dW1', 36: 'tile end',
         44: 'row: combine partials (LDS)', 45: 'row: loss sums + granule stores',
         37: 'row: next tile prefetch', 38: 'XCD level-1 reduce (two-level)',
         40: 'phase B reduce', 46: 'phase C: g slice poll', 47: 'phase C: norm partial poll',
         43: 'phase C: norm + Adam + LDS'}


def main():
    import diag_stamps
    import shutil
    lib_path = ROOT / 'tools' / 'diag_lib' / 'libxagents_hip_diag.so'  # travels to the box
    if '--no-build' not in sys.argv:
        lib_path.parent.mkdir(exist_ok=True)
        shutil.copy(diag_stamps.build(), lib_path)
    if '--build-only' in sys.argv:
        return
    import torch
    from xagents_amd import _lib
    _lib._lib = _lib.load(lib_path)
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    L = _lib._lib
    buf = (ctypes.c_ulonglong * 64)()
    for n in [int(a) for a in sys.argv[1:] if a.isdigit()] or (16, 256):
        envs = ReplayVecEnv('CartPole-v1', n, t_rec=4096, seed=55, device='cuda')
        model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
        agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=False)
        agent.train_step()
        torch.cuda.synchronize()
        L.xa_diag_read_stamps_ppo(buf)
        steps = 3
        for _ in range(steps):
            agent.train_step()
        torch.cuda.synchronize()
        L.xa_diag_read_stamps_ppo(buf)
        vals = {k: buf[k] for k in SLOTS}
        tot = sum(vals.values()) or 1
        print(f'n_envs {n}: {agent.update_blocks} blocks, {tot / steps:.0f} cycles per launch')
        for k, label in SLOTS.items():
            print(f'  slot {k:2d} {label:30s} {vals[k] / steps / 16:10.0f} cyc/opt-step  '
                  f'{100 * vals[k] / tot:5.1f}%')


if __name__ == '__main__':
    main()
