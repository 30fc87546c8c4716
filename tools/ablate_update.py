"""Diagnostic: what each phase of the persistent PPO update costs on the critical path.
Builds libraries whose ppo_update.hip drops one phase (-DXA_ABL_TILE / _ROW / _ADAM; the
results are wrong, the exchange protocol and control flow are intact; -DXA_ABL_P0 / _BSUM /
_CNORM / _LDS drop phase 0, the phase-B sums, the global-norm reduction, the LDS weight refresh), links them with the
other objects of the last in-tree build (build/hip/*.o), and times the update graph of a
16- and a 256-env PPO train step with each (HIP events, 200 replays).
usage: python tools/ablate_update.py [--build-only | --no-build]"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / 'tools' / 'diag_lib'
_T = ['-DXA_ABL_TILE', '-DXA_ABL_ROW', '-DXA_ABL_ADAM']
VARIANTS = {'base': [], 'no-tile': ['-DXA_ABL_TILE'], 'no-row': ['-DXA_ABL_ROW'],
            'no-adam': ['-DXA_ABL_ADAM'], 'no-tile-row-adam': _T,
            'T+no-phase0': _T + ['-DXA_ABL_P0'], 'T+no-Bsum': _T + ['-DXA_ABL_BSUM'],
            'T+no-norm': _T + ['-DXA_ABL_CNORM'], 'T+no-ldsw': _T + ['-DXA_ABL_LDS']}


def build():
    from xagents_amd._build import BUILD_DIR, CFLAGS, HIPCC, build_library
    build_library()
    OUT.mkdir(exist_ok=True)
    others = [str(o) for o in sorted(BUILD_DIR.glob('*.o')) if o.stem != 'ppo_update']
    for name, flags in VARIANTS.items():
        obj = OUT / f'ppo_update_{name}.o'
        subprocess.run([HIPCC, *CFLAGS, *flags, '-c', str(ROOT / 'xagents_amd' / 'csrc' /
                                                           'ppo_update.hip'), '-o', str(obj)],
                       check=True)
        subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-o',
                        str(OUT / f'libxa_abl_{name}.so'), str(obj), *others], check=True)


def main():
    if '--no-build' not in sys.argv:
        build()
    if '--build-only' in sys.argv:
        return
    import torch
    from xagents_amd import _lib
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    for name in VARIANTS:
        _lib._lib = _lib.load(OUT / f'libxa_abl_{name}.so')
        from xagents_amd import PPO
        for n in (16, 256):
            envs = ReplayVecEnv('CartPole-v1', n, t_rec=4096, seed=55, device='cuda')
            model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
            agent = PPO(envs, model, n_steps=128, seed=55, quiet=True)
            for _ in range(3):
                agent.train_step()
            torch.cuda.synchronize()
            g = agent._graph[1]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(200):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            print(f'{name:18s} {n:4d} envs: update graph {a.elapsed_time(b) / 200 * 1e3:8.1f} us',
                  flush=True)


if __name__ == '__main__':
    main()
