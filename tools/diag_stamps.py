"""Diagnostic: per-phase cycle shares of the rollout and ac_grad kernels from
s_memtime stamps (thread 0 of block 0). Builds a separate -DXA_STAMPS library
(build/diag/libxagents_hip_diag.so); production kernels carry no stamps.
Shares are meaningful, absolute times are not (stamps serialise the phases)."""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / 'build' / 'diag'


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    objs = []
    # every source (the loader binds every exported symbol); stamps only where XA_STAMP is used
    for src in sorted(p.stem for p in (ROOT / 'xagents_amd' / 'csrc').glob('*.hip')):
        o = OUT / f'{src}.o'
        subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC',
                        '-ffp-contract=off', '-DXA_STAMPS', '-c',
                        str(ROOT / 'xagents_amd' / 'csrc' / f'{src}.hip'), '-o', str(o)], check=True)
        objs.append(str(o))
    lib = OUT / 'libxagents_hip_diag.so'
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-shared', '-o', str(lib), *objs],
                   check=True)
    return lib


def main():
    lib_path = build() if not (len(sys.argv) > 1 and sys.argv[1] == '--no-build') else (
        ROOT / 'tools' / 'diag_lib' / 'libxagents_hip_diag.so')  # built here, travels to the box
    if len(sys.argv) > 1 and sys.argv[1] == '--build-only':
        return
    import torch
    from xagents_amd import _lib
    _lib._lib = _lib.load(lib_path)  # route every op through the diagnostic build
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    n_envs = next((int(a) for a in sys.argv[1:] if a.isdigit()), 256)
    envs = ReplayVecEnv('CartPole-v1', n_envs, t_rec=4096, seed=55, device='cuda')
    model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
    agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=False)
    L = _lib._lib
    buf = (ctypes.c_ulonglong * 64)()
    for name in ('xa_diag_read_stamps_rollout', 'xa_diag_read_stamps_update'):
        getattr(L, name)(buf)
    for _ in range(3):
        agent.train_step()
    torch.cuda.synchronize()
    for name, slots in (('xa_diag_read_stamps_rollout',
                         {0: 'loop top', 1: 'layer1+LDS bcast',
                          2: 'layer2+tanh', 3: 'heads (3 wave sums)', 4: 'categorical',
                          6: 'env step (record readlanes)', 7: 'chunk pass', 5: 'tail'}),
                        ('xa_diag_read_stamps_update',
                         {20: 'prologue: param/grad loads', 21: 'prologue: norm + barrier',
                          22: 'prologue: Adam + LDS stores', 11: 'adv stats + tile-loop barrier',
                          12: 'gather', 13: 'H1', 14: 'G1 (MFMA)+tanh',
                          15: 'heads+loss', 16: 'dA2', 17: 'G2+G3 (MFMA)', 18: 'dW1',
                          19: 'epilogue (partials)'})):
        getattr(L, name)(buf)
        vals = {k: buf[k] for k in slots}
        tot = sum(vals.values()) or 1
        print(name)
        for k, label in slots.items():
            print(f'  slot {k:2d} {label:45s} {vals[k]:12d} cyc  {100 * vals[k] / tot:5.1f}%')


if __name__ == '__main__':
    main()
