"""Diagnostic: per-block phase timeline of the persistent PPO update (xa_ppo_update) from
the 100 MHz real-time clock, recorded by thread 0 of every logical block at 6 points of
every optimizer step (-DXA_TRACE build: ppo_update.hip's XA_TRACE_PT). Prints, per phase,
the median over the launch's steps of the mean / max over blocks, and the hop latencies
the critical path sees (last row published -> first / last block done with phase B, ...).
usage: python tools/trace_ppo_update.py [--build-only | --no-build] [n_envs ...] [--spread]"""
import ctypes
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / 'tools' / 'diag_lib'
LIB = OUT / 'libxa_trace.so'
STEPS, PTS = 32, 16


def build():
    from xagents_amd._build import BUILD_DIR, CFLAGS, HIPCC, build_library
    build_library()
    OUT.mkdir(exist_ok=True)
    others = [str(o) for o in sorted(BUILD_DIR.glob('*.o')) if o.stem != 'ppo_update']
    obj = OUT / 'ppo_update_trace.o'
    subprocess.run([HIPCC, *CFLAGS, '-DXA_TRACE', '-c',
                    str(ROOT / 'xagents_amd' / 'csrc' / 'ppo_update.hip'), '-o', str(obj)],
                   check=True)
    subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-o', str(LIB), str(obj), *others],
                   check=True)


def analyse(tr, G, K):
    # [block, step, point] in 10-ns ticks: low 32 bits, re-based (wrap-safe within a launch);
    # the shader clock words (slot STEPS - 1, points 9 and 11) keep their raw values
    base = int(tr[0, 0, 0])
    raw = tr.astype(np.int64)
    tr = ((raw - base) & 0xFFFFFFFF).astype(np.int64)
    tr[tr > 0x7FFFFFFF] -= 1 << 32
    tr[:, STEPS - 1, 9] = raw[:, STEPS - 1, 9]
    tr[:, STEPS - 1, 11] = raw[:, STEPS - 1, 11]
    t = tr[:G, :K, :6]
    us = lambda x: x / 100.0  # noqa: E731
    names = ['A: tile (+row into LDS)', 'row granule stores', 'B: wait rows + reduce + publish',
             'C: poll g + norm partials', 'norm + Adam + LDS refresh']
    print(f'  {"phase":34s} {"mean us":>8s} {"max us":>8s}  (median over steps of block mean / max)')
    for i, nm in enumerate(names):
        d = t[:, :, i + 1] - t[:, :, i]
        print(f'  {nm:34s} {us(np.median(d.mean(0))):8.3f} {us(np.median(d.max(0))):8.3f}')
    tt = tr[:G, :K]
    if (tt[:, :, 8] != 0).all():
        tile = ['H1 (VALU tanh)', 'Z2 = H1 W2 (MFMA) + tanh', 'heads + loss + dz',
                'dA2 + head grads', 'dW2, dH1 (MFMA)', 'dW1', 'tile end -> row combine done']
        seq = [0, 8, 9, 10, 11, 12, 13, 14]
        for i, nm in enumerate(tile[:-1]):
            d = tt[:, :, seq[i + 1]] - tt[:, :, seq[i]]
            print(f'    tile: {nm:28s} {us(np.median(d.mean(0))):8.3f} {us(np.median(d.max(0))):8.3f}')
        for a_, b_, nm in ((0, 6, 'loop top -> W1 in registers'), (6, 7, 'H1 computed'),
                           (7, 15, 'H1 stored (wave 0)'), (15, 8, 'B1 barrier wait')):
            d = tt[:, :, b_] - tt[:, :, a_]
            print(f'      H1 {nm:30s} {us(np.median(d.mean(0))):8.3f}')
        d = tt[:, :, 1] - tt[:, :, 14]
        print(f'    row combine into LDS (+loss sums) {us(np.median(d.mean(0))):8.3f} '
              f'{us(np.median(d.max(0))):8.3f}')
    nxt = t[:, 1:, 0] - t[:, :-1, 5]
    print(f'  {"loop top (barrier) -> next A":34s} {us(np.median(nxt.mean(0))):8.3f} '
          f'{us(np.median(nxt.max(0))):8.3f}')
    step = np.diff(t[:, :, 0].min(0))
    print(f'  step period (first block at loop top): median {us(np.median(step)):.3f} us, '
          f'steps {K}, blocks {G}')
    # hand-off latencies on the critical path
    last_row = t[:, :, 2].max(0)
    b_first, b_last = t[:, :, 3].min(0), t[:, :, 3].max(0)
    c_first, c_last = t[:, :, 4].min(0), t[:, :, 4].max(0)
    print(f'  row skew (first -> last row published)       {us(np.median(last_row - t[:, :, 2].min(0))):8.3f}')
    print(f'  last row -> first / last B published          {us(np.median(b_first - last_row)):8.3f} '
          f'{us(np.median(b_last - last_row)):8.3f}')
    print(f'  last B -> first / last C poll done            {us(np.median(c_first - b_last)):8.3f} '
          f'{us(np.median(c_last - b_last)):8.3f}')
    print(f'  A start skew (first -> last block at loop top) '
          f'{us(np.median(t[:, :, 0].max(0) - t[:, :, 0].min(0))):8.3f}')
    # the launch outside the step loop: start (after the election) -> phase-0 hop done ->
    # first loop top; last step's Adam done -> the block's end
    pro = tr[:G, STEPS - 1]
    start, hop = pro[:, 6], pro[:, 7]
    ent = pro[:, 5]
    print(f'  kernel entry (first) -> first / last start    {us(start.min() - ent.min()):8.3f} '
          f'{us(start.max() - ent.min()):8.3f}  (election)')
    print(f'  launch start skew (first -> last block)       {us(start.max() - start.min()):8.3f}')
    for a_, b_, nm in ((6, 0, 'start -> gather done'), (0, 1, 'gather -> adv sums stored'),
                       (1, 2, 'm / v + weights to LDS'), (2, 4, 'advantage totals polled'),
                       (4, 3, 'minibatch statistics')):
        d = pro[:, b_] - pro[:, a_]
        print(f'    phase 0: {nm:34s} {us(np.median(d)):8.3f} {us(d.max()):8.3f}')
    print(f'  first start -> last phase-0 hop done          {us(hop.max() - start.min()):8.3f}')
    print(f'  phase-0 hop done -> first / last loop top     {us(t[:, 0, 0].min() - hop.max()):8.3f} '
          f'{us(t[:, 0, 0].max() - hop.max()):8.3f}')
    st = pro[:, 3]
    print(f'  statistics done -> first / last loop top      {us(t[:, 0, 0].min() - st.max()):8.3f} '
          f'{us(t[:, 0, 0].max() - st.max()):8.3f}')
    print(f'  first start -> last step done (loop span)     {us(t[:, K - 1, 5].max() - start.min()):8.3f}')
    print(f'  last step done -> block 0 end                 {us(pro[0, 10] - t[:, K - 1, 5].max()):8.3f}')


def main():
    if '--no-build' not in sys.argv:
        build()
    if '--build-only' in sys.argv:
        return
    if '--spread' in sys.argv:
        os.environ['XA_PPO_PLACE'] = 'spread'
    import torch
    from xagents_amd import _lib
    _lib._lib = _lib.load(LIB)
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    L = _lib._lib
    L.xa_diag_read_trace_ppo.argtypes = [ctypes.c_void_p]
    buf = np.zeros(256 * STEPS * PTS, np.uint32)
    for n in [int(a) for a in sys.argv[1:] if a.isdigit()] or (16, 256):
        envs = ReplayVecEnv('CartPole-v1', n, t_rec=4096, seed=55, device='cuda')
        model = create_model(envs, 'ppo', 'model', seed=55, device='cuda')
        agent = PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=False)
        for _ in range(4):
            agent.train_step()
        torch.cuda.synchronize()
        assert L.xa_diag_read_trace_ppo(buf.ctypes.data) == 0
        tr = buf.reshape(256, STEPS, PTS)
        G, K = agent.update_blocks, agent.ppo_epochs * agent.n_mb
        clk = tr[:G, STEPS - 1, 8:12].astype(np.int64)
        ghz = (clk[:, 3] - clk[:, 1]) / np.maximum(clk[:, 2] - clk[:, 0], 1) * 0.1
        print(f'n_envs {n}: placement {agent._uargs.placement}, {G} blocks, {K} steps, '
              f'shader clock {np.median(ghz):.2f} GHz (min {ghz.min():.2f})')
        analyse(tr, G, K)


if __name__ == '__main__':
    main()
