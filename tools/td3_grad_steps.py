"""C5 (TD3, 64 BipedalWalker-shaped envs, ReplayBuffer2) gradient steps alone, for a
rocprofv3 kernel trace of one gradient step's launches (tools/gpu_steps.sh profc5).

usage: python tools/td3_grad_steps.py [n_steps]   (XA_LIB=<trace build>: + per-phase times)"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import os

    import numpy as np
    import torch
    from xagents_amd import TD3, _lib
    if os.environ.get('XA_LIB'):
        # the per-phase trace needs a diagnostic build (tools/build_variant.py td3trace
        # -DXA_TD3_TRACE=1 --src td3_update): the product writes no trace
        _lib._lib = _lib.load(os.environ['XA_LIB'])
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = 64
    np.random.seed(55)
    envs = create_envs('BipedalWalker-v3', n, device='cuda', seed=55)
    kw = dict(seed=55, device='cuda')
    actor = create_model(envs, 'td3', 'actor_model', **kw)
    critic = create_model(envs, 'td3', 'critic_model', **kw)
    bufs = create_buffers('td3', 1_000_000, 100, n, initial_size=n * 64)
    agent = TD3(envs, actor, critic, bufs, gradient_steps=1, seed=55, quiet=True)
    agent.fill_buffers()
    for _ in range(10):
        agent.update_weights(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        agent.update_weights(1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n_steps
    print(f'TD3 gradient step: {dt * 1e3:.4f} ms ({n_steps} steps, graph replay)', flush=True)
    if agent._fused_args() is not None and os.environ.get('XA_LIB'):
        # per-phase barrier times of the fused launch (block 0's 100 MHz wall clock, the
        # workspace control area's trace words: [0] start, [i] barrier i done, [15] end)
        import numpy as np
        rows = []
        agent.use_graph = False
        for _ in range(40):
            agent.update_weights(1)
            torch.cuda.synchronize()
            tr = agent._fused_ws[1536:1664].cpu().numpy().view(np.uint64).astype(np.int64)
            rows.append(tr)
        diffs = []
        for tr in rows:
            n = int(np.count_nonzero(tr[1:15] > tr[0]))
            marks = np.asarray(list(tr[:n + 1]) + [tr[15]], np.float64)
            diffs.append(np.diff(marks) / 100.0)  # 100 MHz ticks -> us
        # the launch's phases in barrier order (xa_td3_update's P-numbers: P3 / P6 / P12 run
        # as the row tiles' last jobs of P2 / P5 / P11)
        names = ['P1', 'P2', 'P4', 'P5', 'P7', 'P8', 'P9', 'P10', 'P11', 'P13', 'P14']
        n_max = max(len(x) for x in diffs)
        diffs = [x for x in diffs if len(x) == n_max]
        d = np.median(np.stack(diffs), 0)
        print(f'fused phases (us, block 0, median of {len(diffs)} eager policy launches): ' +
              ' '.join(f'{names[i] if i < len(names) else i} {v:.1f}' for i, v in enumerate(d)) +
              f' | total {d.sum():.1f}', flush=True)
        # inside block 0's first job of each phase: entry, loads issued, operands in LDS,
        # MFMA done (us after the phase's barrier), from the last launch
        tr = rows[-1]
        dt = agent._fused_ws[2048:2048 + 8192].cpu().numpy().view(np.uint64).astype(np.int64)
        pro = dt[8 * 15:8 * 15 + 4]
        if (pro > 0).all() and pro[0] >= tr[0]:
            rel = (pro - tr[0]) / 100.0
            print(f'  prologue: start {rel[0]:.2f} slots issued {rel[1]:.2f} slots in LDS '
                  f'{rel[2]:.2f} P1 loop {rel[3]:.2f} us', flush=True)
        for p in range(len(d) - 1):
            pts = dt[8 * p:8 * p + 4]
            if (pts <= 0).any() or pts[0] < tr[0]:
                continue
            rel = (pts - tr[p]) / 100.0
            print(f'  {names[p] if p < len(names) else p} job: entry {rel[0]:.2f} issued {rel[1]:.2f} ready {rel[2]:.2f} '
                  f'mma {rel[3]:.2f} us', flush=True)


if __name__ == '__main__':
    main()
