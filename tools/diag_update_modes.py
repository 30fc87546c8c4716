"""Diagnostic: duration of the persistent PPO update (xa_ppo_update) by launch pattern, at
16 envs, with HIP events on the launch stream around each update (median of N) and the
wall clock per train step: bench.bench_ppo's own measurement, then loops on the bench's
agent -- the bench's fused_train_step, rollout-graph + update-graph pairs with and without
the per-step episode-stats copies / a host sync, update graphs back to back, eager launches.
With --stamps it routes through the -DXA_STAMPS build (tools/diag_lib) and prints the
stamped cycles per phase of each pattern."""
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tools'))
STAMPS = '--stamps' in sys.argv
N = 20


def run_modes(agent, n):
    import numpy as np
    import torch
    from xagents_amd import _lib
    from diag_ppo_update import SLOTS
    buf = (ctypes.c_ulonglong * 64)()
    assert agent._graph is not None
    stream = torch.cuda.current_stream()
    for mode in ('fused', 'pair', 'probe', 'pair', 'eager'):
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(N)]
        torch.cuda.synchronize()
        if STAMPS:
            _lib._lib.xa_diag_read_stamps_ppo(buf)
        t0 = time.perf_counter()
        for i in range(N):
            if mode == 'fused':
                agent.fused_train_step(ev[i])
                continue
            if mode in ('pair', 'probe'):
                agent._graph[0].replay()  # the rollout graph, as in the bench loop
            ev[i][1].record(stream)
            if mode != 'eager':
                agent._graph[1].replay()
            else:
                agent._update_impl()
            ev[i][2].record(stream)
            if mode == 'probe':
                # the control words and the launch generation after each launch
                agent._queue_episode_stats(agent.b_done, agent.b_epret)
                torch.cuda.synchronize()
                w = agent.update_ws[:512].cpu().view(torch.int32).numpy()
                print(f'  probe {i:2d}: ctl {w[:8].tolist()} xcnt {w[8:16].tolist()} gen {w[64]}'
                      f' status {int(agent.device_status.item())}', flush=True)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / N * 1e6
        t = [a[1].elapsed_time(a[2]) * 1e3 for a in ev]
        line = (f'n={n:3d} {mode:10s} update median {np.median(t):7.1f} us  min {min(t):7.1f}'
                f'  max {max(t):7.1f}  wall/iter {wall:7.1f} us  status '
                f'{int(agent.device_status.item())}')
        if STAMPS:
            _lib._lib.xa_diag_read_stamps_ppo(buf)
            vals = {k: buf[k] for k in SLOTS}
            tot = sum(vals.values()) or 1
            line += f'  stamped {tot / N:9.0f} cyc/launch | ' + ' '.join(
                f'{k}:{v / N / 1000:.0f}k' for k, v in vals.items() if v)
        print(line, flush=True)
    agent._drain_episode_stats()


def main():
    import torch
    from xagents_amd import _lib
    if STAMPS:
        _lib._lib = _lib.load(ROOT / 'tools' / 'diag_lib' / 'libxagents_hip_diag.so')
    import bench
    sys.argv = sys.argv[:1]
    args = bench.parse()
    args.steps, args.warmup = 20, 5
    n = 16
    res = bench.bench_ppo(args, 1, 0, torch.device('cuda'), n)
    print(f'bench_ppo n={n}: update_ms {res["update_ms"]:.4f} rollout_ms {res["rollout_ms"]:.4f}'
          f' ms_per_step {res["ms_per_step"]:.4f} eager update launch_ms '
          f'{res["update_roofline"]["launch_ms"]:.4f}', flush=True)
    run_modes(res['agent'], n)


if __name__ == '__main__':
    main()
