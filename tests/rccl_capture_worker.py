"""Worker for tests/test_gpu_rccl_capture.py: a ONE-rank nccl (= RCCL) process group on the
test GPU, the IPC peer path off, so the PPO train step runs the per-minibatch chain with
every gradient and advantage-sum exchange a dist.all_reduce over RCCL
(xagents/ppo/agent.py:157-191 with the data-parallel exchange). One agent captures that
step -- RCCL collectives included -- as a hipGraph; a second, identically seeded agent runs
it eagerly. After 3 train steps the two must agree bit for bit (same kernels, same order),
and the captured agent must really have replayed its graph. Prints 'RCCL CAPTURE OK 0' and
the per-step wall time of both."""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def make(use_graph):
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 16, t_rec=512, seed=55, device='cuda')
    model = create_model(envs, 'ppo', 'model', seed=21, device='cuda')
    return PPO(envs, model, n_steps=32, seed=21, quiet=True, use_graph=use_graph)


def main():
    assert os.environ.get('XA_PEER_ALLREDUCE') == '0'
    torch.cuda.set_device(0)
    dist.init_process_group('nccl')
    assert dist.get_backend() == 'nccl' and dist.get_world_size() == 1
    eager, graph = make(False), make(True)
    for a in (eager, graph):
        assert a.distributed and a.peer is None and a.update_mode == 'chain', a.update_mode
    np.testing.assert_array_equal(eager.model.theta.cpu().numpy(), graph.model.theta.cpu().numpy())
    times = {}
    for name, a in (('eager', eager), ('graph', graph)):
        a.train_step()  # eager first step (the captured agent captures after it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            a.train_step()
        torch.cuda.synchronize()
        times[name] = (time.perf_counter() - t0) / 2 * 1e3
    assert graph.use_graph and graph._graph is not None, 'the RCCL step was not captured'
    assert eager._graph is None
    for k in ('b_act', 'b_logp', 'b_val', 'b_ret'):
        np.testing.assert_array_equal(getattr(eager, k).cpu().numpy(),
                                      getattr(graph, k).cpu().numpy(), err_msg=k)
    np.testing.assert_array_equal(eager.model.theta.cpu().numpy(), graph.model.theta.cpu().numpy())
    assert int(graph.model.optimizer.iterations.item()) == 3 * 16
    print(f'RCCL step ms: eager {times["eager"]:.3f}, graph {times["graph"]:.3f}', flush=True)
    print('RCCL CAPTURE OK 0', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
