"""Worker for tests/test_gpu_acer.py::test_acer_data_parallel_processes_on_one_gpu: W
processes on ONE HIP device with a gloo process group. Per rank: an ACER agent under the
process group (its own env shard, seed 6 + rank) and a local twin with the same data and
weights but no collectives. After one update: the data-parallel gradient equals the sum of
every rank's local gradient (each the mean over that rank's n_envs x n_steps), the replay
count broadcast keeps the ranks in step, and weights and average weights agree across
ranks. Prints 'ACER DP OK <rank>'."""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _agent(rank, device):
    from xagents_amd import ACER
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    n = 2
    envs = create_envs('PongNoFrameskip-v4', n, device=device, seed=6 + rank)
    model = create_model(envs, 'acer', 'model', seed=4, device=device,
                         optimizer_kwargs=dict(learning_rate=1e-3))
    return ACER(envs, model, create_buffers('acer', 8 * n, 1, n, initial_size=n), n_steps=4,
                seed=8, quiet=True, replay_ratio=2, grad_norm=10.0)


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    dp = _agent(rank, dev)
    local = _agent(rank, dev)
    local.distributed, local.world_size = False, 1
    assert dp.distributed and dp.world_size == world
    for ag in (local, dp):
        slot = ag._acer_rollout()
        ag._acer_update(*ag._slot_views(slot))
    torch.cuda.synchronize()
    lg = local.grad.cpu()
    parts = [torch.empty_like(lg) for _ in range(world)]
    dist.all_gather(parts, lg)
    want = parts[0].clone()
    for p in parts[1:]:
        want += p
    torch.testing.assert_close(dp.grad.cpu(), want, rtol=1e-5, atol=1e-7)
    # a full train step with replays (the count is broadcast from rank 0)
    np.random.seed(100 + rank)  # different host RNG per rank on purpose
    dp.train_step()
    torch.cuda.synchronize()
    for t in (dp.model.theta, dp.avg_model.theta, dp.model.optimizer.iterations):
        tc = t.cpu()
        got = [torch.empty_like(tc) for _ in range(world)]
        dist.all_gather(got, tc)
        for g in got[1:]:
            assert torch.equal(g, got[0]), 'ranks disagree'
    print(f'ACER DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
