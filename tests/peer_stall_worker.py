"""Worker for tests/test_gpu_dp.py::test_peer_stall_falls_back_to_rccl: 2 processes on ONE
HIP device, gloo group, fused PPO data-parallel over the IPC peer all-reduce with a short
exchange timeout (XA_PEER_TIMEOUT_S) and health check every 4 train steps
(XA_PEER_CHECK_STEPS). Rank 1 stalls on the host in the middle of the run, so rank 0's
exchanges time out; the periodic check must notice on every rank, warn, re-broadcast rank
0's parameters and optimizer state, and continue on the process group's all-reduce with
identical weights on both ranks. Prints 'STALL OK <rank>'."""
import sys
import time
import warnings
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 4, t_rec=128, seed=30 + rank, device='cuda')
    model = create_model(envs, 'ppo', 'model', seed=5, device='cuda')
    agent = PPO(envs, model, n_steps=8, seed=5, quiet=True, use_graph=False)
    assert agent.peer is not None, 'the peer all-reduce is not set up'
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter('always')
        for step in range(12):
            if rank == 1 and step == 2:
                time.sleep(3.0)  # a stall longer than the exchange timeout
            agent.train_step()
        torch.cuda.synchronize()
    assert agent.peer is None, 'the stall was not detected'
    assert any('falling back to RCCL' in str(w.message) for w in caught), caught
    theta = agent.model.theta.cpu()
    parts = [torch.empty_like(theta) for _ in range(world)]
    dist.all_gather(parts, theta)
    assert torch.equal(parts[0], parts[1]), 'ranks disagree after the fallback'
    assert np.isfinite(theta.numpy()).all()
    print(f'STALL OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
