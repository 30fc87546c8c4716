"""Worker for tests/test_gpu_dp.py::test_ppo_data_parallel_equals_union: W processes on ONE
HIP device with a gloo process group (plus the IPC peer all-reduce the DP update uses).
Rank r runs the fused PPO train step on its own 8-env shard (replay record seed 55 + r);
rank 0 also runs a single-process agent on the union of the shards (data_parallel=False)
fed the same rollout uniforms and the rank-major union of the ranks' minibatch
permutations. The data-parallel step must equal the union step: rollout buffers bit for
bit, parameters up to the summation order of the gradient (xagents/ppo/agent.py:157-191).
With XA_TEST_SKEW_S > 0 (launch-skew mode) every rank but 0 sleeps that long on the host
before each of XA_TEST_STEPS train steps, so the persistent update's in-launch exchange
waits for a late peer: the step must still equal the union step (first step) and every
later step must leave the ranks' parameters identical with the device status word clean.
Prints 'PPO DP OK <rank>'."""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

N, T, E, M, T_REC = 8, 16, 4, 4, 256
if os.environ.get('XA_TEST_DP_SHAPE') == 'headline':
    # the metric's per-rank shape (16 envs x 128 steps, 4 x 4 minibatches of 512): the ranks
    # run the fixed-shape data-parallel update instantiation
    N, T = 16, 128


def make(record, n, data_parallel=None):
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', n, device='cuda', record=record)
    model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=21, device='cuda')
    return PPO(envs, model, n_steps=T, seed=21, quiet=True, use_graph=False,
               ppo_epochs=E, mini_batches=M, data_parallel=data_parallel)


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from xagents_amd.envs import record_cartpole_replay
    records = [record_cartpole_replay(N, T_REC, seed=55 + r) for r in range(world)]
    uniforms = [np.random.default_rng(100 + r).random((N, T)).astype(np.float32)
                for r in range(world)]
    B, mb = N * T, N * T // M
    perms = [np.stack([np.random.default_rng(200 + 10 * r + e).permutation(B)
                       for e in range(E)]).astype(np.int32) for r in range(world)]
    dp = make(records[rank], N)
    want = os.environ.get('XA_PPO_UPDATE', 'persistent')
    assert dp.distributed and dp.world_size == world and dp.update_mode == want, dp.update_mode
    theta0 = dp.model.theta.cpu().numpy().astype(np.float64)
    u_dp = torch.from_numpy(uniforms[rank]).cuda()
    p_dp = torch.from_numpy(perms[rank]).cuda()
    dp.set_rollout_uniforms(u_dp)
    dp.set_minibatch_permutation(p_dp)
    skew = float(os.environ.get('XA_TEST_SKEW_S', '0'))
    n_steps = int(os.environ.get('XA_TEST_STEPS', '1'))

    def step():
        if skew > 0 and rank > 0:
            time.sleep(skew * rank)  # this rank launches late: the others' launches wait
        dp.train_step()
        torch.cuda.synchronize()
        if dp.update_mode == 'persistent':
            assert int(dp._stats_status.item()) == 0, 'persistent update aborted (status word)'

    step()
    got = {k: getattr(dp, k).cpu() for k in ('b_act', 'b_logp', 'b_val', 'b_ret')}
    got['theta'] = dp.model.theta.cpu()
    gathered = {}
    for k, t in got.items():
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        gathered[k] = parts
    for p in gathered['theta'][1:]:
        assert torch.equal(p, gathered['theta'][0]), 'ranks disagree on theta'
    if rank == 0:
        union_rec = tuple(np.concatenate([r[i] for r in records]) for i in range(5))
        un = make(union_rec, world * N, data_parallel=False)
        assert not un.distributed and un.update_mode == want
        np.testing.assert_array_equal(un.model.theta.cpu().numpy(), theta0)
        un.set_rollout_uniforms(torch.from_numpy(np.concatenate(uniforms)).cuda())
        # union minibatch m = the ranks' minibatch m slices, rank-major, global indices
        up = np.stack([np.concatenate([np.concatenate(
            [r * B + perms[r][e][m * mb:(m + 1) * mb] for r in range(world)])
            for m in range(M)]) for e in range(E)]).astype(np.int32)
        un.set_minibatch_permutation(torch.from_numpy(up).cuda())
        un.train_step()
        torch.cuda.synchronize()
        for k in ('b_act', 'b_logp', 'b_val', 'b_ret'):
            np.testing.assert_array_equal(getattr(un, k).cpu().numpy(),
                                          torch.cat(gathered[k]).numpy(), err_msg=k)
        tu = un.model.theta.cpu().numpy().astype(np.float64)
        td = gathered['theta'][0].numpy().astype(np.float64)
        rel = np.linalg.norm(td - tu) / np.linalg.norm(tu - theta0)
        assert rel < 1e-4, f'data-parallel update deviates from the union update: {rel:.2e}'
        assert int(un.model.optimizer.iterations.item()) == E * M
    assert int(dp.model.optimizer.iterations.item()) == E * M
    for _ in range(n_steps - 1):
        step()
        theta = dp.model.theta.cpu()
        parts = [torch.empty_like(theta) for _ in range(world)]
        dist.all_gather(parts, theta)
        for p in parts[1:]:
            assert torch.equal(p, parts[0]), 'ranks disagree on theta after a skewed step'
        assert torch.isfinite(theta).all()
    assert int(dp.model.optimizer.iterations.item()) == E * M * n_steps
    dist.barrier()
    if getattr(dp, 'dp_blocks', None) is not None:
        dp.dp_blocks.close()
    if dp.peer is not None:
        dp.peer.close()
    print(f'PPO DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
