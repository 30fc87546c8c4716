"""Worker for tests/test_gpu_dp.py::test_cnn_ppo_data_parallel_equals_union: the C4
data-parallel path (PPO with the CNN actor-critic on the layer executor,
xagents_amd/onpolicy_executor.py) with W processes on ONE HIP device over a gloo group.

Rank r runs PPO on its own Breakout-shaped shard of N envs (synthetic uint8 frames,
record seed 55 + r): rollout, the advantage statistics of every minibatch all-reduced
once per train step, and per minibatch the 77 MB gradient all-reduced in buckets (the
dense layers' slice issued while the conv backward still runs). Rank 0 also runs a
single-process agent on the union of the shards (data_parallel=False) fed the same
rollout uniforms and the rank-major union of the ranks' minibatch permutations. The
data-parallel train step must equal the union step (xagents/ppo/agent.py:157-191):
actions bit for bit, log-probs / values / returns to f32 rounding (the union's GEMMs run
at twice the batch, which may pick another split-K count and so another summation
order), parameters identical on every rank and 16 optimizer steps taken. The parameter
bound separates branch flips from everything else: every optimizer step's per-sample head
gradients (d logits, d value) of the data-parallel ranks are compared row by row with the
union's; a sample whose PPO ratio or value sits within f32 rounding of its clip boundary
can take the other branch in one of the two runs, which changes its row by O(1) (every
other row agrees to ~1e-5). Without such a flip the parameters must agree within 2e-5 of
the update's norm; with one (counted and reported, at most 8 per train step) within 5e-4.
ReLU gate flips of units at pre-activation ~0 are counted and reported too.
Prints 'CNN DP OK <rank>'."""
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

N, T, E, M, T_REC = 8, 16, 4, 4, 64


def make(record, n, data_parallel=None):
    from xagents_amd import PPO
    from xagents_amd.envs import Discrete, TransitionReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = TransitionReplayVecEnv('BreakoutNoFrameskip-v4', n, (84, 84, 1), Discrete(4),
                                  np.uint8, device='cuda', record=record)
    model = create_model(envs, 'ppo', 'model', seed=21, device='cuda')
    return PPO(envs, model, n_steps=T, seed=21, quiet=True, ppo_epochs=E, mini_batches=M,
               data_parallel=data_parallel)


def trace_heads(agent):
    """Record every optimizer step's per-sample head gradients (rows of the minibatch:
    [d logits | d value]) and the ReLU gate pattern of every hidden layer of its forward
    (bit-packed rows)."""
    from xagents_amd._lib import XA_ACT_RELU
    rows, gates, fn = [], [], agent._minibatch_step

    def traced(n, k=None):
        fn(n, k)
        rows.append(torch.cat([agent.dlogits[:n], agent.dvalue[:n]], 1).cpu())
        per = None
        for j, ex in enumerate(agent.ex_chunks):
            c0 = j * agent.chunk
            if c0 >= n:
                break
            r = min(ex.B, n - c0)
            ms = [(ex.outs[i][:r].reshape(r, -1) > 0).cpu().numpy()
                  for i, l in enumerate(ex.layers)
                  if l.kind != 'flatten' and ex._act(i) == XA_ACT_RELU]
            per = ms if per is None else [np.concatenate([a, b]) for a, b in zip(per, ms)]
        gates.append([torch.from_numpy(np.packbits(m, axis=1)) for m in per])

    agent._minibatch_step = traced
    return rows, gates


def head_flips(dp_rows, un_rows, world):
    """Samples whose d-logits or d-value part differs between the data-parallel run
    (rank-major concatenation; each rank's loss is its local mean, so its rows carry W x
    the union's 1 / mb) and the union run by more than 1e-3 of that part's norm: the
    clip-branch flips (PPO ratio clip: the policy term; value clip: the value term).
    Returns the flips and the largest part deviation of the other rows."""
    flips, worst = [], 0.0
    for k, (d, u) in enumerate(zip(dp_rows, un_rows)):
        d = d.double().numpy() / world
        u = u.double().numpy()
        for part in (slice(0, -1), slice(-1, None)):
            den = np.maximum(np.linalg.norm(u[:, part], axis=1), 1e-12)
            dev = np.linalg.norm(d[:, part] - u[:, part], axis=1) / den
            bad = np.nonzero(dev > 1e-3)[0]
            flips += [(k, int(i), 'value' if part.start == -1 else 'logits') for i in bad]
            ok = np.delete(dev, bad)
            worst = max(worst, float(ok.max()) if ok.size else 0.0)
    return flips, worst


def gate_flips(dp_gates, un_gates):
    """ReLU units whose gate (pre-activation > 0) differs between the two runs' forwards of
    the same sample at the same optimizer step: (step, layer, count)."""
    out = []
    for k, (d, u) in enumerate(zip(dp_gates, un_gates)):
        for li, (a, b) in enumerate(zip(d, u)):
            n = int(np.unpackbits(np.bitwise_xor(a.numpy(), b.numpy())).sum())
            if n:
                out.append((k, li, n))
    return out


def main():
    if os.environ.get('XA_LIB'):  # a diagnostic variant library (tools/cnn_dp_rel.sh)
        from xagents_amd import _lib
        _lib._lib = _lib.load(os.environ['XA_LIB'])
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from xagents_amd.envs import record_transitions
    base = int(os.environ.get('XA_DP_SEED', '55'))  # tools/cnn_dp_rel.sh sweeps it
    records = [record_transitions(N, T_REC, (84, 84, 1), np.uint8, seed=base + r)
               for r in range(world)]
    uniforms = [np.random.default_rng(100 + r).random((N, T)).astype(np.float32)
                for r in range(world)]
    B, mb = N * T, N * T // M
    perms = [np.stack([np.random.default_rng(200 + 10 * r + e).permutation(B)
                       for e in range(E)]).astype(np.int32) for r in range(world)]
    dp = make(records[rank], N)
    assert dp.executor_path and dp.distributed and dp.world_size == world
    if os.environ.get('XA_TEST_BUCKET_MB'):
        dp.bucket_floats = int(float(os.environ['XA_TEST_BUCKET_MB']) * (1 << 20)) // 4
    theta0 = dp.model.theta.cpu().numpy().astype(np.float64)
    dp.set_rollout_uniforms(torch.from_numpy(uniforms[rank]).cuda())
    dp.set_minibatch_permutation(torch.from_numpy(perms[rank]).cuda())
    it0 = int(dp.model.optimizer.iterations.item())
    dp_rows, dp_gates = trace_heads(dp)
    dp.train_step()
    torch.cuda.synchronize()
    got = {k: getattr(dp, k).cpu() for k in ('b_act', 'b_logp', 'b_val', 'b_ret')}
    got['theta'] = dp.model.theta.cpu()
    gathered = {}
    for k, t in got.items():
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        gathered[k] = parts
    assert len(dp_rows) == E * M
    def cat_ranks(t):
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return torch.cat(parts)
    heads = [cat_ranks(t) for t in dp_rows]
    gates = [[cat_ranks(m) for m in step] for step in dp_gates]
    for p in gathered['theta'][1:]:
        assert torch.equal(p, gathered['theta'][0]), 'ranks disagree on theta'
    assert int(dp.model.optimizer.iterations.item()) - it0 == E * M
    if rank == 0:
        union_rec = tuple(np.concatenate([r[i] for r in records]) for i in range(5))
        un = make(union_rec, world * N, data_parallel=False)
        assert un.executor_path and not un.distributed
        np.testing.assert_array_equal(un.model.theta.cpu().numpy(), theta0)
        un.set_rollout_uniforms(torch.from_numpy(np.concatenate(uniforms)).cuda())
        # union minibatch m = the ranks' minibatch m slices, rank-major, global indices
        up = np.stack([np.concatenate([np.concatenate(
            [r * B + perms[r][e][m * mb:(m + 1) * mb] for r in range(world)])
            for m in range(M)]) for e in range(E)]).astype(np.int32)
        un.set_minibatch_permutation(torch.from_numpy(up).cuda())
        un_rows, un_gates = trace_heads(un)
        un.train_step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(un.b_act.cpu().numpy(), torch.cat(gathered['b_act']).numpy(),
                                      err_msg='actions')
        exact = []
        for k in ('b_logp', 'b_val', 'b_ret'):
            u, d = getattr(un, k).cpu().numpy(), torch.cat(gathered[k]).numpy()
            exact.append(bool(np.array_equal(u, d)))
            np.testing.assert_allclose(d, u, rtol=1e-5, atol=1e-6, err_msg=k)
        tu = un.model.theta.cpu().numpy().astype(np.float64)
        td = gathered['theta'][0].numpy().astype(np.float64)
        rel = np.linalg.norm(td - tu) / np.linalg.norm(tu - theta0)
        flips, worst = head_flips(heads, un_rows, world)
        gflips = gate_flips(gates, un_gates)
        print(f'CNN DP W={world} seed {base}: rollout buffers bit-equal {exact}, theta rel '
              f'{rel:.2e}, clip-branch flips (step, row, part) {flips}, other head rows within '
              f'{worst:.1e}, ReLU gate flips (step, layer, units) {gflips}', flush=True)
        # the union sums each minibatch's weight gradient over W x the rows in one pass, the
        # ranks in parts + an all-reduce: f32 regrouping, which also moves a few ReLU units
        # whose pre-activation sits at ~0 across their gate (reported; measured harmless:
        # 2.4e-7 .. 2.0e-6 with 4 .. 21 of them), unless a sample flips its PPO ratio or
        # value clip branch: that changes its gradient row by O(1) (round 4's 1.2e-4 at
        # record seed 55, profiles/r04ag_dprel.txt). A wrong exchange (a missing rank, a
        # stale bucket) deviates by O(1)
        assert len(flips) <= 8, f'{len(flips)} clip-branch flips: {flips}'
        bound = 2e-5 if not flips else 5e-4
        assert rel < bound, (f'data-parallel update deviates from the union update: {rel:.2e} '
                             f'({len(flips)} clip-branch flips {flips}, gate flips {gflips})')
        assert int(un.model.optimizer.iterations.item()) == E * M
    dist.barrier()
    print(f'CNN DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
