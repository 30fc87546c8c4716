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
order), parameters identical on every rank and 16 optimizer steps taken.

The parameter bound is against a float64 REPLAY of the union train step that takes the
data-parallel ranks' own discrete decisions: starting from theta_0,
every optimizer step runs the f64 forward of the union minibatch (oracle/nets_torch64.py
on the test GPU) with the ReLU gate pattern the ranks' f32 forwards produced, the clipped
PPO loss gradient with each sample's clip branches (policy: ratio clip active or not;
value: unclipped, clipped or cut) as the ranks took them, then clip_by_global_norm and
Keras Adam in f64. A sample whose PPO ratio or value sits within f32 rounding of a clip
boundary, or a unit at pre-activation ~0, may decide differently in f32 and f64; adopting
the device's decisions removes those O(1) jumps, so the data-parallel theta must match the
replay within 2e-5 of the update's norm at every record seed, flips or not. A rank's
branch decision is read from its recorded head-gradient row: the candidate row (f64) of
each branch nearest to it (candidates differ by O(1); an argmin, no threshold). The f32
union run is still compared and its flip counts reported (information only).
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


def replay_f64(model, theta0, it0, grad_norm, rows, heads, gates, world, dev='cuda'):
    """The float64 replay of the union train step with the data-parallel ranks' decisions.
    rows[k] = (x uint8 [n, ...], act, old logp, old value, return) of union minibatch k
    (rank-major), heads[k] = the ranks' recorded [d logits | d value] rows (each rank's
    loss is its local mean: W x the union's scale), gates[k] = their packed ReLU gate rows.
    Returns theta after the E x M steps and the adopted flip counts (samples whose adopted
    branch differs from the f64 forward's own choice; gates likewise)."""
    import nets_torch64 as OT
    import oracle as OR
    dev = torch.device(dev)
    opt = model.optimizer
    f32 = lambda v: float(np.float32(v))  # noqa: E731 (TF ApplyAdam's f32 hyper-parameters)
    th = torch.from_numpy(theta0).to(dev)
    m = np.zeros_like(theta0)
    v = np.zeros_like(theta0)
    relu = [i for i, l in enumerate(model.layers)
            if l.kind != 'flatten' and getattr(l, 'activation', None) == 'relu']
    o_logits, o_value = model.outputs
    clip, ent_coef, v_coef, eps = 0.1, 0.01, 0.5, 1e-8
    branch_flips = gate_flips = 0
    for k, ((x, act, oldlp, oldv, ret), hd, gk) in enumerate(zip(rows, heads, gates)):
        n = x.shape[0]
        assert len(gk) == len(relu), (len(gk), relu)
        gmap = {}
        for i, packed in zip(relu, gk):
            units = int(np.prod(model.layers[i].out_shape))
            mask = np.unpackbits(packed.numpy(), axis=1)[:, :units].astype(bool)
            gmap[i] = torch.from_numpy(mask).to(dev)
        thg = th.clone().requires_grad_(True)
        xd = torch.from_numpy(x).to(dev)
        _, outs = OT.forward(model.layers, thg, xd, model.input_shape, gates=gmap)
        with torch.no_grad():
            _, own = OT.forward(model.layers, th, xd, model.input_shape)
            for i in relu:
                gate_flips += int(((own[i] > 0) != gmap[i].reshape(own[i].shape)).sum())
            del own
        logits, val = outs[o_logits], outs[o_value][:, 0]
        lg = logits.detach().cpu().numpy()
        vv = val.detach().cpu().numpy()
        lsm = OR.log_softmax(lg)
        p = np.exp(lsm)
        A = lg.shape[1]
        logp = lsm[np.arange(n), act]
        H = -(p * lsm).sum(-1)
        adv = ret - oldv
        adv = (adv - adv.mean()) / (adv.std() + eps)
        ratio = np.exp(logp - oldlp)
        onehot = np.eye(A)[act]
        ent = (ent_coef / n) * p * (lsm + H[:, None])
        # candidate rows of every branch (xagents/ppo/agent.py:112-134 as the device's
        # loss: tf.maximum / clip_by_value tie rules)
        dz_on = (-adv * ratio / n)[:, None] * (onehot - p) + ent
        dz_off = ent
        dvo = vv - oldv
        vclip = oldv + np.clip(dvo, -clip, clip)
        dv_c = [v_coef * (vv - ret) / n, v_coef * (vclip - ret) / n, np.zeros(n)]
        d = hd.double().numpy() / world
        pick_on = (np.linalg.norm(dz_on - d[:, :-1], axis=1) <=
                   np.linalg.norm(dz_off - d[:, :-1], axis=1))
        vi = np.argmin(np.stack([np.abs(c - d[:, -1]) for c in dv_c]), axis=0)
        # the f64 forward's own decisions, for the report
        pg1, pg2 = -adv * ratio, -adv * np.clip(ratio, 1 - clip, 1 + clip)
        own_on = (pg1 >= pg2) | ((ratio >= 1 - clip) & (ratio <= 1 + clip))
        vl1, vl2 = (vv - ret) ** 2, (vclip - ret) ** 2
        own_vi = np.where(vl1 >= vl2, 0, np.where((dvo >= -clip) & (dvo <= clip), 1, 2))
        branch_flips += int((pick_on != own_on).sum() + (vi != own_vi).sum())
        dz = np.where(pick_on[:, None], dz_on, dz_off)
        dv = np.choose(vi, dv_c)
        g, = torch.autograd.grad([logits, outs[o_value]], [thg], grad_outputs=[
            torch.from_numpy(dz).to(dev), torch.from_numpy(dv[:, None]).to(dev)])
        del outs, logits, val, thg
        g = g.cpu().numpy()
        gc = OR.clip_by_global_norm_f64(g, grad_norm)[0]
        t0 = th.cpu().numpy()
        t1, m, v = OR.keras_adam_f64(t0, m, v, gc, it0 + k + 1, f32(opt.learning_rate),
                                     f32(opt.beta_1), f32(opt.beta_2), f32(opt.epsilon))
        th = torch.from_numpy(t1).to(dev)
    return th.cpu().numpy(), branch_flips, gate_flips


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
    got['obs'] = dp.obs_buf[:T].cpu()  # [T, N, 84, 84, 1] uint8, the step's frames
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
        sys.path.insert(0, str(ROOT / 'oracle'))
        # the union minibatch rows of every optimizer step: rank-major, each rank's own
        # minibatch slice of its shard (the order the gathered head rows / gates follow)
        rows = []
        for k in range(E * M):
            e, mi = divmod(k, M)
            xs, fields = [], [[] for _ in range(4)]
            for r in range(world):
                idx = perms[r][e][mi * mb:(mi + 1) * mb]
                env, t = idx // T, idx % T  # flat env-major index i = env * T + t
                xs.append(gathered['obs'][r].numpy()[t, env])
                for f, key in enumerate(('b_act', 'b_logp', 'b_val', 'b_ret')):
                    fields[f].append(gathered[key][r].reshape(-1).numpy()[idx])
            act, oldlp, oldv, ret = (np.concatenate(f) for f in fields)
            rows.append((np.concatenate(xs), act.astype(np.int64), oldlp.astype(np.float64),
                         oldv.astype(np.float64), ret.astype(np.float64)))
        th64, bflips64, gflips64 = replay_f64(dp.model, theta0, it0, dp.grad_norm, rows, heads,
                                              gates, world)
        td = gathered['theta'][0].numpy().astype(np.float64)
        rel64 = np.linalg.norm(td - th64) / np.linalg.norm(th64 - theta0)
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
        print(f'CNN DP W={world} seed {base}: theta vs the f64 replay with the ranks\' '
              f'decisions {rel64:.2e} (adopted: {bflips64} clip branches, {gflips64} ReLU gates '
              f'differ from the f64 forward\'s own); vs the f32 union run {rel:.2e} '
              f'(information: rollout buffers bit-equal {exact}, clip-branch flips (step, row, '
              f'part) {flips}, other head rows within {worst:.1e}, ReLU gate flips (step, '
              f'layer, units) {gflips})', flush=True)
        # one bound, flips or not: the replay takes the ranks' discrete decisions, so what
        # remains is f32 rounding (regrouped sums, the all-reduce); a wrong exchange (a
        # missing rank, a stale bucket) deviates by O(1)
        assert rel64 < 2e-5, (f'data-parallel update deviates from the f64 replay of the '
                              f'union step: {rel64:.2e} ({bflips64} adopted branch flips, '
                              f'{gflips64} gate flips)')
        assert int(un.model.optimizer.iterations.item()) == E * M
    dist.barrier()
    print(f'CNN DP OK {rank}', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
