"""GPU parity tests: libxagents_hip.so (through the C ABI) vs the oracle.

Bars: bit-exact for integer actions, returns, rollout buffers and the Adam step
(same f32 operation order as oracle/xa_oracle.c); losses and gradients within
1e-5 relative (f32) of the float64 restatement of the reference TF math.
"""
import numpy as np
import oracle
import pytest
import torch

from xagents_amd import _lib, kernels

pytestmark = pytest.mark.gpu

GAE_GL = lambda g, l: float(np.float32(g * l))  # noqa: E731


def T(x, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(x), device='cuda', dtype=dtype)


def N(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _cases(golden, name):
    d = golden(name)
    for k in range(int(d['n_cases'])):
        yield k, {key[len(f'c{k}_'):]: d[key] for key in d.files if key.startswith(f'c{k}_')}


# ---- returns -------------------------------------------------------------
def test_gae_matches_reference_golden(device, golden):
    for k, c in _cases(golden, 'gae_cases.npz'):
        out = kernels.gae(T(c['rewards'].T), T(c['values'].T), T(c['dones'].T),
                          T(c['next_values']), float(c['gamma']), float(c['lam']))
        np.testing.assert_array_equal(N(out).T, c['returns'].astype(np.float32), err_msg=f'{k}')


def test_nstep_matches_reference_golden(device, golden):
    for k, c in _cases(golden, 'nstep_cases.npz'):
        out = kernels.nstep_returns(T(c['rewards'].T), T(c['dones'].T), T(c['next_values']),
                                    float(c['gamma']))
        np.testing.assert_array_equal(N(out).T, c['returns'], err_msg=f'{k}')


@pytest.mark.parametrize('n,t', [(1000, 300), (256, 128), (3, 1)])
def test_gae_large_vs_oracle(device, n, t):
    rng = np.random.default_rng(n + t)
    rew = rng.standard_normal((n, t)).astype(np.float32)
    val = rng.standard_normal((n, t)).astype(np.float32)
    done = (rng.random((n, t + 1)) < 0.03).astype(np.float32)
    nv = rng.standard_normal(n).astype(np.float32)
    out = kernels.gae(T(rew), T(val), T(done), T(nv), 0.99, 0.95)
    np.testing.assert_array_equal(N(out), oracle.gae(rew, val, done, nv, 0.99, GAE_GL(0.99, 0.95)))


# ---- forward / sampling ------------------------------------------------------
def _theta(obs_dim, A, seed, scale=0.3):
    P = kernels.mlp_param_count(obs_dim, A)
    return (np.random.default_rng(seed).standard_normal(P) * scale).astype(np.float32)


@pytest.mark.parametrize('obs_dim,A', [(4, 2), (6, 3), (8, 4), (2, 3)])
def test_mlp_forward_bit_exact(device, obs_dim, A):
    rng = np.random.default_rng(obs_dim)
    theta = _theta(obs_dim, A, 1)
    obs = (rng.standard_normal((1003, obs_dim)) * 2).astype(np.float32)
    u = rng.random(1003, dtype=np.float32)
    got = kernels.mlp_forward(T(theta), T(obs), A, uniforms=T(u), want_logits=True)
    ref = oracle.mlp_forward(theta, obs, A, uniforms=u)
    for g, r, name in zip(got, ref, ('act', 'logp', 'value', 'ent', 'logits')):
        np.testing.assert_array_equal(N(g), r, err_msg=name)
    acts = rng.integers(0, A, 1003).astype(np.int32)
    got = kernels.mlp_forward(T(theta), T(obs), A, actions=T(acts))
    ref = oracle.mlp_forward(theta, obs, A, actions=acts)
    np.testing.assert_array_equal(N(got[1]), ref[1])
    # float64 sanity of the whole forward
    *_, logits64, v64 = oracle.forward_f64(theta, obs, obs_dim, A)
    np.testing.assert_allclose(ref[4], logits64, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ref[2], v64, rtol=1e-5, atol=1e-5)


# ---- rollout -------------------------------------------------------------------
def _replay_env(n, t_rec, seed):
    from xagents_amd.envs import record_cartpole_replay

    return record_cartpole_replay(n, t_rec, seed=seed)


def _run_rollout(theta, rec, n, t, uniforms, seed, ctr, return_kind, n_rollouts=2, n_actions=2):
    s0, rep_obs, rep_state, rep_rew, rep_done = rec
    od = s0.shape[1]
    dev_env = dict(state=T(s0), done=torch.zeros(n, device='cuda'),
                   cursor=torch.zeros(n, dtype=torch.int32, device='cuda'),
                   ep_return=torch.zeros(n, device='cuda'))
    reps = [T(x) for x in (rep_obs, rep_state, rep_rew, rep_done)]
    host_env = dict(kind=0, state=s0.copy(), done=np.zeros(n, np.float32),
                    cursor=np.zeros(n, np.int32), ep_return=np.zeros(n, np.float32),
                    rep_obs=rep_obs, rep_state=rep_state, rep_rew=rep_rew, rep_done=rep_done)
    th = T(theta)
    ctr_t = torch.tensor([ctr], dtype=torch.int64, device='cuda')
    for r in range(n_rollouts):
        bufs = dict(obs=torch.zeros(n, t, od, device='cuda'),
                    act=torch.zeros(n, t, dtype=torch.int32, device='cuda'),
                    logp=torch.zeros(n, t, device='cuda'), val=torch.zeros(n, t, device='cuda'),
                    ent=torch.zeros(n, t, device='cuda'), rew=torch.zeros(n, t, device='cuda'),
                    done=torch.zeros(n, t + 1, device='cuda'), epret=torch.zeros(n, t, device='cuda'),
                    next_val=torch.zeros(n, device='cuda'), ret=torch.zeros(n, t, device='cuda'))
        a = _lib.XaRolloutArgs()
        a.n_envs, a.n_steps, a.obs_dim, a.n_actions = n, t, od, n_actions
        a.theta = th.data_ptr()
        a.env_kind = 0
        a.env_state, a.env_done = dev_env['state'].data_ptr(), dev_env['done'].data_ptr()
        a.env_cursor, a.ep_return = dev_env['cursor'].data_ptr(), dev_env['ep_return'].data_ptr()
        a.rep_obs, a.rep_state, a.rep_rew, a.rep_done = (x.data_ptr() for x in reps)
        a.t_rec = rep_obs.shape[1]
        u_r = None if uniforms is None else uniforms[r]
        u_t = None if u_r is None else T(u_r)
        a.uniforms = None if u_t is None else u_t.data_ptr()
        a.seed, a.rng_counter = seed, ctr_t.data_ptr()
        for k in ('obs', 'act', 'logp', 'val', 'ent', 'rew', 'done', 'epret', 'next_val', 'ret'):
            setattr(a, {'obs': 'obs_out', 'act': 'act_out', 'logp': 'logp_out', 'val': 'val_out',
                        'ent': 'ent_out', 'rew': 'rew_out', 'done': 'done_out',
                        'epret': 'epret_out', 'next_val': 'next_val', 'ret': 'ret_out'}[k],
                    bufs[k].data_ptr())
        a.return_kind = return_kind
        a.gamma, a.gamma_lam = 0.99, GAE_GL(0.99, 0.95)
        kernels.rollout(a)
        ref = oracle.mlp_rollout(theta, n_actions, host_env, t, uniforms=u_r, seed=seed, ctr=ctr + r,
                                 return_kind=return_kind)
        kernels.counter_bump(ctr_t)
        for k, v in bufs.items():
            np.testing.assert_array_equal(N(v), ref[k], err_msg=f'rollout {r} {k}')
        for k in ('state', 'done', 'cursor', 'ep_return'):
            np.testing.assert_array_equal(N(dev_env[k]), host_env[k], err_msg=f'env {k}')
    return ref


@pytest.mark.parametrize('return_kind', [1, 2])
def test_rollout_replay_uniforms_bit_exact(device, return_kind):
    n, t = 37, 50
    rec = _replay_env(n, 40, seed=5)
    rng = np.random.default_rng(9)
    u = [rng.random((n, t), dtype=np.float32) for _ in range(2)]
    ref = _run_rollout(_theta(4, 2, 3), rec, n, t, u, 0, 0, return_kind)
    assert ref['done'].sum() > 0


@pytest.mark.parametrize('n,t,t_rec,return_kind', [(3, 1, 7, 1), (5, 255, 97, 2), (4, 256, 300, 2),
                                                  (2, 300, 61, 1), (9, 16, 5, 1)])
def test_rollout_replay_ragged_rows_bit_exact(device, n, t, t_rec, return_kind):
    """Step counts around the batched rollout's 16-row tiles and 256-row passes (T + 1 rows,
    the last the bootstrap value), records that wrap inside a pass."""
    rec = _replay_env(n, t_rec, seed=t)
    rng = np.random.default_rng(t)
    u = [rng.random((n, t), dtype=np.float32) for _ in range(2)]
    _run_rollout(_theta(4, 2, t, 0.4), rec, n, t, u, 0, 0, return_kind)


@pytest.mark.parametrize('obs_dim,A', [(8, 4), (2, 3), (6, 3), (4, 2)])
def test_rollout_replay_synthetic_records_bit_exact(device, obs_dim, A):
    """Every (obs, actions) shape the library instantiates, on synthetic records with
    non-integer rewards (the episode-return and return chains must keep the step order
    exactly) and dones at random steps; 160 steps: two passes of 128 rows."""
    n, t, t_rec = 5, 160, 211
    rng = np.random.default_rng(obs_dim * 10 + A)
    s0 = rng.standard_normal((n, obs_dim)).astype(np.float32)
    rep_obs = rng.standard_normal((n, t_rec, obs_dim)).astype(np.float32)
    rep_state = rng.standard_normal((n, t_rec, obs_dim)).astype(np.float32)
    rep_rew = (rng.standard_normal((n, t_rec)) * 3.1).astype(np.float32)
    rep_done = (rng.random((n, t_rec)) < 0.05).astype(np.float32)
    u = [rng.random((n, t), dtype=np.float32) for _ in range(2)]
    for rk in (1, 2):
        _run_rollout(_theta(obs_dim, A, obs_dim + A, 0.4), (s0, rep_obs, rep_state, rep_rew,
                     rep_done), n, t, u, 0, 0, rk, n_actions=A)


def test_rollout_replay_philox_bit_exact(device):
    n, t = 64, 128
    rec = _replay_env(n, 300, seed=6)
    ref = _run_rollout(_theta(4, 2, 4, 0.5), rec, n, t, None, 0x1234567890, 77, 1, n_rollouts=3)
    acts = ref['act']
    assert 0.0 < acts.mean() < 1.0  # both actions are sampled


def test_rollout_cartpole_dynamics(device):
    from xagents_amd.envs import CartPoleVecEnv

    n, t = 16, 64
    env = CartPoleVecEnv(n, seed=3, device='cuda')
    host = dict(kind=1, state=N(env.state).copy(), state64=N(env.state64).copy(),
                done=np.zeros(n, np.float32), cursor=np.zeros(n, np.int32),
                ep_return=np.zeros(n, np.float32))
    theta = _theta(4, 2, 8, 0.2)
    th = T(theta)
    ctr = torch.zeros(1, dtype=torch.int64, device='cuda')
    bufs = [torch.zeros(n, t, 4, device='cuda'), torch.zeros(n, t, dtype=torch.int32, device='cuda')]
    bufs += [torch.zeros(n, t, device='cuda') for _ in range(5)]
    done = torch.zeros(n, t + 1, device='cuda')
    nv = torch.zeros(n, device='cuda')
    a = _lib.XaRolloutArgs()
    a.n_envs, a.n_steps, a.obs_dim, a.n_actions = n, t, 4, 2
    a.theta = th.data_ptr()
    env.fill_rollout_args(a)
    a.seed, a.rng_counter = 99, ctr.data_ptr()
    (a.obs_out, a.act_out, a.logp_out, a.val_out, a.ent_out, a.rew_out, a.epret_out) = (
        b.data_ptr() for b in bufs)
    a.done_out, a.next_val, a.ret_out, a.return_kind = done.data_ptr(), nv.data_ptr(), None, 0
    kernels.rollout(a)
    ref = oracle.mlp_rollout(theta, 2, host, t, seed=99, ctr=0, return_kind=0)
    # gym dynamics in f64 use cos/sin: device and host libm may differ in the last ulp
    np.testing.assert_allclose(N(bufs[0]), ref['obs'], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(N(bufs[1]), ref['act'])
    np.testing.assert_array_equal(N(done), ref['done'])
    np.testing.assert_allclose(N(env.state64), host['state64'], rtol=0, atol=1e-9)
    assert ref['done'].sum() > 0


# ---- update -----------------------------------------------------------------------
def _rand_batch(rng, B, obs_dim, A, theta):
    obs = rng.standard_normal((B, obs_dim)).astype(np.float32)
    acts = rng.integers(0, A, B).astype(np.int32)
    _, logp, val, _, _ = oracle.mlp_forward(theta, obs, A, actions=acts)
    old_logp = (logp + rng.normal(0, 0.1, B)).astype(np.float32)
    old_val = (val + rng.normal(0, 0.3, B)).astype(np.float32)
    ret = (old_val + rng.normal(0, 1.0, B)).astype(np.float32)
    return obs, acts, old_logp, old_val, ret


def _grad_on_gpu(kind, theta, obs, acts, old_logp, old_val, ret, perm, epoch, m, MB,
                 stats=None, count=None):
    B, obs_dim = obs.shape
    A = 2 if theta.size == kernels.mlp_param_count(obs_dim, 2) else 3
    nb = kernels.ac_grad_blocks(MB)
    P = theta.size
    part = torch.zeros(nb, P, device='cuda')
    lossp = torch.zeros(nb, 4, device='cuda')
    keep = [T(theta), T(obs), T(acts), T(old_logp), T(old_val), T(ret)]
    g = _lib.XaAcGradArgs()
    g.obs_dim, g.n_actions, g.loss_kind = obs_dim, A, kind
    g.theta, g.obs, g.actions, g.old_logp, g.old_values, g.returns = (k.data_ptr() for k in keep)
    g.batch, g.mb_size, g.epoch, g.mb_index = B, MB, epoch, m
    sh = _lib.XaShuffle()
    perm_t = T(perm.astype(np.int32)) if perm is not None else None
    sh.perm = None if perm_t is None else perm_t.data_ptr()
    g.shuffle = sh
    if stats is not None:
        keep.append(stats)
        g.adv_stats, g.adv_count = stats.data_ptr(), float(count)
    g.clip_norm, g.entropy_coef, g.value_coef, g.adv_eps = 0.1, 0.01, 0.5, 1e-8
    cnt = min(MB, B - m * MB)
    g.loss_scale = 1.0 / cnt
    g.n_blocks, g.partials, g.loss_partials = nb, part.data_ptr(), lossp.data_ptr()
    kernels.ac_grad(g)
    grad = torch.zeros(P, device='cuda')
    kernels.grad_reduce(part, grad)
    return N(grad), N(lossp).sum(0)


def _assert_grad_close(got, ref, what):
    err = np.abs(got - ref).max() / np.abs(ref).max()
    rel_norm = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert err < 1e-5 and rel_norm < 1e-5, f'{what}: max-rel {err:.2e} norm-rel {rel_norm:.2e}'


@pytest.mark.parametrize('B,MB', [(2048, 512), (1000, 333), (32768, 8192)])
def test_ppo_grad_vs_f64(device, B, MB):
    rng = np.random.default_rng(B)
    theta = _theta(4, 2, 11, 0.2)
    obs, acts, old_logp, old_val, ret = _rand_batch(rng, B, 4, 2, theta)
    E = 2
    perms = np.stack([rng.permutation(B) for _ in range(E)]).astype(np.int32)
    n_mb = (B + MB - 1) // MB
    stats = torch.zeros(kernels.adv_stats_size(B, MB, E), dtype=torch.float64, device='cuda')
    sh = _lib.XaShuffle()
    perm_t = T(perms)
    sh.perm = perm_t.data_ptr()
    kernels.adv_stats(T(ret), T(old_val), B, MB, E, sh, stats)
    st = N(stats).reshape(E, n_mb, -1, 2).sum(2)
    for e in range(E):
        for m in range(n_mb):
            idx = perms[e, m * MB:(m + 1) * MB]
            adv = ret[idx].astype(np.float64) - old_val[idx]
            adv32 = (ret[idx] - old_val[idx]).astype(np.float64)
            np.testing.assert_allclose(st[e, m], [adv32.sum(), (adv32 ** 2).sum()], rtol=1e-11)
            if (e, m) not in ((0, 0), (E - 1, n_mb - 1)):
                continue
            got, lp = _grad_on_gpu(0, theta, obs, acts, old_logp, old_val, ret, perms, e, m, MB,
                                   stats, len(idx))
            advn = oracle.normalize_advantages(ret[idx], old_val[idx])
            terms, ref = oracle.ac_loss_grad_f64(theta, obs[idx], acts[idx], ret[idx],
                                                 old_val[idx], 2, 'ppo', old_logp[idx], advn)
            _assert_grad_close(got, ref, f'e{e} m{m}')
            assert lp[3] == len(idx)
            np.testing.assert_allclose(lp[0], terms['pg_sum'], rtol=1e-5, atol=1e-4)
            np.testing.assert_allclose(lp[1], terms['vl_sum'], rtol=1e-5)
            np.testing.assert_allclose(lp[2], terms['ent_sum'], rtol=1e-5)


def test_a2c_grad_vs_f64(device):
    rng = np.random.default_rng(2)
    B = 1280
    theta = _theta(4, 2, 12, 0.2)
    obs, acts, old_logp, old_val, ret = _rand_batch(rng, B, 4, 2, theta)
    got, lp = _grad_on_gpu(1, theta, obs, acts, old_logp, old_val, ret, None, 0, 0, B)
    terms, ref = oracle.ac_loss_grad_f64(theta, obs, acts, ret, old_val, 2, 'a2c')
    _assert_grad_close(got, ref, 'a2c')
    np.testing.assert_allclose(lp[1], terms['vl_sum'], rtol=1e-5)


def test_feistel_shuffle_matches_oracle(device):
    """The device shuffle (no host perm) visits exactly oracle.shuffle_perm's order."""
    B, MB, E = 4096, 1024, 3
    rng = np.random.default_rng(0)
    ret = rng.standard_normal(B).astype(np.float32)
    val = np.zeros(B, np.float32)
    ctr = torch.tensor([5], dtype=torch.int64, device='cuda')
    sh = _lib.XaShuffle()
    sh.perm, sh.seed, sh.rng_counter = None, 4242, ctr.data_ptr()
    stats = torch.zeros(kernels.adv_stats_size(B, MB, E), dtype=torch.float64, device='cuda')
    kernels.adv_stats(T(ret), T(val), B, MB, E, sh, stats)
    st = N(stats).reshape(E, 4, -1, 2).sum(2)
    for e in range(E):
        p = oracle.shuffle_perm(B, e, 4242, 5)
        for m in range(4):
            np.testing.assert_allclose(st[e, m, 0], ret[p[m * MB:(m + 1) * MB]].astype(np.float64).sum(),
                                       rtol=1e-11)


@pytest.mark.parametrize('P', [4675, 70001])
def test_clip_adam_bit_exact(device, P):
    rng = np.random.default_rng(P)
    theta = rng.standard_normal(P).astype(np.float32)
    m = (rng.standard_normal(P) * 1e-2).astype(np.float32)
    v = np.abs(rng.standard_normal(P) * 1e-3).astype(np.float32)
    g = rng.standard_normal(P).astype(np.float32)
    tt, mt, vt, gt = T(theta), T(m), T(v), T(g)
    step = torch.tensor([4], dtype=torch.int32, device='cuda')
    ws = torch.zeros(1024, dtype=torch.float64, device='cuda')
    gn = torch.zeros(1, device='cuda')
    kernels.clip_adam(tt, mt, vt, gt, step, 7e-4, 0.9, 0.999, 1e-7, clip_norm=0.5,
                      workspace=ws, gnorm_out=gn)
    th_r, m_r, v_r, gn_r = oracle.clip_adam(theta, m, v, g, 4, 7e-4, 0.9, 0.999, 1e-7, 0.5)
    assert abs(float(N(gn)[0]) - gn_r) <= 1e-6 * gn_r
    np.testing.assert_array_equal(N(mt), m_r)
    np.testing.assert_array_equal(N(vt), v_r)
    np.testing.assert_array_equal(N(tt), th_r)


def test_grad_reduce_and_adam_step_counter(device):
    part = torch.randn(37, 999, device='cuda')
    grad = torch.zeros(999, device='cuda')
    step = torch.zeros(1, dtype=torch.int32, device='cuda')
    kernels.grad_reduce(part, grad, step)
    kernels.grad_reduce(part, grad, step)
    ref = N(part).astype(np.float64).sum(0).astype(np.float32)
    np.testing.assert_allclose(N(grad), ref, rtol=1e-6, atol=1e-6)
    assert int(N(step)[0]) == 2


def test_errors_are_loud(device):
    a = _lib.XaRolloutArgs()
    with pytest.raises(_lib.HipLibraryError, match='n_envs'):
        kernels.rollout(a)
    with pytest.raises(_lib.HipLibraryError, match='unsupported'):
        kernels.mlp_forward(torch.zeros(100, device='cuda'), torch.zeros(3, 5, device='cuda'), 2,
                            uniforms=torch.zeros(3, device='cuda'))


@pytest.mark.parametrize('P,nb,clip', [(4675, 256, 0.5), (999, 37, 0.0), (65536, 3, 0.5)])
def test_grad_reduce_adam_tail_bit_exact(device, P, nb, clip):
    """xa_grad_reduce_adam (last block: clip + Keras Adam) == xa_grad_reduce followed by
    xa_clip_adam, bit for bit, incl. the step counter; repeated launches reuse the
    self-resetting arrival counter; the C oracle agrees with the result."""
    rng = np.random.default_rng(P)
    part = T((rng.standard_normal((nb, P)) * 1e-2).astype(np.float32))
    theta = rng.standard_normal(P).astype(np.float32)
    m = (rng.standard_normal(P) * 1e-3).astype(np.float32)
    v = np.abs(rng.standard_normal(P) * 1e-5).astype(np.float32)
    ref = [T(theta), T(m), T(v)]
    got = [T(theta), T(m), T(v)]
    step_r = torch.tensor([6], dtype=torch.int32, device='cuda')
    step_g = torch.tensor([6], dtype=torch.int32, device='cuda')
    arrivals = torch.zeros(1, dtype=torch.int32, device='cuda')
    grad_r = torch.zeros(P, device='cuda')
    grad_g = torch.zeros(P, device='cuda')
    gn = torch.zeros(1, device='cuda')
    ws = torch.zeros(1024, dtype=torch.float64, device='cuda')
    cn = clip if clip > 0 else None
    tail = kernels.adam_tail(*got, step_g, arrivals, 7e-4, 0.9, 0.999, 1e-7, clip_norm=cn,
                             gnorm_out=gn)
    host_th, host_m, host_v = theta, m, v
    for it in range(3):
        kernels.grad_reduce(part, grad_r, step_r)
        kernels.clip_adam(*ref, grad_r, step_r, 7e-4, 0.9, 0.999, 1e-7, clip_norm=cn,
                          workspace=ws)
        kernels.grad_reduce_adam(part, grad_g, tail)
        np.testing.assert_array_equal(N(grad_g), N(grad_r))
        for a, b, name in zip(got, ref, ('theta', 'm', 'v')):
            np.testing.assert_array_equal(N(a), N(b), err_msg=f'{name} it {it}')
        assert int(N(step_g)[0]) == int(N(step_r)[0]) == 7 + it
        assert int(N(arrivals)[0]) == 0
        host_th, host_m, host_v, gn_r = oracle.clip_adam(host_th, host_m, host_v, N(grad_r),
                                                         7 + it, 7e-4, 0.9, 0.999, 1e-7, clip)
        np.testing.assert_array_equal(N(got[0]), host_th)
        assert abs(float(N(gn)[0]) - gn_r) <= 1e-6 * gn_r


def test_grad_reduce_adam_rejects_large_models(device):
    part = torch.zeros(2, 70000, device='cuda')
    z = torch.zeros(70000, device='cuda')
    one = torch.zeros(1, dtype=torch.int32, device='cuda')
    tail = kernels.adam_tail(z, z, z, one, one, 7e-4, 0.9, 0.999, 1e-7)
    with pytest.raises(_lib.HipLibraryError, match='n_params'):
        kernels.grad_reduce_adam(part, z, tail)


def test_pending_optimizer_step_in_ac_grad_prologue(device):
    """xa_ac_grad with a pending step == xa_clip_adam (out of place) followed by a plain
    xa_ac_grad: same new theta/m/v (written by block 0) and the same partial gradients."""
    rng = np.random.default_rng(77)
    B, MB = 4096, 1024
    theta = _theta(4, 2, 21, 0.2)
    obs, acts, old_logp, old_val, ret = _rand_batch(rng, B, 4, 2, theta)
    P = theta.size
    g_pend = T((rng.standard_normal(P) * 1e-2).astype(np.float32))
    m0 = T((rng.standard_normal(P) * 1e-3).astype(np.float32))
    v0 = T(np.abs(rng.standard_normal(P) * 1e-5).astype(np.float32))
    step = torch.tensor([7], dtype=torch.int32, device='cuda')
    th_t = T(theta)
    # reference path: out-of-place clip + Adam, then a plain gradient launch
    th_r, m_r, v_r = (torch.zeros(P, device='cuda') for _ in range(3))
    kernels.clip_adam(th_t, m0, v0, g_pend, step, 7e-4, 0.9, 0.999, 1e-7, clip_norm=0.5,
                      out=(th_r, m_r, v_r))
    nb = kernels.ac_grad_blocks(MB)
    keep = [T(obs), T(acts), T(old_logp), T(old_val), T(ret)]
    perm = T(np.stack([rng.permutation(B)]).astype(np.int32))
    stats = torch.zeros(kernels.adv_stats_size(B, MB, 1), dtype=torch.float64, device='cuda')
    sh = _lib.XaShuffle()
    sh.perm = perm.data_ptr()
    kernels.adv_stats(keep[4], keep[3], B, MB, 1, sh, stats)

    def launch(theta_src, pending):
        part = torch.zeros(nb, P, device='cuda')
        g = _lib.XaAcGradArgs()
        g.obs_dim, g.n_actions, g.loss_kind = 4, 2, 0
        g.theta = theta_src.data_ptr()
        g.obs, g.actions, g.old_logp, g.old_values, g.returns = (k.data_ptr() for k in keep)
        g.batch, g.mb_size, g.epoch, g.mb_index = B, MB, 0, 1
        g.shuffle = sh
        g.adv_stats, g.adv_count = stats.data_ptr(), float(MB)
        g.clip_norm, g.entropy_coef, g.value_coef, g.adv_eps = 0.1, 0.01, 0.5, 1e-8
        g.loss_scale = 1.0 / MB
        g.n_blocks, g.partials = nb, part.data_ptr()
        outs = None
        if pending:
            outs = [torch.zeros(P, device='cuda') for _ in range(3)]
            g.pend_grad, g.pend_m, g.pend_v = g_pend.data_ptr(), m0.data_ptr(), v0.data_ptr()
            g.theta_out, g.m_out, g.v_out = (o.data_ptr() for o in outs)
            g.adam_step = step.data_ptr()
            g.adam = kernels.adam_struct(7e-4, 0.9, 0.999, 1e-7, clip_norm=0.5)
        kernels.ac_grad(g)
        return part, outs

    part_ref, _ = launch(th_r, False)
    part_got, outs = launch(th_t, True)
    for got, ref, name in zip(outs, (th_r, m_r, v_r), ('theta', 'm', 'v')):
        np.testing.assert_array_equal(N(got), N(ref), err_msg=name)
    np.testing.assert_array_equal(N(part_got), N(part_ref))


@pytest.mark.parametrize('sizes', [(16 * 129, 16 * 128, 1), (256 * 129, 256 * 128), (1,), (3, 5)])
def test_copy_to_host_segments_bit_exact(device, sizes):
    """xa_copy_to_host (episode statistics, base.py _copy_to_host): every segment lands in
    its pinned host buffer word for word (f32 bit patterns incl. NaN payloads, int32)."""
    import ctypes
    g = torch.Generator().manual_seed(len(sizes))
    src, dst = [], []
    for i, n in enumerate(sizes):
        if i == 2:
            h = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, generator=g)
        else:
            h = torch.randn(n, generator=g)
            if n:
                h.view(torch.int32)[::7] = 0x7fc01234  # quiet NaN with a payload
        src.append(h.to(device))
        dst.append(torch.full_like(h, 0).pin_memory())
    a = _lib.XaHostCopyArgs()
    a.n_segments = len(sizes)
    for i, (d, h) in enumerate(zip(src, dst)):
        dev = ctypes.c_void_p()
        _lib.call('xa_host_device_pointer', ctypes.c_void_p(h.data_ptr()), ctypes.byref(dev))
        a.src[i], a.dst[i], a.bytes[i] = d.data_ptr(), dev.value, d.numel() * d.element_size()
    _lib.call('xa_copy_to_host', ctypes.byref(a), _lib.stream())
    torch.cuda.synchronize()
    for d, h in zip(src, dst):
        assert torch.equal(d.cpu().view(torch.int32), h.view(torch.int32))
    a.bytes[0] = 6  # not a multiple of 4
    with pytest.raises(_lib.HipLibraryError, match='multiple of 4'):
        _lib.call('xa_copy_to_host', ctypes.byref(a), _lib.stream())
