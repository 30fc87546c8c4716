"""GPU tests of the persistent PPO update (xa_ppo_update): every optimizer step of a train
step in one launch (xagents/ppo/agent.py:96-191), against the float64 restatement
(oracle/oracle.py) and against the per-minibatch launch chain."""
import ctypes

import numpy as np
import oracle
import pytest
import torch

pytestmark = pytest.mark.gpu

OBS, A = 4, 2
LR, B1, B2, EPS, CLIP_G = 7e-4, 0.9, 0.999, 1e-7, 0.5


def _rollout_buffers(B, seed):
    """Synthetic rollout buffers shaped like a CartPole rollout (env-major flat)."""
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((B, OBS)).astype(np.float32)
    act = rng.integers(0, A, B).astype(np.int32)
    val = (rng.standard_normal(B) * 0.5).astype(np.float32)
    ret = (val + rng.standard_normal(B)).astype(np.float32)
    logp = np.log(rng.uniform(0.2, 0.8, B)).astype(np.float32)
    return obs, act, logp, val, ret


def _theta0(seed):
    rng = np.random.default_rng(seed + 100)
    return (rng.standard_normal(4675) * 0.2).astype(np.float32)


def run_update(theta0, bufs, mb_size, epochs, perm=None, n_blocks=None, want=True, trace=False,
               placement=0):
    """Call xa_ppo_update directly; returns theta, m, v, step, grad_out, loss_out, status
    (and, with trace, theta at the start of every optimizer step and every step's
    reduced gradient)."""
    from xagents_amd import kernels
    from xagents_amd._lib import XaPpoUpdateArgs, XaShuffle
    obs, act, logp, val, ret = (torch.as_tensor(x, device='cuda') for x in bufs)
    B = obs.shape[0]
    n_mb = (B + mb_size - 1) // mb_size
    K = epochs * n_mb
    G = kernels.ppo_update_blocks(OBS, A, mb_size)
    assert G > 0
    if n_blocks is not None:
        G = min(G, n_blocks)
    theta = torch.as_tensor(theta0, device='cuda').clone()
    m, v = torch.zeros_like(theta), torch.zeros_like(theta)
    step = torch.zeros(1, dtype=torch.int32, device='cuda')
    nbytes = kernels.ppo_update_workspace_bytes(OBS, A, B, mb_size, epochs, G)
    ws = torch.zeros(nbytes, dtype=torch.uint8, device='cuda')  # zeroed once, as required
    grad = torch.zeros_like(theta)
    loss = torch.zeros(K, G, 4, dtype=torch.float32, device='cuda')
    status = torch.zeros(1, dtype=torch.int32, device='cuda')
    sh = XaShuffle()
    perm_t = None
    if perm is not None:
        perm_t = torch.as_tensor(np.asarray(perm, np.int32).ravel(), device='cuda')
        sh.perm = perm_t.data_ptr()
    else:
        sh.perm = None
    sh.seed, sh.rng_counter = 12345, None
    u = XaPpoUpdateArgs()
    u.obs_dim, u.n_actions, u.batch, u.mb_size, u.epochs = OBS, A, B, mb_size, epochs
    u.shuffle = sh
    u.obs, u.actions, u.old_logp = obs.data_ptr(), act.data_ptr(), logp.data_ptr()
    u.old_values, u.returns = val.data_ptr(), ret.data_ptr()
    u.clip_norm, u.entropy_coef, u.value_coef, u.adv_eps = 0.1, 0.01, 0.5, 1e-8
    u.theta, u.adam_m, u.adam_v, u.adam_step = (theta.data_ptr(), m.data_ptr(), v.data_ptr(),
                                                step.data_ptr())
    u.adam = kernels.adam_struct(LR, B1, B2, EPS, clip_norm=CLIP_G)
    u.workspace, u.workspace_bytes = ws.data_ptr(), nbytes
    u.loss_out = loss.data_ptr() if want else None
    u.grad_out = grad.data_ptr() if want else None
    u.status = status.data_ptr()
    u.n_blocks = G
    u.placement = placement
    if trace:
        th_tr = torch.zeros(K, theta.numel(), dtype=torch.float32, device='cuda')
        g_tr = torch.zeros_like(th_tr)
        u.theta_trace, u.grad_trace = th_tr.data_ptr(), g_tr.data_ptr()
    kernels.ppo_update(u)
    torch.cuda.synchronize()
    out = dict(theta=theta.cpu().numpy(), m=m.cpu().numpy(), v=v.cpu().numpy(),
               step=int(step.item()), grad=grad.cpu().numpy(), loss=loss.cpu().numpy(),
               status=int(status.item()), G=G, K=K)
    if trace:
        out['theta_trace'], out['grad_trace'] = th_tr.cpu().numpy(), g_tr.cpu().numpy()
    return out


def f64_trajectory(theta0, bufs, mb_size, perms):
    """The reference update (ppo/agent.py:139-191) in float64 for given permutations."""
    obs, act, logp, val, ret = bufs
    B = obs.shape[0]
    th = theta0.astype(np.float64)
    m, v = np.zeros_like(th), np.zeros_like(th)
    t = 0
    grads, terms = [], []
    for perm in perms:
        for start in range(0, B, mb_size):
            idx = perm[start:start + mb_size]
            adv = oracle.normalize_advantages(ret[idx], val[idx])
            tm, g = oracle.ac_loss_grad_f64(th, obs[idx], act[idx], ret[idx], val[idx], A, 'ppo',
                                            logp[idx], adv)
            grads.append(g)
            terms.append(tm)
            g, _ = oracle.clip_by_global_norm_f64(g, CLIP_G)
            t += 1
            th, m, v = oracle.keras_adam_f64(th, m, v, g, t, LR, B1, B2, EPS)
    return th, m, v, grads, terms


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


@pytest.mark.parametrize('B,mb', [(512, 512), (8192, 8192), (600, 600)])
def test_single_step_gradient_and_losses_vs_f64(device, B, mb):
    """One optimizer step (E = M = 1): the raw reduced gradient and the per-minibatch loss
    sums are scale-sensitive checks of the fused loss / backward (1e-5 rel)."""
    bufs = _rollout_buffers(B, seed=B)
    theta0 = _theta0(1)
    rng = np.random.default_rng(7)
    perm = rng.permutation(B).astype(np.int32)[None]
    out = run_update(theta0, bufs, mb, 1, perm=perm)
    assert out['status'] == 0 and out['step'] == 1
    th, m, v, grads, terms = f64_trajectory(theta0, bufs, mb, perm)
    assert _rel(out['grad'], grads[0]) < 1e-5
    ls = out['loss'].sum(axis=1)[0]
    assert ls[3] == B
    np.testing.assert_allclose(ls[0], terms[0]['pg_sum'], rtol=1e-5, atol=1e-5 * B)
    np.testing.assert_allclose(ls[1], terms[0]['vl_sum'], rtol=1e-5)
    np.testing.assert_allclose(ls[2], terms[0]['ent_sum'], rtol=1e-5)
    # the first Adam moments carry the clipped gradient's scale: m = (1 - b1) g_clip
    g64, _ = oracle.clip_by_global_norm_f64(grads[0], CLIP_G)
    assert _rel(out['m'], (1 - B1) * g64) < 1e-5
    assert _rel(out['v'], (1 - B2) * g64 * g64) < 2e-5


def test_multi_step_ragged_trajectory_vs_f64(device):
    """2 epochs x 4 minibatches of a 600-sample batch with mb 198, the 4th ragged (the
    reference slices range(0, B, mb): 600 = 3 x 198 + 6): host permutations, Adam moments
    non-zero after the first step."""
    B, mb, E = 600, 198, 2
    bufs = _rollout_buffers(B, seed=11)
    theta0 = _theta0(2)
    rng = np.random.default_rng(3)
    perms = np.stack([rng.permutation(B) for _ in range(E)]).astype(np.int32)
    out = run_update(theta0, bufs, mb, E, perm=perms)
    n_mb = 4
    assert out['status'] == 0 and out['step'] == E * n_mb
    th, m, v, grads, terms = f64_trajectory(theta0, bufs, mb, perms)
    assert _rel(out['theta'] - theta0, th - theta0) < 2e-3
    assert _rel(out['m'], m) < 2e-3
    # every minibatch's sample count (the ragged one has 6)
    counts = out['loss'].sum(axis=1)[:, 3]
    np.testing.assert_array_equal(counts, [198, 198, 198, 6] * E)


@pytest.mark.parametrize('B,mb,blocks', [(4096, 1024, (32, 5)), (16384, 8192, (256, 64, 40, 7)),
                                         (2048, 512, (16, 32, 23))])
def test_block_count_changes_only_the_summation_order(device, B, mb, blocks):
    """Fewer resident blocks than tiles: each block walks several tiles. 64 and more
    blocks reduce the gradient rows inside each XCD's L2 first (two-level), fewer in one
    level; more blocks than 32-sample tiles run 16-sample tiles (mb 512: 32 and 23
    blocks). Only the f32 / f64 summation order of the gradient changes."""
    bufs = _rollout_buffers(B, seed=5)
    theta0 = _theta0(3)
    runs = [run_update(theta0, bufs, mb, 2, n_blocks=g) for g in blocks]
    ref = runs[0]
    assert ref['G'] == blocks[0]
    for r, g in zip(runs, blocks):
        assert r['G'] == g and r['status'] == 0 and r['step'] == 2 * (B // mb)
        assert _rel(r['grad'], ref['grad'].astype(np.float64)) < 1e-5, g
        assert _rel(r['theta'] - theta0, (ref['theta'] - theta0).astype(np.float64)) < 1e-4, g


def test_feistel_shuffle_matches_oracle_permutation(device):
    """No host permutation: the device Feistel shuffle is oracle.shuffle_perm's."""
    B, mb = 1024, 256
    bufs = _rollout_buffers(B, seed=9)
    theta0 = _theta0(4)
    out = run_update(theta0, bufs, mb, 2)
    perms = np.stack([oracle.shuffle_perm(B, e, 12345, 0) for e in range(2)])
    th, m, v, grads, _ = f64_trajectory(theta0, bufs, mb, perms)
    assert out['status'] == 0 and out['step'] == 8
    assert _rel(out['theta'] - theta0, th - theta0) < 2e-3


def test_agent_persistent_update_matches_chain(device, monkeypatch):
    """Same rollout, one train step: the persistent launch and the per-minibatch chain
    give the same parameters up to the f64 reduction order."""
    from test_gpu_agent import make_agent
    monkeypatch.setenv('XA_PPO_UPDATE', 'persistent')
    a = make_agent(n_envs=32, n_steps=64, seed=5, use_graph=False)
    monkeypatch.setenv('XA_PPO_UPDATE', 'chain')
    b = make_agent(n_envs=32, n_steps=64, seed=5, use_graph=False)
    assert a.update_mode == 'persistent' and b.update_mode == 'chain'
    theta0 = a.model.theta.cpu().numpy().astype(np.float64)
    np.testing.assert_array_equal(theta0, b.model.theta.cpu().numpy())
    a.train_step()
    b.train_step()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.b_act.cpu().numpy(), b.b_act.cpu().numpy())
    ta = a.model.theta.cpu().numpy().astype(np.float64)
    tb = b.model.theta.cpu().numpy().astype(np.float64)
    assert np.linalg.norm(ta - tb) / np.linalg.norm(tb - theta0) < 1e-4
    assert int(a.model.optimizer.iterations.item()) == int(b.model.optimizer.iterations.item()) == 16
    assert int(a.device_status.item()) == 0


@pytest.mark.parametrize('n_envs', [16, 64])
def test_graph_replays_back_to_back_equal_eager(device, n_envs):
    """The bench's pattern: hipGraph replays of the persistent update back to back (no
    eager launch in between, 16 blocks / 64 blocks two-level) give the eager result bit
    for bit, with no hand-off timeout."""
    from test_gpu_agent import make_agent
    a = make_agent(n_envs=n_envs, n_steps=128, seed=11, use_graph=True, t_rec=512)
    for _ in range(6):
        a.train_step()
    torch.cuda.synchronize()
    b = make_agent(n_envs=n_envs, n_steps=128, seed=11, use_graph=False, t_rec=512)
    for _ in range(6):
        b.train_step()
    torch.cuda.synchronize()
    assert a._graph is not None and a.update_mode == 'persistent'
    assert int(a.device_status.item()) == 0 and int(b.device_status.item()) == 0
    np.testing.assert_array_equal(a.b_act.cpu().numpy(), b.b_act.cpu().numpy())
    np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())
    np.testing.assert_array_equal(a.model.optimizer.v.cpu().numpy(),
                                  b.model.optimizer.v.cpu().numpy())


def test_bench_loop_graph_replays_equal_eager(device):
    """The bench's exact loop -- fused_train_step with events, host running ahead, the
    per-step episode-statistics copies -- for 40 steps gives the eager replica's
    parameters bit for bit. (A memset node in front of the update once let the runtime's
    copy-kernel arguments land on the control words after ~16 such steps: the launch
    then left early without a timeout.)"""
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv, record_cartpole_replay
    from xagents_amd.utils.common import create_model
    n = 16
    rec = record_cartpole_replay(n, 1024, seed=55)
    agents = []
    for g in (True, False):
        envs = ReplayVecEnv('CartPole-v1', n, device='cuda', record=rec)
        model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                             seed=55, device='cuda')
        agents.append(PPO(envs, model, n_steps=128, seed=55, quiet=True, use_graph=g))
    a, b = agents
    for _ in range(5):
        a.train_step()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(35)]
    for k in range(35):
        a.fused_train_step(events[k])
    torch.cuda.synchronize()
    for _ in range(40):
        b.train_step()
    torch.cuda.synchronize()
    assert a._graph is not None
    assert int(a.device_status.item()) == 0
    assert int(a.model.optimizer.iterations.item()) == 40 * 16
    np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())


@pytest.mark.parametrize('B,mb,placement', [(2048, 512, 0), (2048, 512, 1), (32768, 8192, 0)])
def test_every_optimizer_step_teacher_forced_vs_f64(device, B, mb, placement):
    """All E x M = 16 optimizer steps of one launch at the headline shape (16 envs x 128
    steps, minibatches of 512, XCD-local (placement 0) and spread (1)) and at C2 (32768 /
    8192), teacher-forced: step k's reduced gradient and loss sums are checked against the
    float64 restatement evaluated at the device's own theta_k (1e-5 rel), and
    theta_{k+1} against Keras Adam applied in float64 to theta_k with the device's
    gradient (moments carried in f64). This pins every step the headline runs, not only
    the first (ppo/agent.py:157-191 calling update_gradients, 96-137)."""
    E = 4
    bufs = _rollout_buffers(B, seed=B + 17)
    obs, act, logp, val, ret = bufs
    theta0 = _theta0(6)
    out = run_update(theta0, bufs, mb, E, trace=True, placement=placement)
    K = out['K']
    assert out['status'] == 0 and out['step'] == K == 16
    th_tr, g_tr = out['theta_trace'].astype(np.float64), out['grad_trace'].astype(np.float64)
    np.testing.assert_array_equal(out['theta_trace'][0], theta0)
    perms = [oracle.shuffle_perm(B, e, 12345, 0) for e in range(E)]
    n_mb = B // mb
    m64, v64 = np.zeros(theta0.size), np.zeros(theta0.size)
    worst = dict(grad=0.0, pg=0.0, vl=0.0, ent=0.0, step=0.0)
    for k in range(K):
        e, mi = divmod(k, n_mb)
        idx = perms[e][mi * mb:(mi + 1) * mb]
        adv = oracle.normalize_advantages(ret[idx], val[idx])
        tm, g = oracle.ac_loss_grad_f64(th_tr[k], obs[idx], act[idx], ret[idx], val[idx], A,
                                        'ppo', logp[idx], adv)
        worst['grad'] = max(worst['grad'], _rel(g_tr[k], g))
        ls = out['loss'][k].astype(np.float64).sum(axis=0)
        assert ls[3] == mb
        worst['pg'] = max(worst['pg'], abs(ls[0] - tm['pg_sum']) / max(abs(tm['pg_sum']), mb))
        worst['vl'] = max(worst['vl'], abs(ls[1] - tm['vl_sum']) / abs(tm['vl_sum']))
        worst['ent'] = max(worst['ent'], abs(ls[2] - tm['ent_sum']) / abs(tm['ent_sum']))
        # the optimizer step with the device's own gradient
        gc, _ = oracle.clip_by_global_norm_f64(g_tr[k], CLIP_G)
        th_next, m64, v64 = oracle.keras_adam_f64(th_tr[k], m64, v64, gc, k + 1, LR, B1, B2, EPS)
        dev_next = th_tr[k + 1] if k + 1 < K else out['theta'].astype(np.float64)
        # theta is f32: the step (~lr) is resolved only to f32's spacing at |theta|, so the
        # bound is that rounding plus 1e-5 of the step itself, element by element
        step = th_next - th_tr[k]
        bound = np.spacing(np.abs(th_next).astype(np.float32)).astype(np.float64) + \
            1e-5 * np.abs(step)
        worst['step'] = max(worst['step'], float(np.max(np.abs(dev_next - th_next) / bound)))
    print('worst relative errors over the 16 steps (step: in units of its bound):', worst)
    assert worst['grad'] < 1e-5
    assert worst['pg'] < 1e-5 and worst['vl'] < 1e-5 and worst['ent'] < 1e-5
    assert worst['step'] <= 1.0


@pytest.mark.parametrize('use_graph', [True, False])
def test_episode_statistics_stored_by_the_update_launch(device, monkeypatch, use_graph):
    """The persistent update stores the train step's episode statistics into its two
    mapped host slots (launch-number parity) instead of an xa_copy_to_host launch: over
    12 train steps -- graph replays and eager launches, a bench-style event-timed step in
    between -- the folded episode returns, game count and per-env running state equal the
    copy path's exactly, and every fold saw the launch number it expected."""
    from test_gpu_agent import make_agent
    out = []
    for fused in ('1', '0'):
        monkeypatch.setenv('XA_STATS_IN_UPDATE', fused)
        a = make_agent(n_envs=16, n_steps=128, seed=13, use_graph=use_graph, t_rec=256)
        assert a._stats_fused == (fused == '1')
        for i in range(12):
            if i == 5:
                a.timed_train_step()
                continue
            a.train_step()
        a._drain_episode_stats()
        torch.cuda.synchronize()
        assert a.games > 0
        out.append((list(a.total_rewards), a.games, list(a.dones),
                    np.asarray(a.episode_rewards).tolist()))
    assert out[0] == out[1]
