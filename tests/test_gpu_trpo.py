"""GPU parity of TRPO (xagents/trpo/agent.py) against the float64 restatement
(oracle/trpo_f64.py): Fisher-vector product, surrogate gradient, one full train step
(CG step direction, shs, line search, critic Adam steps). Tolerances: f32 device math vs
f64, relative to each quantity's scale (1e-4 for single products, 2e-3 after the
10-iteration CG and 48 Adam steps, which compound rounding)."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _rel(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-12)


def _agent(device, n_envs=4, n_steps=40, seed=7, **kw):
    from xagents_amd import TRPO
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_model
    envs = create_envs('CartPole-v1', n_envs, mode='transitions', device=device, seed=seed,
                       t_rec=256)
    actor = create_model(envs, 'trpo', 'actor_model', seed=seed, device=device)
    critic = create_model(envs, 'trpo', 'critic_model', seed=seed + 1, device=device)
    return TRPO(envs, actor, critic, n_steps=n_steps, seed=seed, quiet=True, **kw)


def test_fvp_and_surrogate_gradient_vs_f64(device):
    sys.path.insert(0, str(ROOT / 'oracle'))
    import trpo_f64 as TR
    import nets_f64 as O
    agent = _agent(device)
    agent.get_batch()
    B = agent.batch_size
    from xagents_amd._lib import call, stream
    call('xa_normalized_advantages', agent.b_ret.data_ptr(), agent.b_val.data_ptr(), B, 0.0,
         agent.adv.data_ptr(), stream())
    lg = agent.ex_actor.forward(agent.batch_states)[0]
    agent.old_logits.copy_(lg)
    agent._head(agent.old_logits, dlogits=agent.dlogits, out=agent.head_out)
    agent.ex_actor.backward([agent.dlogits], agent.flat_grads)
    agent._prepare_fvp()
    rng = np.random.default_rng(1)
    v = rng.normal(size=agent.actor.n_params).astype(np.float32)
    got = agent.calculate_fvp(torch.from_numpy(v).to(device)).cpu().numpy()
    torch.cuda.synchronize()
    theta = agent.actor.theta.cpu().numpy().astype(np.float64)
    x = agent.batch_states.cpu().numpy().astype(np.float64)
    layers = agent.actor.layers
    ref = TR.fvp(layers, theta, x[::agent.fvp_n_steps], v.astype(np.float64), agent.cg_damping)
    assert _rel(got, ref) < 1e-4
    # surrogate gradient and loss at ratio = 1
    acts = agent.b_act.reshape(-1).cpu().numpy()
    ret, val = agent.b_ret.reshape(-1).cpu().numpy(), agent.b_val.reshape(-1).cpu().numpy()
    adv = ret.astype(np.float64) - val
    adv = (adv - adv.mean()) / adv.std()
    np.testing.assert_allclose(agent.adv.cpu().numpy(), adv, rtol=1e-4, atol=1e-5)
    _, outs = O.forward(layers, theta, x, x.shape[1:])
    dl = TR.surrogate_grad_logits(outs[-1], acts, adv, agent.entropy_coef)
    g = O.backward(layers, theta, x, outs, {len(layers) - 1: dl})
    assert _rel(agent.flat_grads.cpu().numpy(), g) < 1e-4
    loss0 = TR.surrogate(outs[-1], outs[-1], acts, adv, agent.entropy_coef)[0]
    assert abs(agent.head_out[0].item() - loss0) < 1e-5 * max(1.0, abs(loss0))


def test_trpo_train_step_vs_f64(device):
    sys.path.insert(0, str(ROOT / 'oracle'))
    import trpo_f64 as TR
    agent = _agent(device, n_envs=8, n_steps=32, seed=11)
    a0 = agent.actor.theta.cpu().numpy().copy()
    c0 = agent.critic.theta.cpu().numpy().copy()
    np.random.seed(123)
    agent.train_step()
    torch.cuda.synchronize()
    B = agent.batch_size
    np.random.seed(123)
    perms = [np.random.permutation(B) for _ in range(agent.critic_iterations * agent.ppo_epochs)]
    states = agent.batch_states.cpu().numpy()
    acts = agent.b_act.reshape(-1).cpu().numpy()
    ret, val = agent.b_ret.reshape(-1).cpu().numpy(), agent.b_val.reshape(-1).cpu().numpy()
    new_a, new_c, d = TR.trpo_update(
        agent.actor.layers, a0, agent.critic.layers, c0, states, acts, ret, val, perms,
        entropy_coef=agent.entropy_coef, max_kl=agent.max_kl, cg_iterations=agent.cg_iterations,
        cg_residual_tolerance=agent.cg_residual_tolerance, cg_damping=agent.cg_damping,
        actor_iterations=agent.actor_iterations, critic_iterations=agent.critic_iterations,
        fvp_n_steps=agent.fvp_n_steps, mini_batch_size=agent.mini_batch_size,
        lr=agent.critic.optimizer.learning_rate)
    assert abs(agent.last_losses['shs'] - d['shs']) < 2e-3 * abs(d['shs'])
    got_a = agent.actor.theta.cpu().numpy()
    assert _rel(got_a - a0, new_a - a0) < 2e-3, 'actor step'
    got_c = agent.critic.theta.cpu().numpy()
    assert _rel(got_c - c0, new_c - c0) < 2e-3, 'critic Adam steps'
    assert int(agent.critic.optimizer.iterations.cpu()[0]) == len(perms) * agent.mini_batches


def test_trpo_rollout_graph_matches_eager(device):
    """The captured rollout replays exactly what the eager launches compute."""
    outs = []
    for use_graph in (False, True):
        agent = _agent(device, n_envs=4, n_steps=16, seed=5, use_graph=use_graph)
        got = []
        for _ in range(3):
            agent.get_batch()
            got.append([t.cpu().numpy().copy() for t in (agent.batch_states, agent.b_act,
                                                         agent.b_logp, agent.b_ret)])
        outs.append(got)
    for a, b in zip(*outs):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_trpo_fit_runs(device):
    agent = _agent(device, n_envs=4, n_steps=64, seed=3)
    agent.fit(max_steps=4 * 64 * 3)
    assert agent.steps >= 4 * 64 * 3
    assert np.isfinite(agent.actor.theta.cpu().numpy()).all()
    assert np.isfinite(agent.critic.theta.cpu().numpy()).all()
