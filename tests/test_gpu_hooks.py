"""The drop-in surface: a subclass that overrides a reference hook trains through the
composed path (the override is honoured), and gives the fused path's result when the
override restates the reference (xagents/ppo/agent.py:139-191, a2c/agent.py:141-218)."""
import numpy as np
import oracle
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env_model(kind, n, seed):
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', n, t_rec=256, seed=seed, device='cuda')
    model = create_model(envs, kind, 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=seed, device='cuda')
    return envs, model


def test_ppo_get_mini_batches_override_equals_fused(device):
    """A PPO subclass whose get_mini_batches slices fixed permutations trains through
    run_ppo_epochs / update_gradients and matches the fused update given the same
    permutations (PPO.set_minibatch_permutation) and rollout uniforms."""
    from xagents_amd import PPO
    n, T, E = 8, 32, 4
    B = n * T
    rng = np.random.default_rng(5)
    perms = np.stack([rng.permutation(B) for _ in range(E)]).astype(np.int32)
    u = torch.from_numpy(rng.random((n, T)).astype(np.float32)).cuda()

    class FixedPermPPO(PPO):
        calls = 0

        def get_mini_batches(self, *args):
            FixedPermPPO.calls += 1
            out = []
            for e in range(self.ppo_epochs):
                idx = torch.as_tensor(perms[e], device=self.device).long()
                for i in range(0, self.batch_size, self.mini_batch_size):
                    bi = idx[i:i + self.mini_batch_size]
                    out.append([item[bi] for item in args])
            return out

    agents = []
    for cls in (FixedPermPPO, PPO):
        envs, model = _env_model('ppo', n, 3)
        ag = cls(envs, model, n_steps=T, seed=3, quiet=True, use_graph=False)
        ag.set_rollout_uniforms(u)
        agents.append(ag)
    composed, fused = agents
    fused.set_minibatch_permutation(torch.from_numpy(perms).cuda())
    theta0 = fused.model.theta.cpu().numpy().astype(np.float64)
    for ag in agents:
        ag.train_step()
    torch.cuda.synchronize()
    assert FixedPermPPO.calls == 1
    np.testing.assert_array_equal(composed.b_act.cpu().numpy(), fused.b_act.cpu().numpy())
    tc = composed.model.theta.cpu().numpy().astype(np.float64)
    tf = fused.model.theta.cpu().numpy().astype(np.float64)
    rel = np.linalg.norm(tc - tf) / np.linalg.norm(tf - theta0)
    assert rel < 1e-4, f'composed vs fused update: {rel:.2e}'
    assert int(composed.model.optimizer.iterations.item()) == E * 4


def test_a2c_calculate_returns_override(device):
    """An A2C subclass with the reference's numpy calculate_returns
    (a2c/agent.py:141-171) trains through np_train_step + update_gradients; its returns
    are the n-step restatement's bit for bit and the step equals the fused one."""
    from xagents_amd import A2C
    n, T = 8, 5
    rng = np.random.default_rng(6)
    u = torch.from_numpy(rng.random((n, T)).astype(np.float32)).cuda()
    seen = {}

    class HostReturnsA2C(A2C):
        def calculate_returns(self, rewards, dones, values=None, selected_critic_logits=None,
                              selected_importance=None):
            next_values = self.get_model_outputs(
                self.get_states(), self.output_models)[2].cpu().numpy()
            rewards, dones = rewards.cpu().numpy(), dones.cpu().numpy()
            returns = [next_values]
            for step in reversed(range(self.n_steps)):
                returns.append(rewards[step] + self.gamma * returns[-1] * (1.0 - dones[step + 1]))
            out = np.asarray(returns[::-1], np.float32)[:-1]
            seen.update(returns=out, rewards=rewards, dones=dones, next_values=next_values)
            return out

    agents = []
    for cls in (HostReturnsA2C, A2C):
        envs, model = _env_model('a2c', n, 4)
        ag = cls(envs, model, n_steps=T, seed=4, quiet=True, use_graph=False)
        ag.set_rollout_uniforms(u)
        agents.append(ag)
    composed, fused = agents
    for ag in agents:
        ag.train_step()
    torch.cuda.synchronize()
    # [T, N] time-major returns vs the restatement of the reference loop
    ref = oracle.nstep(seen['rewards'].T.copy(), seen['dones'].T.copy(), seen['next_values'],
                       0.99)
    np.testing.assert_array_equal(seen['returns'], ref.T)
    np.testing.assert_array_equal(seen['returns'], fused.b_ret.cpu().numpy().T)
    np.testing.assert_array_equal(composed.model.theta.cpu().numpy(),
                                  fused.model.theta.cpu().numpy())
    assert composed.steps == fused.steps == n * T
