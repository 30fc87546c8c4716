"""TEST/BENCH INFRASTRUCTURE ONLY -- CPU port of the reference's TD3 train step, timed as
bench.py's `cpu_baseline` (kind "port") for config C5; TensorFlow is absent, so torch-CPU
float32 ops stand in for the TF CPU kernels, in the reference's op order:

TD3 (xagents/td3/agent.py:8-110 over DDPG, xagents/ddpg/agent.py:129-166): actor forward
on the N states (no exploration noise, td3/agent.py:57-64), a per-env Python step_envs loop
appending to one ReplayBuffer2 per env (numpy rings, buffers.py:101-148), then for every env
that finished an episode `gradient_steps` gradient steps, each: np.random.randint samples per
buffer, concat_buffer_samples, target actor + clipped N(0, 0.2) smoothing, twin target
critics, two critic MSE (sum over the batch) updates with Keras Adam; every policy_delay-th
step the actor update through critic1 and the Polyak sync of the three target networks.
MLPs per xagents/td3/models: actor 24 -> 400 -> 300 -> 4 (relu, relu, tanh), critics
28 -> 400 -> 300 -> 1 (relu, relu).
"""
import time

import numpy as np
import torch

from cpu_ppo import ReplayEnv


def _mlp(sizes, gen):
    ps = []
    for a, b in zip(sizes[:-1], sizes[1:]):
        ps += [(torch.randn(a, b, generator=gen) * (1.0 / np.sqrt(a))).requires_grad_(True),
               torch.zeros(b, requires_grad=True)]
    return ps


def _fwd(ps, x, out_act=None):
    n = len(ps) // 2
    for i in range(n):
        x = x @ ps[2 * i] + ps[2 * i + 1]
        if i < n - 1:
            x = torch.relu(x)
    return torch.tanh(x) if out_act == 'tanh' else x


class _Adam:
    def __init__(self, ps, lr):
        self.ps, self.lr, self.t = ps, lr, 0
        self.m = [torch.zeros_like(p) for p in ps]
        self.v = [torch.zeros_like(p) for p in ps]

    def step(self, grads):
        self.t += 1
        alpha = self.lr * np.sqrt(1 - 0.999 ** self.t) / (1 - 0.9 ** self.t)
        with torch.no_grad():
            for p, g, m, v in zip(self.ps, grads, self.m, self.v):
                m += (g - m) * (1 - 0.9)
                v += (g * g - v) * (1 - 0.999)
                p -= m * alpha / (torch.sqrt(v) + 1e-7)


class CpuTD3:
    def __init__(self, record, buffer_size=1000, batch_per_env=1, gradient_steps=1,
                 gamma=0.99, tau=0.005, policy_delay=2, lr=1e-3, threads=None, seed=55):
        if threads:
            torch.set_num_threads(threads)
        self.threads = torch.get_num_threads()
        s0, obs, post, rew, done = record
        self.envs = [ReplayEnv(s0[i], obs[i], post[i], rew[i], done[i]) for i in range(len(s0))]
        self.n_envs = len(self.envs)
        self.states = [e.reset() for e in self.envs]
        self.obs_dim, self.act_dim = s0.shape[1], 4
        gen = torch.Generator().manual_seed(seed)
        self.actor = _mlp([self.obs_dim, 400, 300, 4], gen)
        self.critic1 = _mlp([self.obs_dim + 4, 400, 300, 1], gen)
        self.critic2 = _mlp([self.obs_dim + 4, 400, 300, 1], gen)
        self.targets = [[p.detach().clone() for p in m]
                        for m in (self.actor, self.critic1, self.critic2)]
        self.opts = [_Adam(m, lr) for m in (self.actor, self.critic1, self.critic2)]
        self.size, self.k = buffer_size, batch_per_env
        n, s = self.n_envs, buffer_size
        self.rb = [np.zeros((n, s, self.obs_dim), np.float32), np.zeros((n, s, 4), np.float32),
                   np.zeros((n, s, 1), np.float32), np.zeros((n, s, 1), np.float32),
                   np.zeros((n, s, self.obs_dim), np.float32)]
        self.cur = np.zeros(n, np.int64)
        self.gradient_steps, self.gamma, self.tau = gradient_steps, gamma, tau
        self.policy_delay = policy_delay
        self.steps = 0

    def step_envs(self, actions):
        dones = np.zeros(self.n_envs, bool)
        for i, env in enumerate(self.envs):
            state = self.states[i]
            ns, r, d, _ = env.step(actions[i])
            row = self.cur[i] % self.size  # ReplayBuffer2 row rule (saturating size)
            for slot, val in zip(self.rb, (state, actions[i], r, d, ns)):
                slot[i, row] = val
            self.cur[i] = min(self.cur[i] + 1, self.size)
            self.states[i] = env.reset() if d else ns
            dones[i] = d
            self.steps += 1
        return dones

    def fill(self, n):
        for _ in range(n):
            self.step_envs(np.random.uniform(-1, 1, (self.n_envs, 4)).astype(np.float32))

    def sample(self):
        idx = [np.random.randint(0, min(self.cur[i], self.size), self.k)
               for i in range(self.n_envs)]
        return [torch.from_numpy(np.concatenate([f[i, ix] for i, ix in enumerate(idx)]))
                for f in self.rb]

    def gradient_step(self, g):
        s, a, r, d, s2 = self.sample()
        with torch.no_grad():
            noise = torch.clamp(torch.randn(s.shape[0], 4) * 0.2, -0.5, 0.5)
            a2 = torch.clamp(_fwd(self.targets[0], s2, 'tanh') + noise, -1, 1)
            sa2 = torch.cat([s2, a2], 1)
            y = r + (1 - d) * self.gamma * torch.minimum(_fwd(self.targets[1], sa2),
                                                         _fwd(self.targets[2], sa2))
        sa = torch.cat([s, a], 1)
        for critic, opt in ((self.critic1, self.opts[1]), (self.critic2, self.opts[2])):
            loss = ((_fwd(critic, sa) - y) ** 2).mean(1).sum()
            opt.step(torch.autograd.grad(loss, critic))
        if g % self.policy_delay == 0:
            loss = -_fwd(self.critic1, torch.cat([s, _fwd(self.actor, s, 'tanh')], 1)).mean()
            self.opts[0].step(torch.autograd.grad(loss, self.actor, allow_unused=True))
            with torch.no_grad():
                for tgt, src in zip(self.targets, (self.actor, self.critic1, self.critic2)):
                    for t, p in zip(tgt, src):
                        t.mul_(1 - self.tau).add_(p * self.tau)

    def train_step(self):
        with torch.no_grad():
            actions = _fwd(self.actor, torch.from_numpy(np.array(self.states)), 'tanh').numpy()
        dones = self.step_envs(actions)
        for _ in np.nonzero(dones)[0]:
            for g in range(self.gradient_steps):
                self.gradient_step(g)


def time_td3(record, seconds=15.0, threads=None, min_steps=2):
    agent = CpuTD3(record, threads=threads)
    agent.fill(64)
    agent.train_step()
    steps0 = agent.steps
    t0 = time.perf_counter()
    k = 0
    while k < min_steps or time.perf_counter() - t0 < seconds:
        agent.train_step()
        k += 1
    dt = time.perf_counter() - t0
    return (agent.steps - steps0) / dt, dict(train_steps=k, seconds=dt, threads=agent.threads,
                                             n_envs=agent.n_envs)
