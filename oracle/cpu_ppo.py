"""TEST/BENCH INFRASTRUCTURE ONLY -- CPU port of the reference PPO train step,
timed as bench.py's `cpu_baseline` (kind "port"). TensorFlow is not installed, so
the reference tf2 path itself cannot be timed; this port
runs the SAME op sequence on the host cores:

  A2C.get_batch (xagents/a2c/agent.py:96-139): n_steps x [model forward on all env
      states, Categorical sample/log_prob/entropy, BaseAgent.step_envs Python loop
      over envs (xagents/base.py:402-425)]
  PPO.calculate_returns (xagents/ppo/agent.py:48-94): extra forward + numpy GAE loop
  concat_step_batches (xagents/base.py:549-564)
  PPO.run_ppo_epochs (xagents/ppo/agent.py:157-191): 4 epochs x 4 shuffled minibatches
      of forward + loss + autograd backward + clip_by_global_norm + Keras Adam
with torch-CPU float32 tensors standing in for TF CPU ops.
"""
import time
from collections import deque

import numpy as np
import torch


class ReplayEnv:
    """gym-like env over one recorded stream (same data the device ReplayVecEnv uses)."""

    def __init__(self, s0, obs, post, rew, done):
        self.s0, self.obs, self.post, self.rew, self.done = s0, obs, post, rew, done
        self.p = 0

    def reset(self):
        return self.post[self.p - 1] if self.p else self.s0

    def step(self, action):
        p = self.p
        self.p = (p + 1) % len(self.rew)
        return self.obs[p], float(self.rew[p]), bool(self.done[p]), {}


class CpuPPO:
    def __init__(self, record, theta, n_steps=128, gamma=0.99, lam=0.95, epochs=4,
                 mini_batches=4, clip=0.1, ent_coef=0.01, v_coef=0.5, grad_norm=0.5, lr=7e-4,
                 threads=None, seed=55):
        if threads:
            torch.set_num_threads(threads)
        self.threads = torch.get_num_threads()
        s0, obs, post, rew, done = record
        self.envs = [ReplayEnv(s0[i], obs[i], post[i], rew[i], done[i]) for i in range(len(s0))]
        self.n_envs = len(self.envs)
        self.states = [e.reset() for e in self.envs]
        self.dones = [False] * self.n_envs
        self.episode_rewards = np.zeros(self.n_envs)
        self.total_rewards = deque(maxlen=100)
        self.steps = 0
        self.n_steps, self.gamma, self.lam = n_steps, gamma, lam
        self.epochs, self.mini_batches = epochs, mini_batches
        self.clip, self.ent_coef, self.v_coef, self.grad_norm, self.lr = (clip, ent_coef, v_coef,
                                                                          grad_norm, lr)
        obs_dim = s0.shape[1]
        A = 2
        t = torch.from_numpy(np.asarray(theta, np.float32)).clone()
        shapes = [(obs_dim, 64), (64,), (64, 64), (64,), (64, A), (A,), (64, 1), (1,)]
        self.params, off = [], 0
        for s in shapes:
            n = int(np.prod(s))
            self.params.append(t[off:off + n].reshape(s).clone().requires_grad_(True))
            off += n
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.iterations = 0
        self.gen = torch.Generator().manual_seed(seed)

    def model(self, x):
        W1, b1, W2, b2, W3, b3, W4, b4 = self.params
        h = torch.tanh(torch.tanh(x @ W1 + b1) @ W2 + b2)
        return h @ W3 + b3, (h @ W4 + b4).squeeze(-1)

    def get_model_outputs(self, states, actions=None):
        logits, value = self.model(states)
        dist = torch.distributions.Categorical(logits=logits)
        if actions is None:
            actions = dist.sample()
        return actions, dist.log_prob(actions), value, dist.entropy()

    def step_envs(self, actions):
        observations = []
        for i, (env, action) in enumerate(zip(self.envs, actions)):
            state = self.states[i]
            new_state, reward, done, _ = env.step(action)
            self.states[i] = new_state
            self.dones[i] = done
            self.episode_rewards[i] += reward
            observations.append((state, action, reward, done, new_state))
            if done:
                self.total_rewards.append(self.episode_rewards[i])
                self.episode_rewards[i] = 0
                self.states[i] = env.reset()
            self.steps += 1
        return [np.array(item, np.float32) for item in zip(*observations)]

    def get_batch(self):
        states, rewards, actions, values, dones, log_probs = [], [], [], [], [], []
        step_states = np.array(self.states, np.float32)
        step_dones = np.array(self.dones, np.float32)
        with torch.no_grad():
            for _ in range(self.n_steps):
                a, lp, v, _ = self.get_model_outputs(torch.from_numpy(step_states))
                states.append(step_states)
                actions.append(a.numpy())
                values.append(v.numpy())
                log_probs.append(lp.numpy())
                dones.append(step_dones)
                *_, r, step_dones, step_states = self.step_envs(a.numpy())
                rewards.append(r)
        dones.append(step_dones)
        return [np.asarray(x, np.float32) for x in (states, rewards, actions, values, dones,
                                                     log_probs)]

    def calculate_returns(self, rewards, dones, values):
        with torch.no_grad():
            next_values = self.model(torch.from_numpy(np.array(self.states, np.float32)))[1].numpy()
        values = np.concatenate([values, next_values[None]])
        dones = np.concatenate([dones, dones[-1][None]])
        returns, last_lam = [], 0
        for step in reversed(range(self.n_steps)):
            nnt = 1 - dones[step + 1]
            delta = rewards[step] + self.gamma * values[step + 1] * nnt - values[step]
            last_lam = delta + self.gamma * self.lam * nnt * last_lam
            returns.append(last_lam)
        return np.asarray(returns[::-1]) + values[:-1]

    @staticmethod
    def concat_step_batches(*args):
        return [a.swapaxes(0, 1).reshape(-1, *a.shape[2:]) for a in args]

    def update_gradients(self, states, actions, old_values, returns, old_log_probs, advantages):
        _, log_probs, values, entropy = self.get_model_outputs(states, actions)
        entropy = entropy.mean()
        clipped = old_values + torch.clamp(values - old_values, -self.clip, self.clip)
        value_loss = 0.5 * torch.maximum((values - returns) ** 2, (clipped - returns) ** 2).mean()
        ratio = torch.exp(log_probs - old_log_probs)
        pg_loss = torch.maximum(-advantages * ratio,
                                -advantages * torch.clamp(ratio, 1 - self.clip, 1 + self.clip)).mean()
        loss = pg_loss - entropy * self.ent_coef + value_loss * self.v_coef
        grads = torch.autograd.grad(loss, self.params)
        gn = torch.sqrt(sum((g * g).sum() for g in grads))
        scale = self.grad_norm * torch.minimum(1.0 / gn, torch.tensor(1.0 / self.grad_norm))
        self.iterations += 1
        t = self.iterations
        alpha = self.lr * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        with torch.no_grad():
            for p, g, m, v in zip(self.params, grads, self.m, self.v):
                g = g * scale
                m += (g - m) * (1 - 0.9)
                v += (g * g - v) * (1 - 0.999)
                p -= m * alpha / (torch.sqrt(v) + 1e-7)

    def train_step(self):
        states, rewards, actions, values, dones, log_probs = self.get_batch()
        returns = self.calculate_returns(rewards, dones, values)
        batch = [torch.from_numpy(np.ascontiguousarray(x)) for x in self.concat_step_batches(
            states, actions, returns.astype(np.float32), values, log_probs)]
        states, actions, returns, old_values, old_log_probs = batch
        actions = actions.long()
        B = states.shape[0]
        mb = B // self.mini_batches
        indices = torch.arange(B)
        for _ in range(self.epochs):
            indices = indices[torch.randperm(B, generator=self.gen)]
            for i in range(0, B, mb):
                idx = indices[i:i + mb]
                adv = returns[idx] - old_values[idx]
                adv = (adv - adv.mean()) / (adv.std(unbiased=False) + 1e-8)
                self.update_gradients(states[idx], actions[idx], old_values[idx], returns[idx],
                                      old_log_probs[idx], adv)


def time_cpu_baseline(record, theta, n_steps=128, seconds=15.0, threads=None, min_steps=2):
    """Run CpuPPO train steps until `seconds` elapse; returns (env_steps_per_s, info)."""
    agent = CpuPPO(record, theta, n_steps=n_steps, threads=threads)
    agent.train_step()  # warm-up (allocator, autograd graph)
    steps0 = agent.steps
    t0 = time.perf_counter()
    k = 0
    while k < min_steps or time.perf_counter() - t0 < seconds:
        agent.train_step()
        k += 1
    dt = time.perf_counter() - t0
    env_steps = agent.steps - steps0
    return env_steps / dt, dict(train_steps=k, env_steps=env_steps, seconds=dt,
                                threads=agent.threads, n_envs=agent.n_envs)
