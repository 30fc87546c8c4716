"""TEST/BENCH INFRASTRUCTURE ONLY -- CPU ports of the reference's CNN train steps, timed as
bench.py's `cpu_baseline` (kind "port") for the secondary configs; TensorFlow is absent, so
torch-CPU float32 ops stand in for the TF CPU kernels, in the reference's op order:

* CpuCnnPPO (config C4): CpuPPO (oracle/cpu_ppo.py) with the NatureCNN Conv1D actor-critic
  of xagents/ppo/models/cnn-actor-critic.cfg. Keras Conv1D on (B, 84, 84, 1) convolves along
  W with H folded into the batch: conv1d on [B 84, C, W], channels-last
  flatten (common.py:231-260); frames scaled uint8 / 255 (base.py:505-506).
* CpuACER (bench --config acer): see the class docstring.
* CpuDQN (config C3): DQN.train_step (xagents/dqn/agent.py:178-209): epsilon-greedy acting
  on the CNN, per-env Python step_envs loop, ReplayBuffer1 deques + random.sample,
  concat_buffer_samples, double-DQN targets, MSE summed over the batch, Keras Adam.
"""
import random
import time
from collections import deque

import numpy as np
import torch
import torch.nn.functional as F

from cpu_ppo import CpuPPO, ReplayEnv

_CONVS = [(32, 8, 4), (64, 4, 2), (64, 3, 1)]  # filters, kernel, stride


def cnn_params(n_out, gen):
    """Random NatureCNN parameters in Keras layout ((k, C, F) kernels, (in, out) dense)."""
    shapes, c = [], 1
    for f, k, _ in _CONVS:
        shapes += [(k, c, f), (f,)]
        c = f
    shapes += [(37632, 512), (512,)]
    for n in n_out:
        shapes += [(512, n), (n,)]
    return [(torch.randn(s, generator=gen) * (0.05 if len(s) > 1 else 0.0)).requires_grad_(True)
            for s in shapes]


def cnn_forward(params, frames):
    """frames [B, 84, 84, 1] uint8 -> trunk [B, 512] and the heads."""
    B = frames.shape[0]
    x = torch.as_tensor(frames).float() / 255.0
    x = x.reshape(B * 84, 84, 1).permute(0, 2, 1)  # [rows, C, W]
    i = 0
    for f, k, s in _CONVS:
        w, b = params[i], params[i + 1]
        x = F.relu(F.conv1d(x, w.permute(2, 1, 0), b, stride=s))
        i += 2
    x = x.permute(0, 2, 1).reshape(B, -1)  # Keras flatten of (84, 7, 64)
    h = F.relu(x @ params[i] + params[i + 1])
    i += 2
    heads = []
    while i < len(params):
        heads.append(h @ params[i] + params[i + 1])
        i += 2
    return heads


class CpuCnnPPO(CpuPPO):
    def __init__(self, record, n_steps=128, threads=None, seed=55, gamma=0.99, lam=0.95,
                 epochs=4, mini_batches=4, clip=0.1, ent_coef=0.01, v_coef=0.5, grad_norm=0.5,
                 lr=7e-4):
        # CpuPPO.__init__ minus its MLP parameter layout
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
        self.iterations = 0
        self.gen = torch.Generator().manual_seed(seed)
        self.params = cnn_params([4, 1], self.gen)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]

    def model(self, x):
        logits, value = cnn_forward(self.params, x)
        return logits, value.squeeze(-1)

    def get_batch(self):
        states, rewards, actions, values, dones, log_probs = [], [], [], [], [], []
        step_states = np.array(self.states)
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
                step_states = step_states.astype(np.uint8)
                rewards.append(r)
        dones.append(step_dones)
        out = [np.asarray(x, np.float32) for x in (rewards, actions, values, dones, log_probs)]
        return [np.asarray(states, np.uint8)] + out

    def calculate_returns(self, rewards, dones, values):
        with torch.no_grad():
            next_values = self.model(torch.from_numpy(np.array(self.states)))[1].numpy()
        values = np.concatenate([values, next_values[None]])
        dones = np.concatenate([dones, dones[-1][None]])
        returns, last_lam = [], 0
        for step in reversed(range(self.n_steps)):
            nnt = 1 - dones[step + 1]
            delta = rewards[step] + self.gamma * values[step + 1] * nnt - values[step]
            last_lam = delta + self.gamma * self.lam * nnt * last_lam
            returns.append(last_lam)
        return np.asarray(returns[::-1]) + values[:-1]


def time_cnn_ppo(record, n_steps=128, seconds=15.0, threads=None, min_steps=1):
    """CpuCnnPPO train steps (after one warm-up) until `seconds` elapse."""
    agent = CpuCnnPPO(record, n_steps=n_steps, threads=threads)
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


class CpuDQN:
    """DQN.train_step on the host (double DQN, ReplayBuffer1 deques)."""

    def __init__(self, record, buffer_size=1000, batch_per_env=2, gamma=0.99, epsilon=0.02,
                 lr=1e-4, threads=None, seed=55):
        if threads:
            torch.set_num_threads(threads)
        self.threads = torch.get_num_threads()
        s0, obs, post, rew, done = record
        self.envs = [ReplayEnv(s0[i], obs[i], post[i], rew[i], done[i]) for i in range(len(s0))]
        self.n_envs = len(self.envs)
        self.states = [e.reset() for e in self.envs]
        self.buffers = [deque(maxlen=buffer_size) for _ in self.envs]
        self.k, self.gamma, self.epsilon, self.lr = batch_per_env, gamma, epsilon, lr
        gen = torch.Generator().manual_seed(seed)
        self.params = cnn_params([6], gen)
        self.target = [p.detach().clone() for p in self.params]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0
        self.steps = 0

    def q(self, params, frames):
        return cnn_forward(params, frames)[0]

    def step_envs(self, actions):
        for i, (env, a) in enumerate(zip(self.envs, actions)):
            state = self.states[i]
            new_state, reward, done, _ = env.step(a)
            self.buffers[i].append((state, int(a), reward, done, new_state))
            self.states[i] = env.reset() if done else new_state
            self.steps += 1

    def fill(self, n):
        for _ in range(n):
            self.step_envs(np.random.randint(0, 6, self.n_envs))

    def train_step(self):
        # get_actions: one draw decides random-for-all vs greedy-for-all
        if np.random.random() < self.epsilon:
            actions = np.random.randint(0, 6, self.n_envs)
        else:
            with torch.no_grad():
                actions = self.q(self.params, np.array(self.states)).argmax(1).numpy()
        self.step_envs(actions)
        # concat_buffer_samples: random.sample per env, fields concatenated in env order
        samples = [random.sample(b, self.k) for b in self.buffers]
        flat = [t for s in samples for t in s]
        s, a, r, d, ns = (np.array(x) for x in zip(*flat))
        a = torch.from_numpy(a.astype(np.int64))
        r = torch.from_numpy(r.astype(np.float32))
        d = torch.from_numpy(d.astype(np.float32))
        with torch.no_grad():
            q_next_online = self.q(self.params, ns)
            q_next_target = self.q(self.target, ns)
            nv = q_next_target.gather(1, q_next_online.argmax(1, keepdim=True)).squeeze(1)
            y_sel = r + self.gamma * nv * (1 - d)
        q = self.q(self.params, s)
        y = q.detach().clone()
        y[torch.arange(len(a)), a] = y_sel
        loss = ((y - q) ** 2).mean(1).sum()  # Keras MSE per row, minimize sums the batch
        grads = torch.autograd.grad(loss, self.params)
        self.t += 1
        alpha = self.lr * np.sqrt(1 - 0.999 ** self.t) / (1 - 0.9 ** self.t)
        with torch.no_grad():
            for p, g, m, v in zip(self.params, grads, self.m, self.v):
                m += (g - m) * (1 - 0.9)
                v += (g * g - v) * (1 - 0.999)
                p -= m * alpha / (torch.sqrt(v) + 1e-7)


def time_dqn(record, seconds=15.0, threads=None, min_steps=2):
    agent = CpuDQN(record, threads=threads)
    agent.fill(8)
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


class CpuACER:
    """ACER.train_step on the host (xagents/acer/agent.py:363-387): A2C.get_batch rollout
    with the softmax actor, per-env Python step_envs loop, one trajectory per env per step
    into ReplayBuffer1 deques, update_gradients on the fresh batch then poisson(replay_ratio)
    updates on random.sample'd trajectories; Retrace returns as a reversed Python loop,
    trust-region gradient through autograd, global-norm clip, Keras Adam, weight EMA."""

    def __init__(self, record, n_steps=20, buffer_size=64, replay_ratio=4, gamma=0.99,
                 lr=7e-4, threads=None, seed=55, n_actions=6):
        if threads:
            torch.set_num_threads(threads)
        self.threads = torch.get_num_threads()
        s0, obs, post, rew, done = record
        self.envs = [ReplayEnv(s0[i], obs[i], post[i], rew[i], done[i]) for i in range(len(s0))]
        self.n_envs, self.T, self.A = len(self.envs), n_steps, n_actions
        self.states = [e.reset() for e in self.envs]
        self.buffers = [deque(maxlen=buffer_size) for _ in self.envs]
        self.replay_ratio, self.gamma, self.lr = replay_ratio, gamma, lr
        self.eps, self.c, self.delta, self.ent, self.vcoef = 1e-6, 10.0, 1.0, 0.01, 0.5
        gen = torch.Generator().manual_seed(seed)
        self.params = cnn_params([n_actions, n_actions], gen)
        self.avg = [p.detach().clone() for p in self.params]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0
        self.steps = 0

    def get_batch(self):
        N, T = self.n_envs, self.T
        states, rewards, actions, dones, probs = [], [], [], [], []
        for _ in range(T):
            x = np.array(self.states)
            with torch.no_grad():
                p = torch.softmax(cnn_forward(self.params, x)[0], -1)
            a = torch.multinomial(p, 1).squeeze(1).numpy()
            states.append(x)
            probs.append(p.numpy())
            actions.append(a)
            r, d = np.zeros(N, np.float32), np.zeros(N, np.float32)
            for i, env in enumerate(self.envs):
                ns, r[i], d[i], _ = env.step(a[i])
                self.states[i] = env.reset() if d[i] else ns
                self.steps += 1
            rewards.append(r)
            dones.append(d)
        states.append(np.array(self.states))
        batch = [np.asarray(b).swapaxes(0, 1) for b in (states, rewards, actions, dones, probs)]
        for i in range(N):
            self.buffers[i].append(tuple(b[i] for b in batch))
        return batch

    def update(self, batch):
        states, rewards, actions, dones, mu = batch
        N, T, A = self.n_envs, self.T, self.A
        x = states.reshape(N * (T + 1), *states.shape[2:])
        logits, q = cnn_forward(self.params, x)
        p = torch.softmax(logits, -1)
        with torch.no_grad():
            avg_p = torch.softmax(cnn_forward(self.avg, x)[0], -1)
        values = (p * q).sum(-1).reshape(N, T + 1)
        pc = p.reshape(N, T + 1, A)[:, :T]
        qc = q.reshape(N, T + 1, A)[:, :T]
        avg_c = avg_p.reshape(N, T + 1, A)[:, :T]
        a = torch.from_numpy(np.asarray(actions, np.int64))[..., None]
        sel_p = pc.gather(2, a).squeeze(2)
        sel_q = qc.gather(2, a).squeeze(2)
        rho = (sel_p / (torch.from_numpy(np.asarray(mu, np.float32)).gather(2, a).squeeze(2)
                        + self.eps)).detach()
        r, d = torch.from_numpy(rewards), torch.from_numpy(dones)
        ret, cur, rets = None, values[:, T].detach(), []
        for i in reversed(range(T)):
            cur = r[:, i] + self.gamma * cur * (1 - d[:, i])
            rets.append(cur)
            cur = torch.clamp(rho[:, i], max=1.0) * (cur - sel_q[:, i].detach()) \
                + values[:, i].detach()
        ret = torch.stack(rets[::-1], 1)
        adv = (ret - values[:, :T]).detach()
        ent = (-(pc * torch.log(pc + self.eps)).sum(-1)).mean()
        gain = torch.log(sel_p + self.eps) * (adv * torch.clamp(rho, max=self.c))
        loss = (gain.mean() + self.ent * ent) * N * T
        vloss = (0.5 * (ret - sel_q) ** 2).mean() * self.vcoef
        g = torch.autograd.grad(loss, pc, retain_graph=True)[0]
        k = -avg_c / (pc.detach() + self.eps)
        adj = torch.clamp(((k * g).sum(-1) - self.delta) / ((k * k).sum(-1) + self.eps), min=0)
        g = -(g - adj[..., None] * k) / (N * T)
        ga = torch.autograd.grad(pc, self.params, g, retain_graph=True, allow_unused=True)
        gv = torch.autograd.grad(vloss, self.params, allow_unused=True)
        grads = [x if y is None else (y if x is None else x + y) for x, y in zip(ga, gv)]
        norm = torch.sqrt(sum((gi * gi).sum() for gi in grads))
        scale = 10.0 / max(float(norm), 10.0)
        self.t += 1
        alpha = self.lr * np.sqrt(1 - 0.999 ** self.t) / (1 - 0.9 ** self.t)
        with torch.no_grad():
            for prm, gi, m, v, av in zip(self.params, grads, self.m, self.v, self.avg):
                gi = gi * scale
                m += (gi - m) * (1 - 0.9)
                v += (gi * gi - v) * (1 - 0.999)
                prm -= m * alpha / (torch.sqrt(v) + 1e-7)
                av -= (av - prm) * (1 - 0.99)

    def train_step(self):
        self.update(self.get_batch())
        for _ in range(np.random.poisson(self.replay_ratio)):
            samples = [random.sample(b, 1)[0] for b in self.buffers]
            self.update([np.stack(f) for f in zip(*samples)])


def time_acer(record, seconds=15.0, threads=None, min_steps=1, n_steps=20):
    agent = CpuACER(record, n_steps=n_steps, threads=threads)
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
