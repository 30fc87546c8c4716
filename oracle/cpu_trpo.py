"""TEST/BENCH INFRASTRUCTURE ONLY -- CPU port of the reference's TRPO train step, timed as
bench.py's `cpu_baseline` (kind "port") for `--config trpo`; TensorFlow is absent, so
torch-CPU float32 ops stand in for the TF CPU kernels, in the reference's op order
(xagents/trpo/agent.py:301-348):

rollout of n_steps x [actor forward + Categorical sample, critic forward, per-env Python
step_envs loop] (A2C.get_batch, a2c/agent.py:96-139), V(get_states()) and the numpy GAE loop
(ppo/agent.py:48-94), env-major batch, advantages normalised over the batch (321-324);
surrogate loss mean(ratio adv) + entropy_coef mean(H) and its gradient (200-223); conjugate
gradients (150-177) with the Fisher-vector product as the Hessian-vector product of the mean
KL on states[::fvp_n_steps] by double backprop (121-148); shs, the Lagrange multiplier and
the backtracking line search (235-278, 329-345); critic_iterations x ppo_epochs x
mini_batches MSE minibatch updates with Keras Adam (280-299).
Actor / critic: the trpo .cfg MLPs [64, 64] relu (xagents/trpo/models).
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


def _fwd(ps, x):
    n = len(ps) // 2
    for i in range(n):
        x = x @ ps[2 * i] + ps[2 * i + 1]
        if i < n - 1:
            x = torch.relu(x)
    return x


class CpuTRPO:
    def __init__(self, record, n_steps=512, n_actions=2, gamma=0.99, lam=0.95, max_kl=1e-3,
                 cg_iterations=10, cg_damping=1e-3, actor_iterations=10, critic_iterations=3,
                 fvp_n_steps=5, epochs=4, mini_batches=4, entropy_coef=0.01, lr=1e-3,
                 threads=None, seed=55):
        if threads:
            torch.set_num_threads(threads)
        self.threads = torch.get_num_threads()
        s0, obs, post, rew, done = record
        self.envs = [ReplayEnv(s0[i], obs[i], post[i], rew[i], done[i]) for i in range(len(s0))]
        self.n_envs, self.T, self.A = len(self.envs), n_steps, n_actions
        self.states = [e.reset() for e in self.envs]
        self.dones = np.zeros(self.n_envs, np.float32)
        gen = torch.Generator().manual_seed(seed)
        d = s0.shape[1]
        self.actor, self.critic = _mlp([d, 64, 64, n_actions], gen), _mlp([d, 64, 64, 1], gen)
        self.m = [torch.zeros_like(p) for p in self.critic]
        self.v = [torch.zeros_like(p) for p in self.critic]
        self.t = 0
        self.gamma, self.lam, self.max_kl = gamma, lam, max_kl
        self.cg_iterations, self.cg_damping = cg_iterations, cg_damping
        self.actor_iterations, self.critic_iterations = actor_iterations, critic_iterations
        self.fvp_n_steps, self.epochs, self.mini_batches = fvp_n_steps, epochs, mini_batches
        self.entropy_coef, self.lr = entropy_coef, lr
        self.steps = 0

    # ---- rollout + GAE --------------------------------------------------------------
    def get_batch(self):
        N, T = self.n_envs, self.T
        states, actions, values, rewards, dones = [], [], [], [], [self.dones.copy()]
        for _ in range(T):
            x = torch.from_numpy(np.array(self.states, np.float32))
            with torch.no_grad():
                a = torch.distributions.Categorical(logits=_fwd(self.actor, x)).sample()
                v = _fwd(self.critic, x).squeeze(-1)
            states.append(x.numpy())
            actions.append(a.numpy())
            values.append(v.numpy())
            r, d = np.zeros(N, np.float32), np.zeros(N, np.float32)
            for i, env in enumerate(self.envs):
                ns, r[i], d[i], _ = env.step(int(a[i]))
                self.states[i] = env.reset() if d[i] else ns
                self.steps += 1
            rewards.append(r)
            dones.append(d)
        self.dones = dones[-1]
        with torch.no_grad():
            nv = _fwd(self.critic, torch.from_numpy(np.array(self.states, np.float32)))
        vals = np.concatenate([np.array(values), nv.numpy().T], 0)
        dn = np.concatenate([np.array(dones), dones[-1][None]], 0)
        adv, last = np.zeros((T, N), np.float32), 0.0
        for t in reversed(range(T)):
            nnt = 1.0 - dn[t + 1]
            delta = rewards[t] + self.gamma * vals[t + 1] * nnt - vals[t]
            adv[t] = last = delta + self.gamma * self.lam * nnt * last
        ret = adv + vals[:-1]
        em = lambda x: np.asarray(x).swapaxes(0, 1).reshape(N * T, *np.asarray(x).shape[2:])  # noqa
        return em(states), em(actions), em(values), em(ret)

    # ---- actor ------------------------------------------------------------------------
    def _losses(self, s, a, adv, old_logits):
        lp = torch.log_softmax(_fwd(self.actor, s), -1)
        olp = torch.log_softmax(old_logits, -1)
        ratio = torch.exp(lp.gather(1, a[:, None]) - olp.gather(1, a[:, None])).squeeze(1)
        ent = -(lp.exp() * lp).sum(-1).mean()
        kl = (olp.exp() * (olp - lp)).sum(-1).mean()
        return (ratio * adv).mean() + self.entropy_coef * ent, kl

    def _fvp(self, s_sub, old_sub, v):
        lp = torch.log_softmax(_fwd(self.actor, s_sub), -1)
        olp = torch.log_softmax(old_sub, -1)
        kl = (olp.exp() * (olp - lp)).sum(-1).mean()
        g = torch.autograd.grad(kl, self.actor, create_graph=True)
        gv = sum((gi * vi).sum() for gi, vi in zip(g, self._unflat(v)))
        hv = torch.autograd.grad(gv, self.actor)
        return torch.cat([h.reshape(-1) for h in hv]) + self.cg_damping * v

    def _unflat(self, v):
        out, o = [], 0
        for p in self.actor:
            out.append(v[o:o + p.numel()].reshape(p.shape))
            o += p.numel()
        return out

    def train_step(self):
        s, a, old_v, ret = self.get_batch()
        s, a = torch.from_numpy(s), torch.from_numpy(a.astype(np.int64))
        adv = ret - old_v
        adv = torch.from_numpy((adv - adv.mean()) / (adv.std() + 1e-8))
        with torch.no_grad():
            old_logits = _fwd(self.actor, s)
        loss, _ = self._losses(s, a, adv, old_logits)
        g = torch.cat([x.reshape(-1) for x in torch.autograd.grad(loss, self.actor)])
        idx = torch.arange(0, s.shape[0], self.fvp_n_steps)
        s_sub, old_sub = s[idx], old_logits[idx]
        x, r = torch.zeros_like(g), g.clone()
        p, rr = r.clone(), r @ r
        for _ in range(self.cg_iterations):
            if rr <= 1e-10:
                break
            z = self._fvp(s_sub, old_sub, p)
            alpha = rr / (p @ z)
            x += alpha * p
            r -= alpha * z
            rr_new = r @ r
            p = r + (rr_new / rr) * p
            rr = rr_new
        shs = 0.5 * (x @ self._fvp(s_sub, old_sub, x))
        full_step = x / torch.sqrt(shs / self.max_kl)
        w0 = [p.detach().clone() for p in self.actor]
        lr = 1.0
        with torch.no_grad():
            for _ in range(self.actor_iterations):
                for prm, w, st in zip(self.actor, w0, self._unflat(full_step)):
                    prm.copy_(w + lr * st)
                new_loss, kl = self._losses(s, a, adv, old_logits)
                if torch.isfinite(new_loss) and kl <= self.max_kl * 1.5 and new_loss > loss:
                    break
                lr *= 0.5
            else:
                for prm, w in zip(self.actor, w0):
                    prm.copy_(w)
        retv = torch.from_numpy(ret)
        B, mb = s.shape[0], s.shape[0] // self.mini_batches
        for _ in range(self.critic_iterations * self.epochs):
            perm = torch.from_numpy(np.random.permutation(B))
            for i in range(0, B, mb):
                j = perm[i:i + mb]
                vl = ((_fwd(self.critic, s[j]).squeeze(-1) - retv[j]) ** 2).mean()
                grads = torch.autograd.grad(vl, self.critic)
                self.t += 1
                alpha = self.lr * np.sqrt(1 - 0.999 ** self.t) / (1 - 0.9 ** self.t)
                with torch.no_grad():
                    for prm, gi, m, v in zip(self.critic, grads, self.m, self.v):
                        m += (gi - m) * (1 - 0.9)
                        v += (gi * gi - v) * (1 - 0.999)
                        prm -= m * alpha / (torch.sqrt(v) + 1e-7)


def time_trpo(record, seconds=15.0, threads=None, min_steps=1, n_steps=512):
    agent = CpuTRPO(record, n_steps=n_steps, threads=threads)
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
