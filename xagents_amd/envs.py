"""Device-resident vectorized environments.

The reference steps a Python list of gym envs one by one (xagents/base.py:388-426,
created by create_envs, xagents/utils/common.py:145-166). Here the env state of
all n envs lives in HBM and is stepped inside the fused rollout kernel:

* ReplayVecEnv -- synthetic pre-recorded observation replay (BASELINE config 2):
  per env a recorded stream of (obs returned by step, post-reset state, reward,
  done) of length t_rec, generated once on the host from a CartPole-v1
  restatement with a seeded random policy; stepping advances a per-env cursor.
* CartPoleVecEnv -- gym CartPole-v1 dynamics (Euler, f64 state, TimeLimit 500)
  evaluated on device, actions applied.

Both expose the gym-like surface the agents use: len(), observation_space.shape,
action_space (Discrete/Box), seed(), reset().
"""
import numpy as np
import torch

from xagents_amd._lib import XA_ENV_CARTPOLE, XA_ENV_REPLAY
from xagents_amd.nets import default_device


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self._rng = np.random.default_rng()

    def seed(self, seed):
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return int(self._rng.integers(self.n))

    def __repr__(self):
        return f'Discrete({self.n})'


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high = low, high
        self.shape = tuple(shape)
        self.dtype = dtype
        self._rng = np.random.default_rng()

    def seed(self, seed):
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def __repr__(self):
        return f'Box({self.low}, {self.high}, {self.shape}, {np.dtype(self.dtype).name})'


class EnvSpec:
    def __init__(self, id, max_episode_steps=None):
        self.id = id
        self.max_episode_steps = max_episode_steps


class CartPoleNumpy:
    """Vectorized CartPole-v1 restatement (gym classic_control/cartpole.py) in f64,
    used only to RECORD synthetic replay streams on the host."""

    gravity, masspole, total_mass, length = 9.8, 0.1, 1.1, 0.5
    polemass_length, force_mag, tau = 0.05, 10.0, 0.02
    theta_threshold = 12 * 2 * np.pi / 360
    x_threshold = 2.4

    def __init__(self, n, rng, max_episode_steps=500):
        self.n = n
        self.rng = rng
        self.max_episode_steps = max_episode_steps
        self.state = self.rng.uniform(-0.05, 0.05, (n, 4))
        self.elapsed = np.zeros(n, np.int64)

    def step(self, action):
        x, x_dot, theta, theta_dot = self.state.T
        force = np.where(action == 1, self.force_mag, -self.force_mag)
        costheta, sintheta = np.cos(theta), np.sin(theta)
        temp = (force + self.polemass_length * theta_dot ** 2 * sintheta) / self.total_mass
        thetaacc = (self.gravity * sintheta - costheta * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * costheta ** 2 / self.total_mass))
        xacc = temp - self.polemass_length * thetaacc * costheta / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        theta = theta + self.tau * theta_dot
        theta_dot = theta_dot + self.tau * thetaacc
        self.state = np.stack([x, x_dot, theta, theta_dot], 1)
        self.elapsed += 1
        done = ((x < -self.x_threshold) | (x > self.x_threshold)
                | (theta < -self.theta_threshold) | (theta > self.theta_threshold)
                | (self.elapsed >= self.max_episode_steps))
        obs = self.state.astype(np.float32)
        reset = self.rng.uniform(-0.05, 0.05, (self.n, 4))
        self.state = np.where(done[:, None], reset, self.state)
        self.elapsed = np.where(done, 0, self.elapsed)
        return obs, np.ones(self.n, np.float32), done, self.state.astype(np.float32)


def record_cartpole_replay(n_envs, t_rec, seed=55, max_episode_steps=500):
    """Record per-env CartPole-v1 streams under a uniform random policy
    (np.random.default_rng(seed)).

    Returns numpy arrays: s0 [N,4], rep_obs [N,t_rec,4] (obs returned by step p),
    rep_state [N,t_rec,4] (state after step p, post-reset), rep_rew [N,t_rec],
    rep_done [N,t_rec]. The last record of every env is forced terminal with
    post-state s0, so the cursor wrap-around is an ordinary episode boundary.
    """
    rng = np.random.default_rng(seed)
    env = CartPoleNumpy(n_envs, rng, max_episode_steps)
    s0 = env.state.astype(np.float32)
    rep_obs = np.empty((n_envs, t_rec, 4), np.float32)
    rep_state = np.empty((n_envs, t_rec, 4), np.float32)
    rep_rew = np.empty((n_envs, t_rec), np.float32)
    rep_done = np.empty((n_envs, t_rec), np.float32)
    for p in range(t_rec):
        obs, rew, done, post = env.step(rng.integers(0, 2, n_envs))
        rep_obs[:, p], rep_state[:, p], rep_rew[:, p] = obs, post, rew
        rep_done[:, p] = done
    rep_done[:, -1] = 1.0
    rep_state[:, -1] = s0
    return s0, rep_obs, rep_state, rep_rew, rep_done


class DeviceVecEnv:
    """Common device-side env state: the reference's BaseAgent.states / dones /
    episode_rewards arrays (xagents/base.py:105-113) kept in HBM."""

    kind = None

    def __init__(self, env_id, n_envs, obs_shape, action_space, device=None):
        self.spec = EnvSpec(env_id)
        self.n_envs = int(n_envs)
        self.device = torch.device(device) if device is not None else default_device()
        self.observation_space = Box(-np.inf, np.inf, obs_shape)
        self.action_space = action_space
        self.obs_dim = int(np.prod(obs_shape))
        n, dev = self.n_envs, self.device
        self.state = torch.zeros(n, self.obs_dim, dtype=torch.float32, device=dev)
        self.done = torch.zeros(n, dtype=torch.float32, device=dev)
        self.cursor = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ep_return = torch.zeros(n, dtype=torch.float32, device=dev)
        self.state64 = None
        self._seed = None

    def __len__(self):
        return self.n_envs

    def __iter__(self):
        return iter([self] * self.n_envs)

    def __getitem__(self, i):
        return self  # envs[0].observation_space / action_space access pattern

    def seed(self, seed):
        self._seed = seed
        self.action_space.seed(seed)

    def fill_rollout_args(self, a):
        a.env_kind = self.kind
        a.env_state = self.state.data_ptr()
        a.env_done = self.done.data_ptr()
        a.env_cursor = self.cursor.data_ptr()
        a.ep_return = self.ep_return.data_ptr()


class ReplayVecEnv(DeviceVecEnv):
    kind = XA_ENV_REPLAY

    def __init__(self, env_id='CartPole-v1', n_envs=1, t_rec=4096, seed=55, device=None,
                 record=None):
        super().__init__(env_id, n_envs, (4,), Discrete(2), device)
        s0, rep_obs, rep_state, rep_rew, rep_done = record or record_cartpole_replay(
            n_envs, t_rec, seed)
        self.t_rec = rep_obs.shape[1]
        dev = self.device
        self.s0 = torch.from_numpy(s0).to(dev)
        self.rep_obs = torch.from_numpy(np.ascontiguousarray(rep_obs)).to(dev)
        self.rep_state = torch.from_numpy(np.ascontiguousarray(rep_state)).to(dev)
        self.rep_rew = torch.from_numpy(np.ascontiguousarray(rep_rew)).to(dev)
        self.rep_done = torch.from_numpy(np.ascontiguousarray(rep_done)).to(dev)
        self.reset()

    def reset(self):
        self.state.copy_(self.s0)
        self.cursor.zero_()
        self.done.zero_()
        self.ep_return.zero_()
        return self.state

    def fill_rollout_args(self, a):
        super().fill_rollout_args(a)
        a.rep_obs = self.rep_obs.data_ptr()
        a.rep_state = self.rep_state.data_ptr()
        a.rep_rew = self.rep_rew.data_ptr()
        a.rep_done = self.rep_done.data_ptr()
        a.t_rec = self.t_rec


class CartPoleVecEnv(DeviceVecEnv):
    kind = XA_ENV_CARTPOLE
    max_episode_steps = 500

    def __init__(self, n_envs=1, seed=None, device=None):
        super().__init__('CartPole-v1', n_envs, (4,), Discrete(2), device)
        self.state64 = torch.zeros(self.n_envs, 4, dtype=torch.float64, device=self.device)
        self._seed = seed
        self.reset()

    def reset(self):
        rng = np.random.default_rng(self._seed)
        s = rng.uniform(-0.05, 0.05, (self.n_envs, 4))
        self.state64.copy_(torch.from_numpy(s))
        self.state.copy_(torch.from_numpy(s.astype(np.float32)))
        self.cursor.zero_()
        self.done.zero_()
        self.ep_return.zero_()
        return self.state

    def fill_rollout_args(self, a):
        super().fill_rollout_args(a)
        a.env_state64 = self.state64.data_ptr()
        a.max_episode_steps = self.max_episode_steps


def record_transitions(n_envs, t_rec, obs_shape, dtype, seed=55, mean_episode=200,
                       reward_prob=0.02):
    """Synthetic pre-recorded transition streams for the off-policy configs
    (C3 Pong-shaped uint8 (84, 84, 1) frames i.i.d. uniform 0..255;
    C5 BipedalWalker-shaped f32 obs ~ N(0, 1)). Per env: s0, rep_obs [t_rec] (obs
    returned by step p), rep_state [t_rec] (post-reset state), rewards in {-1, 0, 1}
    (Pong-like, prob reward_prob each sign), episode ends ~ Geometric(1 / mean_episode);
    the last record is terminal with post-state s0 so the cursor wrap is an episode
    boundary. Generated from np.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    shape = (n_envs, t_rec) + tuple(obs_shape)

    def frames(sh):
        if np.dtype(dtype) == np.uint8:
            return rng.integers(0, 256, size=sh, dtype=np.uint8)
        return rng.standard_normal(sh).astype(dtype)

    s0 = frames((n_envs,) + tuple(obs_shape))
    rep_obs = frames(shape)
    rep_done = (rng.random((n_envs, t_rec)) < 1.0 / mean_episode).astype(np.float32)
    rep_done[:, -1] = 1.0
    rep_state = rep_obs.copy()
    resets = frames(shape)
    m = rep_done.astype(bool)
    rep_state[m] = resets[m]
    rep_state[:, -1] = s0
    u = rng.random((n_envs, t_rec))
    rep_rew = np.where(u < reward_prob, 1.0, np.where(u > 1 - reward_prob, -1.0, 0.0))
    return s0, rep_obs, rep_state, rep_rew.astype(np.float32), rep_done


class TransitionReplayVecEnv:
    """Off-policy device env over pre-recorded transitions (Atari-shaped uint8 frames
    or continuous-control f32 vectors). Stepping -- and the replay-ring append of
    BaseAgent.step_envs(store_in_buffers=True), xagents/base.py:388-426 -- is one
    xa_replay_env_step launch; the actions are stored but do not change the stream."""

    def __init__(self, env_id, n_envs, obs_shape, action_space, obs_dtype=np.uint8,
                 t_rec=256, seed=55, device=None, record=None, mean_episode=200):
        self.spec = EnvSpec(env_id)
        self.n_envs = int(n_envs)
        self.device = torch.device(device) if device is not None else default_device()
        low, high = (0, 255) if np.dtype(obs_dtype) == np.uint8 else (-np.inf, np.inf)
        self.observation_space = Box(low, high, obs_shape, obs_dtype)
        self.action_space = action_space
        self.obs_dtype = np.dtype(obs_dtype)
        self.obs_shape = tuple(obs_shape)
        s0, rep_obs, rep_state, rep_rew, rep_done = record or record_transitions(
            n_envs, t_rec, obs_shape, obs_dtype, seed, mean_episode)
        self.t_rec = rep_obs.shape[1]
        dev = self.device
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.s0, self.rep_obs, self.rep_state = tt(s0), tt(rep_obs), tt(rep_state)
        self.rep_rew, self.rep_done = tt(rep_rew), tt(rep_done)
        self.state = torch.empty_like(self.s0)
        self.cursor = torch.zeros(self.n_envs, dtype=torch.int32, device=dev)
        self.done = torch.zeros(self.n_envs, dtype=torch.float32, device=dev)
        self.ep_return = torch.zeros(self.n_envs, dtype=torch.float32, device=dev)
        self.obs_bytes = int(np.prod(self.obs_shape)) * self.obs_dtype.itemsize
        self.reset()

    def __len__(self):
        return self.n_envs

    def __getitem__(self, i):
        return self

    def __iter__(self):
        return iter([self] * self.n_envs)

    def seed(self, seed):
        self.action_space.seed(seed)

    def reset(self):
        self.state.copy_(self.s0)
        self.cursor.zero_()
        self.done.zero_()
        self.ep_return.zero_()
        return self.state

    def fill_step_args(self, a):
        a.n_envs, a.t_rec, a.obs_bytes = self.n_envs, self.t_rec, self.obs_bytes
        a.rep_obs, a.rep_state = self.rep_obs.data_ptr(), self.rep_state.data_ptr()
        a.rep_rew, a.rep_done = self.rep_rew.data_ptr(), self.rep_done.data_ptr()
        a.state, a.cursor = self.state.data_ptr(), self.cursor.data_ptr()
        a.ep_return, a.done = self.ep_return.data_ptr(), self.done.data_ptr()


class WalkerVecEnv(TransitionReplayVecEnv):
    """BipedalWalker-v3 device stand-in (csrc/walker.hip): real
    action-dependent dynamics with BipedalWalker's 24-value observation, 4 motor commands
    in [-1, 1], reward formula and termination (not Box2D: a planar kinematic walker on flat
    ground). Each env step is one xa_walker_step launch (pre_step, given the step's actions)
    into the one-step record that xa_replay_env_step then turns into the agent's state,
    rewards, dones and replay-ring append, as for the other transition envs."""

    def __init__(self, env_id='BipedalWalker-v3', n_envs=1, seed=55, device=None):
        n = int(n_envs)
        z = np.zeros((n, 1, 24), np.float32)
        record = (np.zeros((n, 24), np.float32), z, z.copy(), np.zeros((n, 1), np.float32),
                  np.zeros((n, 1), np.float32))
        self._ready = False
        super().__init__(env_id, n, (24,), Box(-1.0, 1.0, (4,)), np.float32, seed=seed,
                         device=device, record=record)
        self.walker_seed = int(seed if seed is not None else 0) % 2**64
        self.walker_state = torch.zeros(n, 18, dtype=torch.float32, device=self.device)
        self.episode = torch.zeros(n, dtype=torch.int32, device=self.device)
        self._ready = True
        self.reset()

    def _args(self, reset_only, actions=0, act_ld=4):
        from xagents_amd._lib import XaWalkerStepArgs
        a = XaWalkerStepArgs()
        a.n_envs, a.state, a.episode = self.n_envs, self.walker_state.data_ptr(), \
            self.episode.data_ptr()
        a.actions, a.act_ld, a.seed, a.reset_only = actions, act_ld, self.walker_seed, \
            int(reset_only)
        return a

    def reset(self):
        """BipedalWalker.reset of every env into the state. The initial push is drawn from
        the env's episode counter, which only a finished episode advances (xa_walker_step),
        so repeated reset() calls without steps in between replay the same initial state."""
        super().reset()
        if not self._ready:
            return self.state
        import ctypes
        from xagents_amd._lib import call, stream
        a = self._args(True)
        a.out_post = self.state.data_ptr()
        call('xa_walker_step', ctypes.byref(a), stream())
        return self.state

    def pre_step(self, actions=None, act_ld=4):
        """env.step of every env with `actions` (a device tensor [N, 4] f32, or a pointer
        to rows of 4 f32 at row stride act_ld) into the one-step record."""
        import ctypes
        from xagents_amd._lib import call, stream
        if actions is None:
            raise ValueError('WalkerVecEnv.pre_step needs the step\'s actions')
        ptr = actions if isinstance(actions, int) else actions.data_ptr()
        if not isinstance(actions, int):
            assert actions.dtype == torch.float32 and actions.is_contiguous()
            act_ld = actions.shape[-1]
        a = self._args(False, ptr, act_ld)
        a.out_obs, a.out_post = self.rep_obs.data_ptr(), self.rep_state.data_ptr()
        a.out_rew, a.out_done = self.rep_rew.data_ptr(), self.rep_done.data_ptr()
        call('xa_walker_step', ctypes.byref(a), stream())


def create_envs(env_name, n=1, preprocess=False, *args, mode='replay', seed=55, device=None,
                t_rec=4096, **kwargs):
    """Device counterpart of xagents.utils.common.create_envs (common.py:145-166).

    Returns ONE vectorized env object of length n (the agents accept it wherever the
    reference takes a list of gym envs).
    """
    if 'NoFrameskip' in env_name and preprocess:
        # AtariWrapper on device over a synthetic raw RGB frame stream (atari.py)
        from xagents_amd.atari import AtariFrameVecEnv
        actions = {'PongNoFrameskip-v4': 6, 'BreakoutNoFrameskip-v4': 4}.get(env_name, 6)
        return AtariFrameVecEnv(env_name, n, actions, *args, seed=seed, device=device,
                                t_raw=kwargs.pop('t_raw_frames', 64), **kwargs)
    if 'NoFrameskip' in env_name:
        # Atari-shaped synthetic replay: frames as AtariWrapper emits them (84, 84, 1)
        # uint8 (xagents/utils/common.py:67-142); the wrapper itself is not rebuilt
        actions = {'PongNoFrameskip-v4': 6, 'BreakoutNoFrameskip-v4': 4}.get(env_name, 6)
        return TransitionReplayVecEnv(env_name, n, (84, 84, 1), Discrete(actions), np.uint8,
                                      t_rec=min(t_rec, 256), seed=seed, device=device)
    if env_name.startswith('BipedalWalker'):
        if mode == 'dynamics':
            return WalkerVecEnv(env_name, n, seed=seed, device=device)
        return TransitionReplayVecEnv(env_name, n, (24,), Box(-1.0, 1.0, (4,)), np.float32,
                                      t_rec=t_rec, seed=seed, device=device)
    assert not preprocess, (f'Cannot use AtariWrapper or --preprocess for non-atari '
                            f'environment {env_name}')
    if env_name != 'CartPole-v1':
        raise NotImplementedError(f'No device environment for {env_name}')
    if mode == 'replay':
        return ReplayVecEnv(env_name, n, t_rec=t_rec, seed=seed, device=device)
    if mode == 'dynamics':
        return CartPoleVecEnv(n, seed=seed, device=device)
    if mode == 'transitions':
        # the same CartPole record behind the executor env step (models run by the layer
        # executor, e.g. TRPO's separate actor and critic)
        return TransitionReplayVecEnv(env_name, n, (4,), Discrete(2), np.float32, seed=seed,
                                      device=device,
                                      record=record_cartpole_replay(n, t_rec, seed))
    raise ValueError(f'Unknown env mode {mode}')
