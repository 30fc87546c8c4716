"""Factory layer with the signatures of xagents/utils/common.py:
create_model / create_models (430-512), create_buffers (515-565), create_agent
(568-624), register_models (309-339), write_from_dict (416-427). ModelReader lives
in xagents_amd.nets (device models instead of Keras graphs).
"""
from pathlib import Path

from xagents_amd.utils.buffers import ReplayBuffer1, ReplayBuffer2


class LazyFrames:
    """The reference's Atari frame container (xagents/utils/common.py:23-64): wraps a
    uint8 frame array, materialised once on first use; np.asarray / len / indexing /
    count() behave as there. Here frames live in HBM rings, so agent.states hands out
    LazyFrames over host copies for user code; the device path never builds them."""

    def __init__(self, frames):
        self.frames = frames
        self.out = None
        self.dtype = frames.dtype
        self.shape = frames.shape

    def process_frame(self):
        if self.out is None:
            import numpy as np
            self.out = np.array(self.frames)
            self.frames = None
        return self.out

    def __array__(self, dtype=None, copy=None):
        out = self.process_frame()
        return out if dtype is None else out.astype(dtype)

    def __len__(self):
        return len(self.process_frame())

    def __getitem__(self, i):
        return self.process_frame()[i]

    def count(self):
        frames = self.process_frame()
        return frames.shape[frames.ndim - 1]


class DeviceStates:
    """BaseAgent.states as the reference exposes it -- a per-env sequence (base.py:105,
    407-424) -- over the device env's [n_envs, *obs] state tensor: states[i] is a host
    copy (LazyFrames for image observations, a numpy array otherwise), np.asarray(states)
    the stacked host array; `.tensor` is the device tensor itself."""

    def __init__(self, tensor):
        self.tensor = tensor

    def __len__(self):
        return self.tensor.shape[0]

    def _host(self, x):
        a = x.detach().cpu().numpy()
        return LazyFrames(a) if a.ndim >= 2 else a

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._host(x) for x in self.tensor[i]]
        return self._host(self.tensor[i])

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def __array__(self, dtype=None, copy=None):
        a = self.tensor.detach().cpu().numpy()
        return a if dtype is None else a.astype(dtype)


def write_from_dict(_dict, path):
    """Append one row to a parquet dataset (training history)."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    pq.write_to_dataset(pa.Table.from_pydict(_dict), root_path=path, compression='gzip')


def _cfg_group(path, group):
    for key in ('cnn', 'ann'):
        if key in path:
            group[key].append(path)


def register_models(agents):
    """Attach default .cfg paths found under each agent's models/ folder."""
    for agent_data in agents.values():
        folder = Path(agent_data['module'].__file__).parent / 'models'
        if not folder.exists():
            continue
        groups = {k: {'cnn': [], 'ann': []} for k in ('actor_model', 'critic_model', 'model')}
        for cfg in sorted(p.as_posix() for p in folder.iterdir() if p.suffix == '.cfg'):
            name = Path(cfg).name
            has_actor, has_critic = 'actor' in name, 'critic' in name
            if has_actor == has_critic:
                _cfg_group(cfg, groups['model'])
            elif has_actor:
                _cfg_group(cfg, groups['actor_model'])
            else:
                _cfg_group(cfg, groups['critic_model'])
        for key, val in groups.items():
            if any(val.values()):
                agent_data[key] = val


def create_model(env, agent_id, model_type, optimizer_kwargs=None, seed=None, model_cfg=None,
                 device=None):
    """Output-unit rules of xagents/utils/common.py:447-487: [n_actions] (+[1] for
    actor-critic cfgs, acer duplicates, critics output 1; td3/ddpg critics take
    obs + action inputs)."""
    import xagents_amd
    from xagents_amd.envs import Box, Discrete
    from xagents_amd.nets import Adam, ModelReader

    space = env.action_space
    units = [space.n if isinstance(space, Discrete) else space.shape[0]]
    network_type = 'cnn' if len(env.observation_space.shape) == 3 else 'ann'
    try:
        model_cfg = model_cfg or xagents_amd.agents[agent_id][model_type][network_type][0]
    except (IndexError, KeyError):
        model_cfg = None
    folder = Path(xagents_amd.agents[agent_id]['module'].__file__).parent / 'models'
    assert model_cfg, (
        f'You should specify `model_cfg`. No default '
        f'{network_type.upper()} model found in\n{folder}'
    )
    name = Path(model_cfg).name
    if agent_id == 'acer':
        units.append(units[-1])
    elif 'actor' in name and 'critic' in name:
        units.append(1)
    elif 'critic' in name:
        units[0] = 1
    input_shape = env.observation_space.shape
    if agent_id in ('td3', 'ddpg') and 'critic' in name:
        assert isinstance(space, Box), (
            f'Invalid environment: {env.spec.id}. {agent_id.upper()} supports '
            f'environments with a Box action space only, got {space}'
        )
        input_shape = (input_shape[0] + space.shape[0],)
    reader = ModelReader(model_cfg, units, input_shape, Adam(**(optimizer_kwargs or {})), seed,
                         device=device)
    return reader.build_model()


def create_models(options, env, agent_id, **kwargs):
    models = {}
    for model_type in ('model', 'actor_model', 'critic_model'):
        if model_type in options:
            cfg = options[model_type]
            cfg = cfg if isinstance(cfg, (str, Path)) else None
            models[model_type] = create_model(env, agent_id, model_type, model_cfg=cfg, **kwargs)
    return models


def create_buffers(agent_id, max_size, batch_size, n_envs, initial_size=None, as_total=True):
    """One buffer per env; totals are split with integer division when as_total
    (xagents/utils/common.py:515-565)."""
    initial_size = initial_size or max_size
    if as_total:
        max_size, initial_size, batch_size = (v // n_envs for v in (max_size, initial_size,
                                                                    batch_size))
    if agent_id == 'acer':
        batch_size = 1
    kwargs = dict(initial_size=initial_size, batch_size=batch_size)
    if agent_id in ('td3', 'ddpg'):
        return [ReplayBuffer2(max_size, 5, **kwargs) for _ in range(n_envs)]
    return [ReplayBuffer1(max_size, **kwargs) for _ in range(n_envs)]


def create_agent(agent_id, agent_kwargs, non_agent_kwargs, trial=None):
    """Build envs, models (and buffers) then the agent (xagents/utils/common.py:568-624)."""
    import xagents_amd
    from xagents_amd.envs import create_envs

    agent_kwargs['trial'] = trial
    envs = create_envs(non_agent_kwargs['env'], non_agent_kwargs['n_envs'],
                       non_agent_kwargs.get('preprocess', False),
                       mode=non_agent_kwargs.get('env_mode', 'replay'),
                       seed=agent_kwargs.get('seed') or 55)
    agent_kwargs['envs'] = envs
    optimizer_kwargs = {
        'learning_rate': non_agent_kwargs['lr'],
        'beta_1': non_agent_kwargs['beta1'],
        'beta_2': non_agent_kwargs['beta2'],
        'epsilon': non_agent_kwargs['opt_epsilon'],
    }
    agent_kwargs.update(create_models(agent_kwargs, envs[0], agent_id,
                                      optimizer_kwargs=optimizer_kwargs,
                                      seed=agent_kwargs.get('seed'), device=envs.device))
    agent_cls = xagents_amd.agents[agent_id]['agent']
    if issubclass(agent_cls, xagents_amd.OffPolicy) or agent_id == 'acer':
        agent_kwargs['buffers'] = create_buffers(
            agent_id, non_agent_kwargs['buffer_max_size'], non_agent_kwargs['buffer_batch_size'],
            non_agent_kwargs['n_envs'], non_agent_kwargs['buffer_initial_size'])
    agent = agent_cls(**agent_kwargs)
    weights = non_agent_kwargs.get('weights')
    if weights:
        n_models = len(agent.output_models)
        assert len(weights) == n_models, f'Expected {n_models} weights to load, got {len(weights)}'
        for weight, model in zip(weights, agent.output_models):
            model.load_weights(weight).expect_partial()
    return agent
