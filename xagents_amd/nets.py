"""Device-resident models built from the reference's .cfg grammar.

Mirrors xagents.utils.common.ModelReader (xagents/utils/common.py:169-290): INI
sections `convolutional-*`, `flatten-*`, `dense-*` with keys filters/size/stride/
units/activation/initializer/gain/common/output. Instead of a Keras graph the
reader produces a model whose parameters live in ONE flat f32 device buffer in
Keras `trainable_variables` order (kernel (in, out), bias per layer, layer creation
order), with Keras-Adam state (m, v, iterations) beside it. Forward/backward run
in libxagents_hip.so; there is no CPU compute path.
"""
import configparser
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch

MLP_HIDDEN = 64


class Adam:
    """Keras OptimizerV2 Adam configuration + device state.

    Defaults match tf.keras.optimizers.Adam; xagents passes lr/beta1/beta2/epsilon
    from the CLI (xagents/utils/common.py:589-594, xagents/utils/cli.py:14-37).
    """

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **_):
        self.learning_rate = float(learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.m = None
        self.v = None
        self.iterations = None  # device int32 [1] (Keras `iterations`)

    def get_config(self):
        return {
            'name': 'Adam',
            'learning_rate': self.learning_rate,
            'beta_1': self.beta_1,
            'beta_2': self.beta_2,
            'epsilon': self.epsilon,
        }

    def bind(self, n_params, device):
        self.m = torch.zeros(n_params, dtype=torch.float32, device=device)
        self.v = torch.zeros(n_params, dtype=torch.float32, device=device)
        self.iterations = torch.zeros(1, dtype=torch.int32, device=device)


@dataclass
class LayerSpec:
    name: str
    kind: str  # dense | convolutional | flatten
    units: int = 0
    activation: str = None
    initializer: str = None
    gain: float = None
    filters: int = 0
    size: int = 0
    stride: int = 1
    common: bool = False
    output: bool = False
    input_index: int = -1  # index into the layer list this layer reads (-1: model input)
    in_features: int = 0
    out_shape: tuple = field(default_factory=tuple)


def orthogonal(shape, gain, rng):
    """tf.keras.initializers.Orthogonal (QR of a normal matrix, sign-fixed)."""
    num_rows = int(np.prod(shape[:-1]))
    num_cols = shape[-1]
    flat = (max(num_cols, num_rows), min(num_cols, num_rows))
    a = rng.standard_normal(flat)
    q, r = np.linalg.qr(a)
    q *= np.sign(np.diag(r))
    if num_rows < num_cols:
        q = q.T
    return (gain * q.reshape(shape)).astype(np.float32)


def glorot_uniform(shape, rng):
    """tf.keras.initializers.GlorotUniform (fan_in = prod(shape[:-1]) for 2D/conv)."""
    receptive = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    fan_in = shape[-2] * receptive
    fan_out = shape[-1] * receptive
    limit = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-limit, limit, size=shape).astype(np.float32)


class DeviceModel:
    """A model parsed from .cfg with flat device parameters."""

    fused_kind = None

    def __init__(self, layers, input_shape, optimizer=None, seed=None, device=None):
        self.layers = layers
        self.input_shape = tuple(input_shape)
        self.optimizer = optimizer
        self.seed = seed
        self.device = torch.device(device) if device is not None else default_device()
        self.outputs = [i for i, l in enumerate(layers) if l.output]
        self.weight_shapes = []
        for layer in layers:
            if layer.kind == 'dense':
                self.weight_shapes += [(layer.in_features, layer.units), (layer.units,)]
            elif layer.kind == 'convolutional':
                self.weight_shapes += [(layer.size, layer.in_features, layer.filters),
                                       (layer.filters,)]
        self.n_params = int(sum(np.prod(s) for s in self.weight_shapes))
        self.theta = torch.from_numpy(np.concatenate(
            [w.ravel() for w in self._init_weights()])).to(self.device)
        if optimizer is not None:
            optimizer.bind(self.n_params, self.device)

    def _init_weights(self):
        weights = []
        for layer in self.layers:
            if layer.kind not in ('dense', 'convolutional'):
                continue
            if layer.kind == 'dense':
                shape = (layer.in_features, layer.units)
                nb = layer.units
            else:
                shape = (layer.size, layer.in_features, layer.filters)
                nb = layer.filters
            # a seeded Keras initializer yields the same draw on every call
            # (xagents/utils/common.py:198-216 passes the same seed to each layer)
            rng = np.random.default_rng(self.seed)
            name = layer.initializer or 'glorot_uniform'
            if name == 'orthogonal':
                w = orthogonal(shape, layer.gain if layer.gain is not None else 1.0, rng)
            else:
                w = glorot_uniform(shape, rng)
            weights += [w, np.zeros(nb, np.float32)]
        return weights

    def clone(self, theta=None):
        """Same architecture, own parameter buffer (copy of this model's unless
        `theta` is given), no optimizer: the target networks of DQN / DDPG / TD3."""
        import copy
        m = copy.copy(self)
        m.theta = self.theta.clone() if theta is None else theta
        m.optimizer = None
        return m

    # -- Keras-compatible weight access ------------------------------------
    def get_weights(self):
        flat = self.theta.detach().cpu().numpy()
        out, off = [], 0
        for s in self.weight_shapes:
            n = int(np.prod(s))
            out.append(flat[off:off + n].reshape(s).copy())
            off += n
        return out

    def set_weights(self, weights):
        assert len(weights) == len(self.weight_shapes), (
            f'Expected {len(self.weight_shapes)} weight arrays, got {len(weights)}')
        flat = []
        for w, s in zip(weights, self.weight_shapes):
            w = np.asarray(w, np.float32)
            assert w.shape == tuple(s), f'Expected weight shape {s}, got {w.shape}'
            flat.append(w.ravel())
        self.theta.copy_(torch.from_numpy(np.concatenate(flat)).to(self.device))

    @property
    def trainable_variables(self):
        return self.get_weights()

    def save_weights(self, path):
        """Flat checkpoint (weights + Adam state); the reference's TF `.tf` format
        cannot be produced without TF (xagents/base.py:227-229)."""
        state = {'theta': self.theta.detach().cpu().numpy()}
        if self.optimizer is not None and self.optimizer.m is not None:
            state['adam_m'] = self.optimizer.m.cpu().numpy()
            state['adam_v'] = self.optimizer.v.cpu().numpy()
            state['adam_t'] = self.optimizer.iterations.cpu().numpy()
        np.savez(Path(path), **state)

    def load_weights(self, path):
        p = Path(path)
        if not p.exists() and p.with_suffix(p.suffix + '.npz').exists():
            p = p.with_suffix(p.suffix + '.npz')
        with np.load(p, allow_pickle=False) as data:
            theta = data['theta']
            assert theta.size == self.n_params, (
                f'Checkpoint holds {theta.size} parameters, model has {self.n_params}')
            self.theta.copy_(torch.from_numpy(theta).to(self.device))
            if 'adam_m' in data and self.optimizer is not None:
                self.optimizer.m.copy_(torch.from_numpy(data['adam_m']).to(self.device))
                self.optimizer.v.copy_(torch.from_numpy(data['adam_v']).to(self.device))
                self.optimizer.iterations.copy_(
                    torch.from_numpy(data['adam_t']).to(self.device))
        return self

    def expect_partial(self):
        return self


class ActorCriticMLP(DeviceModel):
    """obs -> 64 tanh -> 64 tanh (common) -> {A logits, 1 value}: the topology of
    xagents/{a2c,ppo}/models/ann-actor-critic.cfg, run by the fused HIP kernels."""

    fused_kind = 'actor_critic_mlp'

    def __init__(self, layers, input_shape, n_actions, **kwargs):
        self.n_actions = n_actions
        self.obs_dim = int(input_shape[0])
        super().__init__(layers, input_shape, **kwargs)

    def __call__(self, inputs, training=False):
        """[logits, value] for a [B, obs] batch (Keras model call semantics)."""
        from xagents_amd import kernels
        obs = torch.as_tensor(inputs, dtype=torch.float32, device=self.device).reshape(
            -1, self.obs_dim).contiguous()
        _, _, value, _, logits = kernels.mlp_forward(
            self.theta, obs, self.n_actions,
            actions=torch.zeros(obs.shape[0], dtype=torch.int32, device=self.device),
            want_logits=True)
        return [logits, value.unsqueeze(-1)]


def default_device():
    return torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu')


def _is_actor_critic_mlp(layers, input_shape, units):
    dense = [l for l in layers if l.kind == 'dense']
    if len(input_shape) != 1 or len(dense) != 4 or len(layers) != 4:
        return False
    d0, d1, d2, d3 = dense
    return (d0.units == MLP_HIDDEN and d1.units == MLP_HIDDEN and d0.activation == 'tanh'
            and d1.activation == 'tanh' and d1.common and d2.output and d3.output
            and d2.input_index == 1 and d3.input_index == 1 and d3.units == 1
            and d2.activation in (None, 'linear') and d3.activation in (None, 'linear'))


class ModelReader:
    """Parse a .cfg into a device model (xagents/utils/common.py:169-290)."""

    def __init__(self, cfg_file, output_units, input_shape, optimizer=None, seed=None,
                 device=None):
        self.initializers = ('orthogonal', 'glorot_uniform')
        self.cfg_file = cfg_file
        with open(cfg_file) as cfg:
            self.parser = configparser.ConfigParser()
            self.parser.read_file(cfg)
        self.optimizer = optimizer
        self.output_units = output_units
        self.input_shape = input_shape
        self.seed = seed
        self.device = device
        self.output_count = 0

    def get_initializer(self, section):
        name = self.parser[section].get('initializer')
        if self.seed is not None:
            name = name or 'glorot_uniform'
        gain = self.parser[section].get('gain')
        return (name if name in self.initializers else None), (float(gain) if gain else None)

    def _parse(self):
        sections = self.parser.sections()
        assert sections, f'Empty model configuration {self.cfg_file}'
        layers = []
        shape = tuple(np.atleast_1d(self.input_shape))
        current, common = -1, None
        shapes = {-1: shape}
        for section in sections:
            sec = self.parser[section]
            layer = None
            if section.startswith('convolutional'):
                init, gain = self.get_initializer(section)
                in_shape = shapes[current]
                size, stride = int(sec['size']), int(sec['stride'])
                out_w = (in_shape[-2] - size) // stride + 1
                layer = LayerSpec(section, 'convolutional', filters=int(sec['filters']),
                                  size=size, stride=stride, activation=sec.get('activation'),
                                  initializer=init, gain=gain, input_index=current,
                                  in_features=in_shape[-1])
                layer.out_shape = (*in_shape[:-2], out_w, layer.filters)
            if section.startswith('flatten'):
                layer = LayerSpec(section, 'flatten', input_index=current)
                layer.out_shape = (int(np.prod(shapes[current])),)
            if section.startswith('dense'):
                units = sec.get('units')
                if not units:
                    assert len(self.output_units) > self.output_count, (
                        'Output units given are less than dense layers required')
                    units = self.output_units[self.output_count]
                    self.output_count += 1
                init, gain = self.get_initializer(section)
                src = common if common is not None else current
                layer = LayerSpec(section, 'dense', units=int(units),
                                  activation=sec.get('activation'), initializer=init, gain=gain,
                                  input_index=src, in_features=int(shapes[src][-1]))
                layer.out_shape = (*shapes[src][:-1], int(units))
            if layer is None:
                continue
            layers.append(layer)
            current = len(layers) - 1
            shapes[current] = layer.out_shape
            if sec.get('common'):
                layer.common = True
                common = current
            if sec.get('output'):
                layer.output = True
        self.output_count = 0
        return layers

    def build_model(self):
        layers = self._parse()
        kwargs = dict(optimizer=self.optimizer, seed=self.seed, device=self.device)
        shape = tuple(np.atleast_1d(self.input_shape))
        if _is_actor_critic_mlp(layers, shape, self.output_units):
            return ActorCriticMLP(layers, shape, n_actions=layers[2].units, **kwargs)
        return DeviceModel(layers, shape, **kwargs)
