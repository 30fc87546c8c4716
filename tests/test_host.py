"""CPU tests of the host surface: buffers, factories, .cfg loader, the C ABI
exports, and the replay-env semantics of the rollout against the reference's own
BaseAgent.step_envs (tests/golden/step_envs.npz)."""
import random
import re
from pathlib import Path

import numpy as np
import oracle
import pytest

from xagents_amd._lib import XA_RING_DEQUE
from xagents_amd.utils.buffers import BaseBuffer, ReplayBuffer1, ReplayBuffer2
from xagents_amd.utils.common import create_buffers

ROOT = Path(__file__).resolve().parents[1]


# ---- buffers (xagents/tests/test_buffers.py cases + golden sequences) -------
@pytest.mark.parametrize('buffer_type', [ReplayBuffer1, ReplayBuffer2])
@pytest.mark.parametrize(
    'size, initial_size, batch_size, exception_kw',
    [
        [100, 0, 32, 'Buffer initial size should be > 0, got'],
        [-100, 100, 32, 'Buffer size should be > 0'],
        [10, None, 32, 'should be <= size'],
        [100, 200, 32, 'Buffer initial size exceeds max size'],
        [100, 50, 32, None],
        [100, None, 32, None],
    ],
)
def test_buffer_sizes(buffer_type, size, initial_size, batch_size, exception_kw):
    kwargs = dict(size=size, initial_size=initial_size, batch_size=batch_size)
    if buffer_type is ReplayBuffer2:
        kwargs['slots'] = 1
    if exception_kw:
        with pytest.raises(AssertionError, match=exception_kw):
            buffer_type(**kwargs)
    else:
        b = buffer_type(**kwargs)
        assert (b.size, b.batch_size) == (size, batch_size)
        assert b.initial_size == (initial_size or size)


def test_base_buffer_abstract():
    b = BaseBuffer(32)
    with pytest.raises(NotImplementedError, match='should be implemented'):
        b.append(1)
    with pytest.raises(NotImplementedError, match='should be implemented'):
        b.get_sample()


def test_replay_buffers_match_reference_sequences(golden):
    g = golden('buffers.npz')
    random.seed(11)
    rb = ReplayBuffer1(6, batch_size=3)
    for i in range(10):
        rb.append(np.full(2, i, np.int64), i, float(i) * 0.5, i % 3 == 0, np.full(2, -i, np.int64))
    for k in range(4):
        for f, arr in enumerate(rb.get_sample()):
            np.testing.assert_array_equal(arr, g[f'rb1_s{k}_f{f}'])
    assert rb.current_size == int(g['rb1_current_size'])
    rb1 = ReplayBuffer1(4, batch_size=1)
    random.seed(5)
    for i in range(4):
        rb1.append(i, 10 * i)
    one = rb1.get_sample()
    assert isinstance(one, tuple) == bool(g['rb1_one_is_tuple'])
    np.testing.assert_array_equal(np.asarray(one), g['rb1_one'])
    np.random.seed(3)
    rb2 = ReplayBuffer2(5, 3, batch_size=4)
    for i in range(9):
        rb2.append(np.arange(3, dtype=np.float32) + i, float(i), i % 2 == 0)
    for f, slot in enumerate(rb2.slots):
        np.testing.assert_array_equal(slot, g[f'rb2_slot{f}'])  # row-0 overwrite quirk
    assert rb2.current_size == int(g['rb2_current_size'])
    for k in range(3):
        for f, arr in enumerate(rb2.get_sample()):
            np.testing.assert_array_equal(arr, g[f'rb2_s{k}_f{f}'])


def test_create_buffers_matches_reference(golden):
    rows = golden('create_buffers.npz')['rows']
    i = 0
    for agent_id in ('dqn', 'td3', 'ddpg', 'acer'):
        for args in [(10000, 32, 16, None, True), (200000, 16, 16, 10000, False),
                     (1000000, 64, 32, None, True), (1000000, 100, 64, None, True),
                     (50000, 8, 3, 1000, False)]:
            bufs = create_buffers(agent_id, *args)
            got = [len(bufs), bufs[0].size, bufs[0].initial_size, bufs[0].batch_size,
                   int(isinstance(bufs[0], ReplayBuffer2))]
            assert got == rows[i].tolist(), (agent_id, args)
            i += 1


class _StubAgent:
    pass


def test_concat_buffer_samples_matches_reference(golden):
    from xagents_amd.base import BaseAgent

    g = golden('concat_buffer_samples.npz')
    random.seed(21)
    s = _StubAgent()
    s.n_envs = 3
    s.buffers = [ReplayBuffer1(8, batch_size=2) for _ in range(3)]
    s.batch_dtypes = ['uint8', 'int64', 'float64', 'bool', 'uint8']
    for b, buf in enumerate(s.buffers):
        for i in range(5):
            buf.append(np.full((2, 2), 10 * b + i, np.uint8), i, 0.25 * i, i == 4,
                       np.full((2, 2), 100 + 10 * b + i, np.uint8))
    res = BaseAgent.concat_buffer_samples(s)
    for f, arr in enumerate(res):
        np.testing.assert_array_equal(arr, g[f'dqn_f{f}'])
        assert arr.dtype == g[f'dqn_f{f}'].dtype
    s1 = _StubAgent()
    s1.n_envs = 2
    s1.buffers = [ReplayBuffer1(4, batch_size=1) for _ in range(2)]
    for buf in s1.buffers:
        buf.append(np.zeros(2), 1, 0.0, False, np.zeros(2))
    err = str(g['k1_error'])
    with pytest.raises(ValueError, match=err.split(': ', 1)[1]):
        BaseAgent.concat_buffer_samples(s1)


def test_concat_step_batches_matches_reference(golden):
    from xagents_amd.base import BaseAgent

    g = golden('concat_step_batches.npz')
    out = BaseAgent.concat_step_batches(g['states'], g['actions'], g['vec'])
    for o, key in zip(out, ('out_states', 'out_actions', 'out_vec')):
        np.testing.assert_array_equal(o, g[key])
    import torch

    out_t = BaseAgent.concat_step_batches(torch.from_numpy(g['states']),
                                          torch.from_numpy(g['actions']))
    np.testing.assert_array_equal(out_t[0].numpy(), g['out_states'])
    np.testing.assert_array_equal(out_t[1].numpy(), g['out_actions'])


# ---- model loader -------------------------------------------------------------
def _env(obs=(4,), n=2):
    from xagents_amd.envs import Box, Discrete

    class E:
        observation_space = Box(-1, 1, obs)
        action_space = Discrete(n)

    return E()


def test_model_reader_actor_critic_mlp():
    from xagents_amd.nets import ActorCriticMLP
    from xagents_amd.utils.common import create_model

    m = create_model(_env(), 'ppo', 'model', seed=55, device='cpu')
    assert isinstance(m, ActorCriticMLP)
    assert m.n_params == 4675
    shapes = [w.shape for w in m.get_weights()]
    assert shapes == [(4, 64), (64,), (64, 64), (64,), (64, 2), (2,), (64, 1), (1,)]
    w = m.get_weights()
    # Keras Orthogonal(gain): columns orthogonal with norm = gain
    W2 = w[2].astype(np.float64)
    np.testing.assert_allclose(W2.T @ W2, 2.0 * np.eye(64), atol=1e-4)
    assert np.all(w[1] == 0) and np.all(w[7] == 0)
    m2 = create_model(_env(), 'ppo', 'model', seed=55, device='cpu')
    np.testing.assert_array_equal(m2.theta.numpy(), m.theta.numpy())


def test_model_reader_output_units_rules(tmp_path):
    from xagents_amd.nets import ModelReader

    cfg = tmp_path / 'cnn.cfg'
    cfg.write_text('[convolutional-0]\nfilters=32\nsize=8\nstride=4\nactivation=relu\n\n'
                   '[convolutional-1]\nfilters=64\nsize=4\nstride=2\nactivation=relu\n\n'
                   '[convolutional-2]\nfilters=64\nsize=3\nstride=1\nactivation=relu\n\n'
                   '[flatten-0]\n\n[dense-0]\nunits=512\nactivation=relu\n\n[dense-1]\noutput=1\n')
    m = ModelReader(str(cfg), [6], (84, 84, 1), None, seed=1, device='cpu').build_model()
    # Conv1D on (84,84,1) convolves along width only
    assert [l.out_shape for l in m.layers] == [(84, 20, 32), (84, 9, 64), (84, 7, 64), (37632,),
                                               (512,), (6,)]
    assert m.n_params == 288 + 8256 + 12352 + 19_268_096 + 3078
    with pytest.raises(AssertionError, match='Output units given are less'):
        ModelReader(str(cfg), [], (84, 84, 1), None, device='cpu').build_model()


# ---- C ABI -------------------------------------------------------------------
def test_library_exports_every_header_symbol():
    from xagents_amd import _lib

    header = (ROOT / 'include' / 'xagents_hip.h').read_text()
    declared = set(re.findall(r'^\s*(?:int|size_t|const char\*)\s+(xa_\w+)\(', header, re.M))
    assert declared and declared == set(_lib.EXPORTED_SYMBOLS)
    lib = _lib.load()  # no compute calls without a GPU
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.xa_abi_version() == 2
    assert lib.xa_mlp_param_count(4, 2) == 4675 == oracle.lib().xo_mlp_param_count(4, 2)
    assert lib.xa_ac_grad_blocks(8192) == 256 and lib.xa_ac_grad_blocks(100) == 4
    assert lib.xa_ppo_adv_stats_size(32768, 8192, 4) == 2 * 4 * 4 * 8


def test_library_is_built_from_this_tree(monkeypatch):
    """The library carries the hash of the sources it was built from; the loader refuses a
    stale one (a build from other sources) with a message, never a silent mismatch."""
    from xagents_amd import _build, _lib
    assert _build.library_hash() == _build.source_hash()
    assert _lib.load().xa_build_hash().decode() == _build.source_hash()
    monkeypatch.setattr(_lib, '_lib', None)
    monkeypatch.setattr(_build, 'source_hash', lambda: '0' * 16)
    with pytest.raises(_lib.HipLibraryError, match='stale'):
        _lib.load()


def test_product_never_imports_oracle():
    for p in (ROOT / 'xagents_amd').rglob('*.py'):
        src = p.read_text()
        assert 'import oracle' not in src and 'from oracle' not in src, p


# ---- env semantics of the rollout vs the reference step_envs ------------------
def test_replay_rollout_env_semantics_match_reference_step_envs(golden):
    """Pre-reset obs feed the policy, post-reset obs are carried, rewards/dones and
    the finished-episode returns follow BaseAgent.step_envs (xagents/base.py:388-426)."""
    g = golden('step_envs.npz')
    n, T = g['s0'].shape[0], g['new_states'].shape[0]
    rng = np.random.default_rng(0)
    theta = (rng.standard_normal(4675) * 0.1).astype(np.float32)
    env = dict(kind=0, state=g['s0'].copy(), done=np.zeros(n, np.float32),
               cursor=np.zeros(n, np.int32), ep_return=np.zeros(n, np.float32),
               rep_obs=g['rep_obs'], rep_state=g['rep_state'], rep_rew=g['rep_rew'],
               rep_done=g['rep_done'])
    out = oracle.mlp_rollout(theta, 2, env, T, uniforms=rng.random((n, T), dtype=np.float32))
    # policy input of step t+1 == new_states returned by step t
    np.testing.assert_array_equal(out['obs'][:, 1:].transpose(1, 0, 2), g['new_states'][:-1])
    np.testing.assert_array_equal(out['obs'][:, 0], g['s0'])
    np.testing.assert_array_equal(out['rew'].T, g['rewards'])
    np.testing.assert_array_equal(out['done'][:, 1:].T, g['dones'])
    np.testing.assert_array_equal(env['state'], g['post_states'][-1])
    d = out['done'][:, 1:]
    t_idx, e_idx = np.nonzero(d.T)
    np.testing.assert_array_equal(out['epret'][e_idx, t_idx], g['total_rewards'])
    np.testing.assert_array_equal(env['ep_return'], g['episode_rewards'].astype(np.float32))


def test_replay_record_is_consistent():
    from xagents_amd.envs import record_cartpole_replay

    s0, obs, post, rew, done = record_cartpole_replay(8, 300, seed=55)
    assert done[:, -1].all() and np.array_equal(post[:, -1], s0)
    nd = done[:, :-1] == 0
    np.testing.assert_array_equal(obs[:, :-1][nd], post[:, :-1][nd])
    assert np.all(np.abs(post[:, :-1][done[:, :-1] == 1]) <= 0.05)
    assert 0.01 < done.mean() < 0.2 and np.all(rew == 1)


def test_rb2_batched_randint_matches_per_buffer_calls():
    """DeviceReplay.sample_slots draws all RB2 indices in one randint call when every
    buffer has the same size: legacy numpy yields exactly the values of the reference's
    per-buffer np.random.randint(0, size, k) calls in env order (buffers.py:137-148)."""
    for size, n, k in ((5, 64, 2), (31250, 32, 2), (1000, 7, 3), (2 ** 20 + 7, 4, 1)):
        np.random.seed(11)
        ref = np.concatenate([np.random.randint(0, size, k) for _ in range(n)])
        np.random.seed(11)
        got = np.random.randint(0, size, n * k)
        np.testing.assert_array_equal(ref, got)


def test_rb1_fast_sampler_matches_random_sample():
    """DeviceReplay's RB1 draw (replay._sample_ranges through getrandbits) returns exactly the
    reference's per-buffer random.sample(range(length), k) results (buffers.py:96-104) and
    leaves the module RNG in the same state, across the pool (n <= 21) and set branches."""
    from xagents_amd.replay import DeviceReplay, _fast_sampler
    fast = _fast_sampler()
    assert fast is not None
    cases = [[0], [2, 3, 21, 22], [5, 30, 100], [31250] * 32, [1, 2, 3, 4, 1000],
             list(range(6, 60, 7))]
    for lengths in cases:
        for k in (0, 1, 2, 3, 6, 10):
            if k > min(lengths):
                continue
            random.seed(sum(lengths) + k)
            ref = [q for n in lengths for q in random.sample(range(n), k)]
            after_ref = random.random()
            random.seed(sum(lengths) + k)
            got = fast(lengths, k)
            assert got == ref and random.random() == after_ref, (lengths, k)
    # the ring slots of a full and a wrapped deque (start + pos) % size, env-major
    rep = DeviceReplay.__new__(DeviceReplay)
    rep.kind, rep.n, rep.cap, rep.k = XA_RING_DEQUE, 3, 50, 2
    rep.host_count = np.array([7, 50, 133], np.int64)
    random.seed(5)
    want = []
    for i, cnt in enumerate(rep.host_count.tolist()):
        length = min(cnt, 50)
        want += [i * 50 + (cnt - length + p) % 50 for p in random.sample(range(length), 2)]
    random.seed(5)
    np.testing.assert_array_equal(rep.sample_slots(), want)


# ---- LazyFrames and the per-env states view (xagents/utils/common.py:23-64) --------------
def test_lazyframes_and_states_view():
    import torch
    from xagents_amd.utils.common import DeviceStates, LazyFrames
    frames = np.arange(84 * 84, dtype=np.uint8).reshape(84, 84, 1)
    lf = LazyFrames(frames)
    assert lf.dtype == np.uint8 and lf.shape == (84, 84, 1)
    np.testing.assert_array_equal(np.asarray(lf), frames)
    assert lf.frames is None  # materialised once
    assert len(lf) == 84 and lf.count() == 1
    np.testing.assert_array_equal(lf[3], frames[3])
    assert np.asarray(lf, dtype=np.float32).dtype == np.float32
    images = torch.from_numpy(np.stack([frames, frames + 1]))
    view = DeviceStates(images)
    assert len(view) == 2 and isinstance(view[1], LazyFrames)
    np.testing.assert_array_equal(np.asarray(view[1]), frames + 1)
    np.testing.assert_array_equal(np.asarray(view), images.numpy())
    vec = DeviceStates(torch.zeros(3, 4))
    assert isinstance(vec[0], np.ndarray) and vec[0].shape == (4,)
    assert [s.shape for s in vec] == [(4,)] * 3


def test_fill_buffers_draws_actions_env_by_env():
    """OffPolicy.fill_buffers draws env 0's random actions first, then env 1's
    (xagents/base.py:702-730)."""
    from types import SimpleNamespace
    from xagents_amd.base import OffPolicy
    from xagents_amd.envs import Discrete
    from xagents_amd.utils.buffers import ReplayBuffer2
    space = Discrete(6)
    space.seed(3)
    bufs = [ReplayBuffer2(10, 5, initial_size=4, batch_size=2) for _ in range(3)]
    bufs[1].current_size = 1  # env 1 needs only 3 more
    stub = SimpleNamespace(envs=[SimpleNamespace(action_space=space)], buffers=bufs, n_envs=3)
    plan, need = OffPolicy._fill_action_plan(stub)
    assert need == [4, 3, 4] and plan.shape == (4, 3)
    ref = Discrete(6)
    ref.seed(3)
    draws = [int(ref.sample()) for _ in range(11)]
    assert list(plan[:, 0]) == draws[0:4]
    assert list(plan[:3, 1]) == draws[4:7]
    assert list(plan[:, 2]) == draws[7:11]


def test_ctypes_structs_match_the_c_abi(tmp_path):
    """Every argument struct the ctypes binding mirrors has the C header's size and field
    offsets (gcc on include/xagents_hip.h): a drifted mirror would hand kernels shifted
    pointers."""
    import ctypes
    import shutil
    import subprocess
    from xagents_amd import _lib
    if shutil.which('gcc') is None:
        pytest.skip('gcc not available')
    structs = [v for k, v in vars(_lib).items() if k.startswith('Xa') and isinstance(v, type)
               and issubclass(v, ctypes.Structure)]
    assert len(structs) >= 10
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "xagents_hip.h"',
             'int main(void) {']
    for s in structs:
        lines.append(f'  printf("{s.__name__} size %zu\\n", sizeof({s.__name__}));')
        for f in s._fields_:
            lines.append(f'  printf("{s.__name__} {f[0]} %zu\\n", offsetof({s.__name__}, {f[0]}));')
    lines += ['  return 0;', '}']
    src = tmp_path / 'abi.c'
    src.write_text('\n'.join(lines) + '\n')
    exe = tmp_path / 'abi'
    subprocess.run(['gcc', '-std=c11', '-I', str(ROOT / 'include'), str(src), '-o', str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = {}
    for line in out.splitlines():
        name, field, val = line.split()
        got[(name, field)] = int(val)
    for s in structs:
        assert got[(s.__name__, 'size')] == ctypes.sizeof(s), s.__name__
        for f in s._fields_:
            assert got[(s.__name__, f[0])] == getattr(s, f[0]).offset, (s.__name__, f[0])


def test_fused_td3_entry_points_validate_sizes():
    """xa_td3_update / xa_td3_act refuse shapes beyond their tiles with a message (checked
    before any device call, so this runs without a GPU), and size their workspaces on the
    host (control words, activations, head partials, tickets grow with the batch)."""
    import ctypes
    from xagents_amd import _lib
    lib = _lib.load()
    a = _lib.XaTd3ActArgs()
    a.n, a.obs_dim, a.act_dim, a.h1, a.h2, a.ld_out = 64, 24, 5, 400, 300, 5
    assert lib.xa_td3_act(ctypes.byref(a), None) != 0
    assert b'act <= 4' in lib.xa_last_error()
    a.act_dim, a.ld_out, a.h1 = 4, 4, 402
    assert lib.xa_td3_act(ctypes.byref(a), None) != 0
    assert b'multiples of 4' in lib.xa_last_error()
    a.h1 = 400
    assert lib.xa_td3_act(ctypes.byref(a), None) != 0  # no buffers
    assert b'missing buffers' in lib.xa_last_error()
    u = _lib.XaTd3UpdateArgs()
    u.batch, u.obs_dim, u.act_dim, u.h1, u.h2 = 300, 24, 4, 400, 300
    assert lib.xa_td3_update(ctypes.byref(u), None) != 0
    assert b'batch <= 256' in lib.xa_last_error()
    w64 = lib.xa_td3_update_workspace_bytes(64, 24, 4, 400, 300)
    w128 = lib.xa_td3_update_workspace_bytes(128, 24, 4, 400, 300)
    assert 0 < w64 < w128
    assert lib.xa_td3_act_workspace_bytes(64, 24, 4, 400, 300) == w64
