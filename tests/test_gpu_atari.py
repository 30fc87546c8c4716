"""GPU parity of xa_atari_step (AtariWrapper on device, xagents/utils/common.py:67-142)
against the pure-Python AtariWrapper restatement (oracle/atari_oracle.py): processed
frames, rewards and dones bit-exact; the reference's own shape test
(xagents/tests/test_common_utils.py:11-25) repeated on device. Parity vs cv2 itself is
unpinned (no cv2 here), see the oracle header."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('max_frame,resize_shape,skips', [
    (False, (84, 84), 4), (True, (84, 84), 4), (True, (50, 97), 3), (False, (61, 61), 2)])
def test_atari_step_matches_wrapper_restatement(device, max_frame, resize_shape, skips):
    sys.path.insert(0, str(ROOT / 'oracle'))
    import atari_oracle as AO
    from xagents_amd.atari import AtariFrameVecEnv, record_raw_frames
    n, t_raw, steps = 3, 23, 9
    raw = record_raw_frames(n, t_raw, seed=4, mean_episode=6, reward_prob=0.3)
    env = AtariFrameVecEnv('PongNoFrameskip-v4', n, frame_skips=skips,
                           resize_shape=resize_shape, max_frame=max_frame, device=device,
                           raw=raw)
    s0_ref, ref = AO.run_envs(*raw, steps, skips, resize_shape, max_frame)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(env.state.cpu().numpy().reshape(s0_ref.shape), s0_ref)
    for t in range(steps):
        env.pre_step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(
            env.rep_obs.cpu().numpy()[:, 0].reshape(ref['new_states'][t].shape),
            ref['new_states'][t], err_msg=f'step {t}: frame returned by step')
        np.testing.assert_array_equal(
            env.rep_state.cpu().numpy()[:, 0].reshape(ref['states'][t].shape),
            ref['states'][t], err_msg=f'step {t}: post-reset state')
        np.testing.assert_array_equal(env.rep_rew.cpu().numpy()[:, 0], ref['rewards'][t])
        np.testing.assert_array_equal(env.rep_done.cpu().numpy()[:, 0], ref['dones'][t])
    assert ref['dones'].any() and ref['rewards'].any()


@pytest.mark.parametrize('resize_shape', [[random.randint(50, 100)] * 2 for _ in range(3)])
def test_atari_wrapper_shapes(device, resize_shape):
    """xagents/tests/test_common_utils.py:11-25 on device."""
    from xagents_amd.envs import create_envs
    env = create_envs('PongNoFrameskip-v4', 2, True, resize_shape=resize_shape,
                      device=device, t_raw_frames=8)
    reset_state = env.reset()
    env.pre_step()
    state = env.rep_obs[:, 0]
    assert state.shape[1:] == reset_state.shape[1:] == (*resize_shape, 1)
    assert env.observation_space.shape == (*resize_shape, 1)


def test_dqn_replay_ring_holds_preprocessed_frames(device):
    """DQN over the device AtariWrapper: the replay ring receives exactly the frames the
    reference's step_envs would store (state before the step, pre-reset frame after)."""
    sys.path.insert(0, str(ROOT / 'oracle'))
    import atari_oracle as AO
    from xagents_amd import DQN
    from xagents_amd.atari import AtariFrameVecEnv, record_raw_frames
    from xagents_amd.utils.buffers import ReplayBuffer1
    from xagents_amd.utils.common import create_model
    n, steps = 2, 7
    raw = record_raw_frames(n, 19, seed=9, mean_episode=8)
    env = AtariFrameVecEnv('PongNoFrameskip-v4', n, max_frame=True, device=device, raw=raw)
    bufs = [ReplayBuffer1(16, batch_size=2) for _ in range(n)]
    model = create_model(env, 'dqn', 'model', seed=3, device=device)
    agent = DQN(env, model, bufs, seed=11, quiet=True)
    for t in range(steps):
        agent._env_step(torch.zeros(n, dtype=torch.int32, device=device))
    torch.cuda.synchronize()
    s0, ref = AO.run_envs(*raw, steps, 4, (84, 84), True)
    prev = np.concatenate([s0[None], ref['states'][:-1]])
    got_s = agent.replay.states.cpu().numpy()[:, :steps]
    got_ns = agent.replay.new_states.cpu().numpy()[:, :steps]
    np.testing.assert_array_equal(got_s, prev.transpose(1, 0, 2, 3, 4))
    np.testing.assert_array_equal(got_ns, ref['new_states'].transpose(1, 0, 2, 3, 4))
    np.testing.assert_array_equal(agent.replay.rewards.cpu().numpy()[:, :steps],
                                  ref['rewards'].T)
