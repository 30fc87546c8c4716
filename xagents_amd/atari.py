"""AtariWrapper on device (xagents/utils/common.py:67-142).

The reference wraps every gym Atari env in `AtariWrapper`: `step` repeats the action
`frame_skips` times (reward summed, stop at done), optionally keeps the pixelwise max of
the last two raw frames (`max_frame`), and `process_frame` turns the 210 x 160 RGB frame
into a (84, 84, 1) uint8 frame with `cv2.cvtColor(COLOR_BGR2GRAY)` + `cv2.resize`
(INTER_LINEAR). Here the raw frames of all envs live in HBM and one `xa_atari_step`
launch (csrc/atari.hip) does the skip walk and the whole preprocessing for every env,
writing the processed frames into the one-step record that the replay-ring env step
(`xa_replay_env_step`) consumes -- so the preprocessed frame goes straight from the raw
frame to the agent's state / replay ring without touching the host.

No emulator exists in this image (gym / ALE are absent), so the raw frames are a
synthetic pre-recorded stream (`record_raw_frames`), like the other device envs.
"""
import ctypes

import numpy as np
import torch

from xagents_amd._lib import XaAtariStepArgs, call, stream
from xagents_amd.envs import Discrete, TransitionReplayVecEnv

INTER_RESIZE_COEF_BITS = 11
INTER_RESIZE_COEF_SCALE = 1 << INTER_RESIZE_COEF_BITS


def _round_short(v):
    """saturate_cast<short>(float): cvRound (round half to even) then clamp."""
    return int(np.clip(np.rint(np.float32(v)), -32768, 32767))


def cv_resize_linear_tables(src_h, src_w, out_h, out_w):
    """cv::resize's INTER_LINEAR index / coefficient tables for 8-bit images
    (imgproc/src/resize.cpp: fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx),
    borders clamped with fx = 0 on x; coefficients float -> short at scale 2048).
    Returns xofs [out_w] int32, alpha [2 out_w] int16, yofs [out_h] int32,
    beta [2 out_h] int16 (source row clamping happens when the rows are read)."""
    scale_x = 1.0 / (out_w / src_w)
    scale_y = 1.0 / (out_h / src_h)
    xofs = np.zeros(out_w, np.int32)
    alpha = np.zeros(2 * out_w, np.int16)
    for dx in range(out_w):
        fx = np.float32((dx + 0.5) * scale_x - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0.0), 0
        if sx >= src_w - 1:
            fx, sx = np.float32(0.0), src_w - 1
        xofs[dx] = sx
        alpha[2 * dx] = _round_short(np.float32(np.float32(1.0) - fx) * np.float32(2048))
        alpha[2 * dx + 1] = _round_short(fx * np.float32(2048))
    yofs = np.zeros(out_h, np.int32)
    beta = np.zeros(2 * out_h, np.int16)
    for dy in range(out_h):
        fy = np.float32((dy + 0.5) * scale_y - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        yofs[dy] = sy
        beta[2 * dy] = _round_short(np.float32(np.float32(1.0) - fy) * np.float32(2048))
        beta[2 * dy + 1] = _round_short(fy * np.float32(2048))
    return xofs, alpha, yofs, beta


def record_raw_frames(n_envs, t_raw, height=210, width=160, seed=55, mean_episode=800,
                      reward_prob=0.005):
    """Synthetic raw emulator stream per env: RGB uint8 frames i.i.d. uniform, Pong-like
    rewards in {-1, 0, 1}, episode ends ~ Geometric(1 / mean_episode) raw frames; the last
    frame is terminal so the cursor wrap lands on frame 0, a reset frame. Generated from
    np.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n_envs, t_raw, height, width, 3), dtype=np.uint8)
    done = (rng.random((n_envs, t_raw)) < 1.0 / mean_episode).astype(np.float32)
    done[:, -1] = 1.0
    u = rng.random((n_envs, t_raw))
    rew = np.where(u < reward_prob, 1.0, np.where(u > 1 - reward_prob, -1.0, 0.0))
    return frames, rew.astype(np.float32), done


class AtariFrameVecEnv(TransitionReplayVecEnv):
    """n Atari envs behind AtariWrapper, stepped on device.

    Constructor arguments follow AtariWrapper(env, frame_skips=4, resize_shape=(84, 84),
    max_frame=False) (common.py:72-95), including its assertion. The observation space is
    (*resize_shape, 1) as the reference declares it; frames are laid out as cv2.resize
    returns them for dsize = resize_shape, i.e. (resize_shape[1], resize_shape[0])."""

    def __init__(self, env_id, n_envs, n_actions=6, frame_skips=4, resize_shape=(84, 84),
                 max_frame=False, t_raw=64, seed=55, device=None, raw=None,
                 mean_episode=800):
        assert frame_skips > 1, 'frame_skips must be >= 1'
        self.skips = int(frame_skips)
        self.frame_shape = tuple(int(v) for v in resize_shape)
        self.max_frame = bool(max_frame)
        out_w, out_h = self.frame_shape
        obs_shape = (*self.frame_shape, 1)
        z = np.zeros((n_envs, 1) + obs_shape, np.uint8)
        record = (np.zeros((n_envs,) + obs_shape, np.uint8), z, z.copy(),
                  np.zeros((n_envs, 1), np.float32),
                  np.zeros((n_envs, 1), np.float32))
        frames, rew, done = raw if raw is not None else record_raw_frames(
            n_envs, t_raw, seed=seed, mean_episode=mean_episode)
        assert frames.shape[0] == n_envs and frames.shape[-1] == 3 and frames.ndim == 5
        self._raw_ready = False
        super().__init__(env_id, n_envs, obs_shape, Discrete(n_actions), np.uint8, seed=seed,
                         device=device, record=record)
        dev = self.device
        self.t_raw, self.raw_h, self.raw_w = frames.shape[1], frames.shape[2], frames.shape[3]
        self.raw_frames = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
        self.raw_rew = torch.from_numpy(np.ascontiguousarray(rew, np.float32)).to(dev)
        self.raw_done = torch.from_numpy(np.ascontiguousarray(done, np.float32)).to(dev)
        self.raw_cursor = torch.zeros(n_envs, dtype=torch.int32, device=dev)
        xofs, alpha, yofs, beta = cv_resize_linear_tables(self.raw_h, self.raw_w, out_h, out_w)
        self.tables = [torch.from_numpy(t).to(dev) for t in (xofs, alpha, yofs, beta)]
        self._args = XaAtariStepArgs()
        a = self._args
        a.n_envs, a.t_raw, a.height, a.width = n_envs, self.t_raw, self.raw_h, self.raw_w
        a.out_h, a.out_w = out_h, out_w
        a.frames, a.raw_rew = self.raw_frames.data_ptr(), self.raw_rew.data_ptr()
        a.raw_done, a.raw_cursor = self.raw_done.data_ptr(), self.raw_cursor.data_ptr()
        a.skips, a.max_frame = self.skips, int(self.max_frame)
        a.xofs, a.alpha, a.yofs, a.beta = (t.data_ptr() for t in self.tables)
        self._raw_ready = True
        self.reset()

    def reset(self):
        """AtariWrapper.reset for every env: raw cursor to each stream's first (reset)
        frame, processed alone into the state."""
        super().reset()
        if not self._raw_ready:
            return self.state
        self.raw_cursor.zero_()
        a = self._args
        a.reset_only = 1
        a.out_step, a.out_post, a.out_rew, a.out_done = None, self.state.data_ptr(), None, None
        call('xa_atari_step', ctypes.byref(a), stream())
        return self.state

    def pre_step(self, actions=None, act_ld=None):
        """AtariWrapper.step (frame skip + preprocessing) of every env into the one-step
        record that the following xa_replay_env_step consumes (the synthetic raw stream
        does not depend on the actions)."""
        a = self._args
        a.reset_only = 0
        a.out_step, a.out_post = self.rep_obs.data_ptr(), self.rep_state.data_ptr()
        a.out_rew, a.out_done = self.rep_rew.data_ptr(), self.rep_done.data_ptr()
        call('xa_atari_step', ctypes.byref(a), stream())
