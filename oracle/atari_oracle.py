"""TEST INFRASTRUCTURE ONLY -- oracle for xa_atari_step (xagents_amd/csrc/atari.hip).

Only tests/ may import this module; the product never does.

Pure-Python restatement of the reference's AtariWrapper (xagents/utils/common.py:67-142)
over a scripted raw-frame env, and of the two OpenCV calls it makes
(common.py:104-105), following OpenCV's published 8-bit fixed-point algorithms:
  * cv2.cvtColor(frame, cv2.COLOR_BGR2GRAY): RGB2Gray<uchar> (imgproc color_rgb):
    Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14 with channel 0 read as B;
  * cv2.resize(frame, (w, h)) (INTER_LINEAR): cv::resize's tables
    (fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx), x borders clamped with
    fx = 0, coefficients rounded to short at scale 2048), HResizeLinear (int sums) and
    VResizeLinear with FixedPtCast<int, uchar, 22> ((v + 2^21) >> 22, saturated).
Parity status: UNPINNED against cv2 / gym -- neither is installed here and the
reference's own test (xagents/tests/test_common_utils.py:11-25) checks only shapes,
which tests/test_atari.py repeats. OpenCV's SIMD vertical pass (VResizeLinearVec_32s8u)
rounds differently ((S >> 4) * b >> 16 sums, then (v + 2) >> 2) and may differ from this
scalar path by 1 on some pixels; this restatement follows the scalar reference path.
Known answers pin the restatement itself: identity resize, constant images, pure colours.
"""
import numpy as np


def bgr2gray(frame):
    """cv2.cvtColor(frame, cv2.COLOR_BGR2GRAY) for uint8 [H, W, 3]."""
    f = frame.astype(np.int64)
    return ((f[..., 0] * 1868 + f[..., 1] * 9617 + f[..., 2] * 4899 + (1 << 13)) >> 14).astype(
        np.uint8)


def _coef(fx):
    """(1 - fx, fx) in float32, times 2048, rounded half-to-even to short."""
    one = np.float32(1.0)
    c0 = np.float32(np.float32(one - fx) * np.float32(2048))
    c1 = np.float32(fx * np.float32(2048))
    return int(np.rint(c0)), int(np.rint(c1))


def resize_linear(img, out_w, out_h):
    """cv2.resize(img, (out_w, out_h)) for a uint8 [H, W] image, INTER_LINEAR."""
    H, W = img.shape
    scale_x = 1.0 / (out_w / W)
    scale_y = 1.0 / (out_h / H)
    src = img.astype(np.int64)
    out = np.zeros((out_h, out_w), np.uint8)
    xs = []
    for dx in range(out_w):
        fx = np.float32((dx + 0.5) * scale_x - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0.0), 0
        if sx >= W - 1:
            fx, sx = np.float32(0.0), W - 1
        xs.append((sx, *_coef(fx)))
    for dy in range(out_h):
        fy = np.float32((dy + 0.5) * scale_y - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        b0, b1 = _coef(fy)
        rows = [min(max(sy, 0), H - 1), min(max(sy + 1, 0), H - 1)]
        hs = []
        for r in rows:
            # HResizeLinear: sx + 1 is only read where its coefficient is non-zero
            hs.append([src[r, sx] * a0 + (src[r, sx + 1] * a1 if a1 else 0)
                       for sx, a0, a1 in xs])
        for dx in range(out_w):
            v = (hs[0][dx] * b0 + hs[1][dx] * b1 + (1 << 21)) >> 22
            out[dy, dx] = min(max(v, 0), 255)
    return out


def process_frame(frame, resize_shape):
    """AtariWrapper.process_frame (common.py:95-106) without the LazyFrames wrapper:
    [h, w, 1] uint8 for dsize = resize_shape = (w, h)."""
    g = bgr2gray(frame)
    return resize_linear(g, resize_shape[0], resize_shape[1])[..., None]


class RawStreamEnv:
    """Scripted gym env over one env's raw stream: reset() -> frames[cursor] (the reset
    frame), step() -> next frame with its reward / done; after a done, reset() moves to the
    next frame (the reset frame)."""

    def __init__(self, frames, rew, done):
        self.frames, self.rew, self.done = frames, rew, done
        self.c = -1

    def reset(self):
        self.c = (self.c + 1) % len(self.frames)
        return self.frames[self.c]

    def step(self, action):
        self.c = (self.c + 1) % len(self.frames)
        return self.frames[self.c], float(self.rew[self.c]), bool(self.done[self.c]), {}


class AtariWrapperRef:
    """AtariWrapper.step / reset (common.py:108-142) over a RawStreamEnv."""

    def __init__(self, env, frame_skips=4, resize_shape=(84, 84), max_frame=False):
        assert frame_skips > 1, 'frame_skips must be >= 1'
        self.env = env
        self.skips = frame_skips
        self.frame_shape = resize_shape
        self.max_frame = max_frame
        self.frame_buffer = []

    def _append(self, s):
        self.frame_buffer = (self.frame_buffer + [s])[-2:]  # deque(maxlen=2)

    def step(self, action):
        total_reward = 0
        state, done = None, None
        for _ in range(self.skips):
            state, reward, done, info = self.env.step(action)
            if self.max_frame:
                self._append(state)
                state = np.max(np.stack(self.frame_buffer), axis=0)
            total_reward += reward
            if done:
                break
        return process_frame(state, self.frame_shape), total_reward, done, {}

    def reset(self):
        state = self.env.reset()
        if self.max_frame:
            self.frame_buffer = []
            self._append(state)
        return process_frame(state, self.frame_shape)


def run_envs(frames, rew, done, n_steps, frame_skips=4, resize_shape=(84, 84),
             max_frame=False):
    """BaseAgent.step_envs bookkeeping (base.py:388-426) for n envs over n_steps: returns
    s0 [n, h, w, 1] and per step (new_states = pre-reset frame, states = post-reset frame,
    rewards, dones) stacked over steps."""
    envs = [AtariWrapperRef(RawStreamEnv(frames[i], rew[i], done[i]), frame_skips,
                            resize_shape, max_frame) for i in range(len(frames))]
    states = [e.reset() for e in envs]
    s0 = np.stack(states)
    out = {'new_states': [], 'states': [], 'rewards': [], 'dones': []}
    for _ in range(n_steps):
        ns, rs, ds = [], [], []
        for i, e in enumerate(envs):
            s, r, d, _ = e.step(0)
            ns.append(s)
            rs.append(r)
            ds.append(d)
            states[i] = e.reset() if d else s
        out['new_states'].append(np.stack(ns))
        out['states'].append(np.stack(states))
        out['rewards'].append(np.array(rs, np.float32))
        out['dones'].append(np.array(ds, np.float32))
    return s0, {k: np.stack(v) for k, v in out.items()}
