"""AtariWrapper restatement (oracle/atari_oracle.py) known answers and the host-side
cv::resize tables of xagents_amd/atari.py (CPU). Parity against cv2 itself is unpinned
(no cv2 / gym here); these pin the restatement by cases whose answer is forced."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / 'oracle'))
import atari_oracle as AO  # noqa: E402


def test_gray_known_answers():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0],
                    [10, 20, 30]]], np.uint8)
    g = AO.bgr2gray(px)[0]
    # (c0 1868 + c1 9617 + c2 4899 + 8192) >> 14, channel 0 read as blue
    assert list(g) == [29, 150, 76, 255, 0, (10 * 1868 + 20 * 9617 + 30 * 4899 + 8192) >> 14]


def test_resize_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (13, 17), dtype=np.uint8)
    np.testing.assert_array_equal(AO.resize_linear(img, 17, 13), img)
    for v in (0, 1, 128, 255):
        c = np.full((210, 160), v, np.uint8)
        np.testing.assert_array_equal(AO.resize_linear(c, 84, 84), np.full((84, 84), v))


def test_resize_halving_is_pair_mean():
    # scale 2: fx = 2 dx + 0.5 -> taps (2 dx, 2 dx + 1) with 1024 / 1024
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (8, 8), dtype=np.uint8).astype(np.int64)
    out = AO.resize_linear(img.astype(np.uint8), 4, 4).astype(np.int64)
    h = img[:, 0::2] * 1024 + img[:, 1::2] * 1024
    exp = (h[0::2] * 1024 + h[1::2] * 1024 + (1 << 21)) >> 22
    np.testing.assert_array_equal(out, exp)


@pytest.mark.parametrize('shape', [(210, 160, 84, 84), (210, 160, 50, 97), (20, 30, 40, 45),
                                   (7, 5, 3, 11)])
def test_host_tables_match_oracle(shape):
    """The product's cv::resize tables (atari.py) against the oracle's own restatement:
    equal tables make the kernel's integer path the oracle's."""
    from xagents_amd.atari import cv_resize_linear_tables
    H, W, oh, ow = shape
    xofs, alpha, yofs, beta = cv_resize_linear_tables(H, W, oh, ow)
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (H, W), dtype=np.uint8)
    # evaluate the kernel's formula from the tables on the host
    src = img.astype(np.int64)
    sx1 = np.minimum(xofs + 1, W - 1)
    r0 = np.clip(yofs, 0, H - 1)
    r1 = np.clip(yofs + 1, 0, H - 1)
    a0, a1 = alpha[0::2].astype(np.int64), alpha[1::2].astype(np.int64)
    b0, b1 = beta[0::2].astype(np.int64), beta[1::2].astype(np.int64)
    h0 = src[r0][:, xofs] * a0 + src[r0][:, sx1] * a1
    h1 = src[r1][:, xofs] * a0 + src[r1][:, sx1] * a1
    v = np.clip((h0 * b0[:, None] + h1 * b1[:, None] + (1 << 21)) >> 22, 0, 255)
    np.testing.assert_array_equal(v, AO.resize_linear(img, ow, oh))


def test_frame_skips_assertion():
    from xagents_amd.atari import AtariFrameVecEnv
    with pytest.raises(AssertionError, match='frame_skips must be >= 1'):
        AtariFrameVecEnv('PongNoFrameskip-v4', 2, frame_skips=1)
    with pytest.raises(AssertionError, match='frame_skips must be >= 1'):
        AO.AtariWrapperRef(None, frame_skips=1)


def test_oracle_wrapper_skip_and_max_semantics():
    """Scripted stream: rewards summed over the skipped frames, early stop at a done, the
    max over the last two raw frames, reset frame processed alone."""
    T, H, W = 12, 4, 4
    frames = np.zeros((1, T, H, W, 3), np.uint8)
    for t in range(T):
        frames[0, t] = t * 10
    rew = np.arange(T, dtype=np.float32)[None]
    done = np.zeros((1, T), np.float32)
    done[0, 6] = 1
    done[0, -1] = 1
    s0, out = AO.run_envs(frames, rew, done, 3, frame_skips=4, resize_shape=(W, H),
                          max_frame=True)
    g = lambda v: AO.bgr2gray(np.full((1, 1, 3), v, np.uint8))[0, 0]  # noqa: E731
    assert s0[0, 0, 0, 0] == g(0)
    # step 1: frames 1..4, reward 1+2+3+4, max(frame 3, frame 4) = frame 4
    assert out['rewards'][0, 0] == 10 and out['dones'][0, 0] == 0
    assert out['new_states'][0, 0, 0, 0, 0] == g(40)
    # step 2: frames 5, 6 (done) -> reward 11, terminal frame 6, reset frame 7 alone
    assert out['rewards'][1, 0] == 11 and out['dones'][1, 0] == 1
    assert out['new_states'][1, 0, 0, 0, 0] == g(60)
    assert out['states'][1, 0, 0, 0, 0] == g(70)
    # step 3: frames 8..11, 11 is terminal (wrap)
    assert out['rewards'][2, 0] == 8 + 9 + 10 + 11 and out['dones'][2, 0] == 1
