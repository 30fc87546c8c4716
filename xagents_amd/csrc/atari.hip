// AtariWrapper on device (xagents/utils/common.py:67-142): frame skip with reward sum and
// early stop on done, max over the last two raw frames (max_frame), cv2.cvtColor
// COLOR_BGR2GRAY and cv2.resize INTER_LINEAR to the (84, 84) training frame, written
// straight into the uint8 observation record the replay-ring env step consumes.
//
// Raw frames are a per-env stream [n_envs, t_raw, H, W, 3] u8 with per-frame reward and
// done: stepping into frame t yields raw_rew[t], raw_done[t]; the frame after a done frame
// is the env.reset() frame. raw_cursor[i] = the frame the env last emitted.
//
// Arithmetic is OpenCV's fixed-point 8-bit path, integer-exact:
//   gray  = (1868 c0 + 9617 c1 + 4899 c2 + 2^13) >> 14        (RGB2Gray<uchar>, yuv_shift 14)
//   h(r)  = g(r, sx) alpha0 + g(r, sx + 1) alpha1             (HResizeLinear, coef scale 2048)
//   out   = sat_u8((h(sy) beta0 + h(sy + 1) beta1 + 2^21) >> 22)  (VResizeLinear, FixedPtCast 22)
// with the xofs / alpha / yofs / beta tables computed on the host exactly as cv::resize
// does (float coefficients rounded to short). One thread per output pixel: the 2 x 2
// source taps x 3 channels x (1 or 2) frames are read straight from HBM (the whole raw
// frame is ~100 KB and the output 7 KB, so the kernel is a byte-moving one: no LDS).
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

XA_DEV int gray_at(const uint8_t* f, const uint8_t* p, int64_t off) {
  int c0 = f[off], c1 = f[off + 1], c2 = f[off + 2];
  if (p) {
    c0 = max(c0, (int)p[off]);
    c1 = max(c1, (int)p[off + 1]);
    c2 = max(c2, (int)p[off + 2]);
  }
  return (c0 * 1868 + c1 * 9617 + c2 * 4899 + (1 << 13)) >> 14;
}

XA_DEV int resize_px(const XaAtariStepArgs& a, const uint8_t* f, const uint8_t* p, int dy,
                     int dx) {
  const int W = a.width, H = a.height;
  const int sx = a.xofs[dx], sx1 = min(sx + 1, W - 1);
  const int a0 = a.alpha[2 * dx], a1 = a.alpha[2 * dx + 1];
  const int sy = a.yofs[dy];
  const int r0 = min(max(sy, 0), H - 1), r1 = min(max(sy + 1, 0), H - 1);
  const int b0 = a.beta[2 * dy], b1 = a.beta[2 * dy + 1];
  const int64_t o0 = (int64_t)r0 * W * 3, o1 = (int64_t)r1 * W * 3;
  const int h0 = gray_at(f, p, o0 + 3 * sx) * a0 + gray_at(f, p, o0 + 3 * sx1) * a1;
  const int h1 = gray_at(f, p, o1 + 3 * sx) * a0 + gray_at(f, p, o1 + 3 * sx1) * a1;
  const int v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
  return min(max(v, 0), 255);
}

// frame-skip walk from the cursor: final frame, whether it ended the episode, reward sum
XA_DEV int skip_walk(const XaAtariStepArgs& a, int i, int& done, float& rew) {
  int c = a.raw_cursor[i];
  done = 0;
  rew = 0.0f;
  const float* rr = a.raw_rew + (int64_t)i * a.t_raw;
  const float* rd = a.raw_done + (int64_t)i * a.t_raw;
  for (int k = 0; k < a.skips; ++k) {
    c = c + 1 < a.t_raw ? c + 1 : 0;
    rew = rew + rr[c];
    if (rd[c] != 0.0f) {
      done = 1;
      break;
    }
  }
  return c;
}

__global__ __launch_bounds__(256) void atari_frames_kernel(XaAtariStepArgs a) {
  const int i = blockIdx.y;
  const int npx = a.out_h * a.out_w;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= npx) return;
  const int dy = e / a.out_w, dx = e - dy * a.out_w;
  const int64_t fb = (int64_t)a.height * a.width * 3;
  const uint8_t* env_frames = a.frames + (int64_t)i * a.t_raw * fb;
  uint8_t* post = a.out_post + (int64_t)i * npx;
  if (a.reset_only) {
    post[e] = (uint8_t)resize_px(a, env_frames + (int64_t)a.raw_cursor[i] * fb, nullptr, dy, dx);
    return;
  }
  int done;
  float rew;
  const int c = skip_walk(a, i, done, rew);
  const int prev = c > 0 ? c - 1 : a.t_raw - 1;
  const uint8_t v = (uint8_t)resize_px(a, env_frames + (int64_t)c * fb,
                                       a.max_frame ? env_frames + (int64_t)prev * fb : nullptr,
                                       dy, dx);
  a.out_step[(int64_t)i * npx + e] = v;
  if (done) {
    // BaseAgent.step_envs resets a done env (base.py:420-424): AtariWrapper.reset clears
    // the max-frame buffer, so the reset frame is processed alone
    const int r = c + 1 < a.t_raw ? c + 1 : 0;
    post[e] = (uint8_t)resize_px(a, env_frames + (int64_t)r * fb, nullptr, dy, dx);
  } else {
    post[e] = v;
  }
}

// per-env scalars after every frame block has read the cursor
__global__ void atari_scalars_kernel(XaAtariStepArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_envs || a.reset_only) return;
  int done;
  float rew;
  const int c = skip_walk(a, i, done, rew);
  if (a.out_rew) a.out_rew[i] = rew;
  if (a.out_done) a.out_done[i] = (float)done;
  a.raw_cursor[i] = done ? (c + 1 < a.t_raw ? c + 1 : 0) : c;
}

}  // namespace

extern "C" int xa_atari_step(const XaAtariStepArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_atari_step: null args");
  const XaAtariStepArgs& a = *p;
  XA_CHECK_ARG(a.n_envs > 0 && a.t_raw > 1 && a.height > 0 && a.width > 0 && a.out_h > 0 &&
                   a.out_w > 0,
               "xa_atari_step: bad sizes");
  XA_CHECK_ARG(a.frames && a.raw_cursor && a.xofs && a.alpha && a.yofs && a.beta && a.out_post,
               "xa_atari_step: null pointer");
  XA_CHECK_ARG(a.reset_only || (a.raw_rew && a.raw_done && a.out_step && a.skips >= 1),
               "xa_atari_step: a step needs raw_rew, raw_done, out_step and skips >= 1");
  XA_CHECK_ARG((int64_t)a.out_h * a.out_w < (1 << 30), "xa_atari_step: output frame too large");
  hipStream_t s = (hipStream_t)stream;
  const int npx = a.out_h * a.out_w;
  hipLaunchKernelGGL(atari_frames_kernel, dim3((npx + 255) / 256, a.n_envs), dim3(256), 0, s, a);
  XA_CHECK_LAUNCH("xa_atari_step (frames)");
  if (!a.reset_only) {
    hipLaunchKernelGGL(atari_scalars_kernel, dim3((a.n_envs + 63) / 64), dim3(64), 0, s, a);
    XA_CHECK_LAUNCH("xa_atari_step (scalars)");
  }
  return 0;
}
