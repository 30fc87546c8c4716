// BipedalWalker-v3 device stand-in: continuous-control dynamics with the real env's
// observation layout (24), action space (4 motor commands in [-1, 1]), reward formula and
// termination rules, stepped on device so the off-policy (TD3 / DDPG) and Gaussian
// on-policy agents train without host envs. Replaces gym's env.step / env.reset inside
// BaseAgent.step_envs (xagents/base.py:388-426, the gym call at base.py:408) for
// BipedalWalker ids; SURVEY.md section 8(f) rank 4 ("BipedalWalker stand-ins").
//
// Not Box2D: gym's BipedalWalker is a Box2D rigid-body simulation (contacts, joint motors,
// hilly terrain) that neither this image nor the reference ships. The stand-in keeps its
// interface and constants and replaces the physics by a planar kinematic walker on flat
// ground:
//   joints   hip / knee speeds follow the motor command (first order, speed-limited),
//            angles integrate them inside the gym joint limits
//   legs     two 2-link legs (LEG_H each) hang from the hull; the lowest foot carries the
//            hull (support height), a stance foot stays put, so moving it backwards in the
//            hull frame moves the hull forwards; out of contact the hull falls under gravity
//   hull     pitch driven by the hip motors' reaction, a restoring term and damping
//   lidar    10 rays fanned forward-down over the flat ground
//   reward   shaping = 130 x / SCALE - 5 |angle|; reward = shaping - previous shaping
//            - 0.00035 MOTORS_TORQUE sum |clip(a)|; -100 and done when the hull touches
//            the ground or x < 0; done at the terrain end or after 1600 steps (TimeLimit)
// Every step is f32 arithmetic in a fixed order with explicit fmaf and restated sin / cos,
// so the C oracle (oracle/xa_oracle.c xo_walker_step) reproduces it bit for bit.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr float kScale = 30.0f, kFps = 50.0f, kDt = 1.0f / 50.0f;
constexpr float kMotorsTorque = 80.0f, kSpeedHip = 4.0f, kSpeedKnee = 6.0f;
constexpr float kLegH = 34.0f / 30.0f, kHipDy = 0.2f, kHullHalfH = 0.25f;
constexpr float kLidarRange = 160.0f / 30.0f;
constexpr float kGravity = 10.0f, kMotorGain = 40.0f, kJointDamp = 2.0f;
constexpr float kReact = 2.0f, kRestore = 3.0f, kPitchDamp = 1.0f, kAirDrag = 0.5f;
constexpr float kTerrainStep = 14.0f / 30.0f;
constexpr float kTerrainEnd = (200.0f - 10.0f) * (14.0f / 30.0f);  // (LENGTH - GRASS) STEP
constexpr float kStartX = 20.0f * (14.0f / 30.0f) * 0.5f;          // STARTPAD STEP / 2
constexpr int kMaxSteps = 1600;
// cos(1.5 i / 10), i = 0..9, rounded to f32 (the lidar rays' angles from straight down)
__constant__ float kLidarCos[10] = {1.0f,        0.98877108f, 0.95533649f, 0.90044710f,
                                    0.82533561f, 0.73168887f, 0.62160997f, 0.49757105f,
                                    0.36235775f, 0.21901920f};

constexpr float kHipLo = -0.8f, kHipHi = 1.1f, kKneeLo = -1.6f, kKneeHi = -0.1f;

// sin / cos for |x| <= 2 pi: reduction to [-pi, pi], then the Taylor polynomials of degree
// 15 / 16 in Horner form (|error| < 1e-6 on [-pi, pi]); the oracle restates the same
// operations
XA_DEV float wk_reduce(float x) {
  const float k = rintf(x * 0.159154943f);
  return fmaf(-k, 6.28318548f, x);
}
XA_DEV float wk_sin(float x) {
  const float r = wk_reduce(x), r2 = r * r;
  float p = fmaf(r2, -7.6471637e-13f, 1.6059044e-10f);
  p = fmaf(r2, p, -2.5052108e-08f);
  p = fmaf(r2, p, 2.7557319e-06f);
  p = fmaf(r2, p, -1.9841270e-04f);
  p = fmaf(r2, p, 8.3333333e-03f);
  p = fmaf(r2, p, -1.6666667e-01f);
  p = fmaf(r2, p, 1.0f);
  return r * p;
}
XA_DEV float wk_cos(float x) {
  const float r = wk_reduce(x), r2 = r * r;
  float p = fmaf(r2, 4.7794773e-14f, -1.1470746e-11f);
  p = fmaf(r2, p, 2.0876757e-09f);
  p = fmaf(r2, p, -2.7557319e-07f);
  p = fmaf(r2, p, 2.4801587e-05f);
  p = fmaf(r2, p, -1.3888889e-03f);
  p = fmaf(r2, p, 4.1666667e-02f);
  p = fmaf(r2, p, -0.5f);
  return fmaf(r2, p, 1.0f);
}
XA_DEV float wk_clip(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

// per-env state [N][kWalkerState]: x, y, angle, vx, vy, omega, q[4], dq[4], prev shaping,
// steps; foot x of the previous step (hull frame) per leg
enum { S_X, S_Y, S_TH, S_VX, S_VY, S_W, S_Q, S_DQ = S_Q + 4, S_SHAPE = S_DQ + 4, S_STEPS,
       S_FX0, S_FX1, S_N };
static_assert(S_N == XA_WALKER_STATE, "state size");

struct Feet {
  float x[2], y[2];
};
// foot positions relative to the hull centre
XA_DEV Feet feet(const float* s) {
  Feet f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float a1 = s[S_TH] + s[S_Q + 2 * j];
    const float a2 = a1 + s[S_Q + 2 * j + 1];
    f.x[j] = fmaf(kLegH, wk_sin(a1), kLegH * wk_sin(a2));
    f.y[j] = (-kHipDy - kLegH * wk_cos(a1)) - kLegH * wk_cos(a2);
  }
  return f;
}

XA_DEV void observe(const float* s, const float (&contact)[2], float* o) {
  o[0] = s[S_TH];
  o[1] = 2.0f * s[S_W] / kFps;
  o[2] = 0.3f * s[S_VX] * (600.0f / kScale) / kFps;
  o[3] = 0.3f * s[S_VY] * (400.0f / kScale) / kFps;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    o[4 + 5 * j] = s[S_Q + 2 * j];
    o[5 + 5 * j] = s[S_DQ + 2 * j] / kSpeedHip;
    o[6 + 5 * j] = s[S_Q + 2 * j + 1] + 1.0f;
    o[7 + 5 * j] = s[S_DQ + 2 * j + 1] / kSpeedKnee;
    o[8 + 5 * j] = contact[j];
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) o[14 + i] = fminf(1.0f, s[S_Y] / (kLidarRange * kLidarCos[i]));
}

// BipedalWalker.reset: hull at the start pad standing on straight legs, a random initial
// push (INITIAL_RANDOM) drawn from Philox(env, episode; seed)
XA_DEV void reset(float* s, int env, int episode, uint64_t seed, float (&contact)[2]) {
  const xa_u4 r = xa_philox((uint32_t)env, (uint32_t)episode, 0x3a1cu, 0u, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
  for (int k = 0; k < S_N; ++k) s[k] = 0.0f;
  s[S_X] = kStartX;
  s[S_VX] = (xa_u01(r.x) * 2.0f - 1.0f) * 0.2f;
  s[S_Q + 1] = kKneeHi;
  s[S_Q + 3] = kKneeHi;
  const Feet f = feet(s);
  s[S_Y] = -fminf(f.y[0], f.y[1]);
  s[S_FX0] = f.x[0];
  s[S_FX1] = f.x[1];
  s[S_SHAPE] = 130.0f * s[S_X] / kScale;
  contact[0] = contact[1] = 1.0f;
}

__global__ __launch_bounds__(256) void walker_step_kernel(XaWalkerStepArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n_envs) return;
  float s[S_N];
#pragma unroll
  for (int k = 0; k < S_N; ++k) s[k] = a.state[(size_t)e * S_N + k];
  float contact[2];
  if (a.reset_only) {
    const int ep = a.episode[e];
    reset(s, e, ep, a.seed, contact);
    observe(s, contact, a.out_post + (size_t)e * XA_WALKER_OBS);
  } else {
    const float* act = a.actions + (size_t)e * a.act_ld;
    float u[4], cost = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u[i] = wk_clip(act[i], -1.0f, 1.0f);
      cost = cost + fabsf(u[i]);
    }
    // joints: motor-driven speeds, speed limits, angle limits
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool hip = (i & 1) == 0;
      const float vmax = hip ? kSpeedHip : kSpeedKnee;
      float dq = s[S_DQ + i];
      dq = dq + kDt * fmaf(kMotorGain, u[i], -kJointDamp * dq);
      dq = wk_clip(dq, -vmax, vmax);
      float q = fmaf(kDt, dq, s[S_Q + i]);
      const float lo = hip ? kHipLo : kKneeLo, hi = hip ? kHipHi : kKneeHi;
      if (q < lo || q > hi) dq = 0.0f;
      s[S_Q + i] = wk_clip(q, lo, hi);
      s[S_DQ + i] = dq;
    }
    // hull pitch: hip motor reaction, restoring torque, damping
    s[S_W] = s[S_W] + kDt * ((-kReact * (u[0] + u[2]) - kRestore * s[S_TH]) - kPitchDamp * s[S_W]);
    s[S_TH] = fmaf(kDt, s[S_W], s[S_TH]);
    // legs: support height and contacts; stance feet stay put
    const Feet f = feet(s);
    const float support = -fminf(f.y[0], f.y[1]);
    s[S_VY] = s[S_VY] - kGravity * kDt;
    float y = fmaf(kDt, s[S_VY], s[S_Y]);
    bool grounded = false;
    if (y <= support) {
      y = support;
      s[S_VY] = fmaxf(s[S_VY], 0.0f);
      grounded = true;
    }
    s[S_Y] = y;
    float push = 0.0f, n_st = 0.0f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      contact[j] = grounded && f.y[j] <= fminf(f.y[0], f.y[1]) + 0.02f ? 1.0f : 0.0f;
      if (contact[j] > 0.0f) {
        push = push - (f.x[j] - s[S_FX0 + j]);
        n_st = n_st + 1.0f;
      }
    }
    s[S_VX] = n_st > 0.0f ? push / (n_st * kDt) : s[S_VX] * (1.0f - kAirDrag * kDt);
    s[S_X] = fmaf(kDt, s[S_VX], s[S_X]);
    s[S_FX0] = f.x[0];
    s[S_FX1] = f.x[1];
    s[S_STEPS] = s[S_STEPS] + 1.0f;
    // reward and termination (bipedal_walker.py step)
    const float shaping = 130.0f * s[S_X] / kScale - 5.0f * fabsf(s[S_TH]);
    float reward = shaping - s[S_SHAPE];
    s[S_SHAPE] = shaping;
    reward = reward - 0.00035f * kMotorsTorque * cost;
    const bool game_over = s[S_Y] - kHullHalfH < 0.0f || fabsf(s[S_TH]) > 1.0f;
    bool done = false;
    if (game_over || s[S_X] < 0.0f) {
      reward = -100.0f;
      done = true;
    }
    if (s[S_X] > kTerrainEnd || s[S_STEPS] >= (float)kMaxSteps) done = true;
    observe(s, contact, a.out_obs + (size_t)e * XA_WALKER_OBS);
    a.out_rew[e] = reward;
    a.out_done[e] = done ? 1.0f : 0.0f;
    if (done) {
      const int ep = a.episode[e] + 1;
      a.episode[e] = ep;
      reset(s, e, ep, a.seed, contact);
    }
    observe(s, contact, a.out_post + (size_t)e * XA_WALKER_OBS);
  }
#pragma unroll
  for (int k = 0; k < S_N; ++k) a.state[(size_t)e * S_N + k] = s[k];
}

}  // namespace

extern "C" int xa_walker_step(const XaWalkerStepArgs* args, void* stream) {
  XA_CHECK_ARG(args != nullptr, "xa_walker_step: null args");
  const XaWalkerStepArgs& a = *args;
  XA_CHECK_ARG(a.n_envs > 0 && a.state && a.episode && a.out_post,
               "xa_walker_step: null state / episode / out_post or n_envs <= 0");
  XA_CHECK_ARG(a.reset_only || (a.actions && a.act_ld >= 4 && a.out_obs && a.out_rew &&
                                a.out_done),
               "xa_walker_step: a step needs actions (act_ld >= 4), out_obs, out_rew, out_done");
  hipLaunchKernelGGL(walker_step_kernel, dim3((a.n_envs + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, a);
  XA_CHECK_LAUNCH("xa_walker_step");
  return 0;
}
