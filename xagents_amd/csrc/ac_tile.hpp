// One 32-sample tile of the actor-critic MLP update: forward, PPO / A2C loss and
// backward into per-thread gradient accumulators, shared by the per-minibatch
// xa_ac_grad kernel (ac_update.hip) and the persistent whole-train-step PPO update
// (ppo_update.hip). Replaces PPO.update_gradients' forward / loss / tape.gradient
// (xagents/ppo/agent.py:96-134) and A2C.train_step's (xagents/a2c/agent.py:190-216).
//
// Tile schedule (256 threads = 4 waves, S = 32 samples):
//   H1 = tanh(X W1 + b1)                (VALU, K = obs)
//   Z2 = H1 W2                          (MFMA f32 16x16x4, K = 64)
//   heads + loss + dL/dz                (8 lanes per sample, xor shuffles)
//   dA2 = (dZ W34^T) * (1 - H2^2)       (VALU, K = A + 1)
//   dW2 += H1^T dA2 ; dH1 = dA2 W2^T    (MFMA f32 16x16x4, K = 32 / 64)
//   dW1 += X^T dA1                      (VALU, K = 32)
// MFMA operands are read from LDS as contiguous 16-byte rows: the K index lane
// group q feeds is remapped to a contiguous block (k = 16q + kk), which only
// reorders the f32 accumulation (tolerance-checked against float64).
//
// Parameter slices: thread t owns a 4x4 block of W2 (rows 4(t>>4).., cols 4(t&15)..)
// and RPT of the remaining parameters (index t + 256 q of the non-W2 list); the
// optimizer step runs on these slices and they fill the LDS weight tiles.
#pragma once
#include <math.h>
#include <stddef.h>

#include "../../include/xagents_hip.h"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace xa_ac {

constexpr int H = XA_MLP_HIDDEN;
constexpr int S = 32;    // samples per tile
constexpr int LDW = 68;  // LDS row stride of [*][64] tiles (16-B aligned, conflict-spreading)
constexpr int LDT = 36;  // LDS row stride of transposed [64][32] tiles

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Update-path math on the hardware transcendental units (v_exp_f32 / v_log_f32 /
// v_rcp_f32, about 1 ulp): the update's outputs are floating-point gradients checked
// against float64 with a tolerance, so it does not need the rollout's restated
// bit-exact sequences (xa_expf / xa_logf / xa_tanhf, whose integer action indices the C
// oracle must reproduce). tanh keeps xa_tanhf's rational form, with the division by a
// refined reciprocal.
XA_DEV float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
XA_DEV float flog(float x) { return __builtin_amdgcn_logf(x) * 0.693147180559945309f; }
XA_DEV float frcp(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  return fmaf(fmaf(-x, r, 1.0f), r, r);  // one Newton step
}
XA_DEV float ftanh(float x) {
  const float c = 7.90531110763549805f;
  const float xc = fminf(fmaxf(x, -c), c);
  const float x2 = xc * xc;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  p = xc * p;
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  return p * frcp(q);
}

// D = A B + C on a 16x16 tile, K = 4: lane l feeds A[l&15][k=l>>4], B[k=l>>4][l&15];
// D[row = 4*(l>>4) + r][col = l&15] lands in register r (exact f32 fma chain).
XA_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct Offs {
  int w1, b1, w2, b2, w3, b3, w4, b4, P;
};
__host__ __device__ constexpr Offs offs(int obs, int A) {
  Offs o{};
  o.w1 = 0;
  o.b1 = obs * H;
  o.w2 = o.b1 + H;
  o.b2 = o.w2 + H * H;
  o.w3 = o.b2 + H;
  o.b3 = o.w3 + H * A;
  o.w4 = o.b3 + A;
  o.b4 = o.w4 + H;
  o.P = o.b4 + 1;
  return o;
}

template <int OBS, int A>
struct Dims {
  static constexpr int AH = A + 1;            // logits + value head
  static constexpr int NSLOT = AH + 2 + OBS;  // per-feature partial sums combined at the end
  static constexpr int NREST = OBS * H + H + H + H * A + A + H + 1;  // parameters outside W2
  static constexpr int RPT = (NREST + 255) / 256;                    // of them per thread
};

// All LDS of a tile kernel in ONE object (16-B aligned rows first).
template <int OBS, int A>
struct TileLds {
  static constexpr int AH = Dims<OBS, A>::AH, NSLOT = Dims<OBS, A>::NSLOT;
  float sW2[H * LDW];   // [i][j]
  float sW2T[H * LDW];  // [j][k] = W2[k][j]
  float sH1[S * LDW];   // [s][i]
  float sH1T[H * LDT];  // [i][s]
  float sH2[S * LDW];   // [s][j]; then dA1 [s][i]
  float sdA2[S * LDW];  // [s][j]
  float sdA2T[H * LDT]; // [j][s]
  float sW1[OBS * H], sb1[H], sb2[H], sW34[H * AH], sb34[AH];
  float sX[S * OBS], sdZ[S * AH];
  float sAct[S], sOldLp[S], sOldV[S], sRet[S], sAdvIn[S];
  int sValid[S];
  float sRed[4 * H * NSLOT];
  float sLoss[4][4];
  double sNorm[4];
};

// per-thread gradient / loss accumulators of the tiles one block processes
template <int OBS, int A>
struct TileAcc {
  static constexpr int AH = A + 1;
  f32x4 gW2[4];
  float gW34[AH], gW1[OBS];
  float gb1, gb2, gb34;
  float l_pg, l_v, l_ent, l_cnt;
  XA_DEV void zero() {
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) gW2[jt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int a = 0; a < AH; ++a) gW34[a] = 0.0f;
#pragma unroll
    for (int k = 0; k < OBS; ++k) gW1[k] = 0.0f;
    gb1 = gb2 = gb34 = 0.0f;
    l_pg = l_v = l_ent = l_cnt = 0.0f;
  }
};

struct LossCfg {
  bool is_ppo, has_adv_in;
  float loss_scale, clip_norm, value_coef, entropy_coef, adv_eps;
  float adv_mean, adv_std;
  float adv_rstd;  // 1 / (adv_std + adv_eps), set with adv_std
};

// A thread's slice of the flat parameter vector (see the file comment).
template <int OBS, int A>
struct ParamSlice {
  static constexpr int RPT = Dims<OBS, A>::RPT, NREST = Dims<OBS, A>::NREST;
  int k0, j0;
  int ri[RPT];    // flat index of rest value q, -1 past the end
  int rdst[RPT];  // its float offset inside TileLds (the LDS weight tiles), -1 past the end
  XA_DEV void init(int tid) {
    typedef TileLds<OBS, A> T;
    constexpr int AH = A + 1;
    const Offs o = offs(OBS, A);
    k0 = 4 * (tid >> 4);
    j0 = 4 * (tid & 15);
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int r = tid + 256 * q;
      const int e = r < NREST ? (r < o.w2 ? r : r + H * H) : -1;
      ri[q] = e;
      int d = -1;
      if (e < 0) d = -1;
      else if (e < o.b1) d = (int)(offsetof(T, sW1) / 4) + e;
      else if (e < o.w2) d = (int)(offsetof(T, sb1) / 4) + (e - o.b1);
      else if (e < o.w3) d = (int)(offsetof(T, sb2) / 4) + (e - o.b2);
      else if (e < o.b3) {
        const int jj = (e - o.w3) / A, a = (e - o.w3) - jj * A;
        d = (int)(offsetof(T, sW34) / 4) + jj * AH + a;
      } else if (e < o.w4) d = (int)(offsetof(T, sb34) / 4) + (e - o.b3);
      else if (e < o.b4) d = (int)(offsetof(T, sW34) / 4) + (e - o.w4) * AH + A;
      else d = (int)(offsetof(T, sb34) / 4) + A;
      rdst[q] = d;
    }
  }
  XA_DEV size_t w2_off(int rr) const { return (size_t)offs(OBS, A).w2 + (k0 + rr) * H + j0; }
  // 16 W2 values (4 rows of float4) + RPT rest values of a flat [P] vector
  XA_DEV void load(const float* base, float (&w)[16], float (&r)[RPT]) const {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const float4 t4 = *reinterpret_cast<const float4*>(&base[w2_off(rr)]);
      w[4 * rr] = t4.x; w[4 * rr + 1] = t4.y; w[4 * rr + 2] = t4.z; w[4 * rr + 3] = t4.w;
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) r[q] = base[ri[q] >= 0 ? ri[q] : 0];
  }
  XA_DEV void store(float* base, const float (&w)[16], const float (&r)[RPT]) const {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      *reinterpret_cast<float4*>(&base[w2_off(rr)]) =
          make_float4(w[4 * rr], w[4 * rr + 1], w[4 * rr + 2], w[4 * rr + 3]);
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (ri[q] >= 0) base[ri[q]] = r[q];
  }
  // the slice into the LDS weight tiles (W2 and its transpose, W1, biases, heads)
  XA_DEV void to_lds(TileLds<OBS, A>& L, const float (&w)[16], const float (&r)[RPT]) const {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      *reinterpret_cast<float4*>(&L.sW2[(k0 + rr) * LDW + j0]) =
          make_float4(w[4 * rr], w[4 * rr + 1], w[4 * rr + 2], w[4 * rr + 3]);
      *reinterpret_cast<float4*>(&L.sW2T[(j0 + rr) * LDW + k0]) =
          make_float4(w[rr], w[4 + rr], w[8 + rr], w[12 + rr]);
    }
    // the rest values through their precomputed LDS offsets (no per-lane range branches)
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (rdst[q] >= 0) reinterpret_cast<float*>(&L)[rdst[q]] = r[q];
  }
};

// Forward + loss + backward of the tile staged in L.sX / sAct / sRet / sOldV / sOldLp /
// sAdvIn / sValid (the caller's barrier made them visible). Ends after the dW1 phase
// (no trailing barrier).
struct NoStamp {
  XA_DEV void operator()(int) const {}
};

// Where a tile's per-sample inputs come from: the TileLds staging arrays, or packed LDS
// records {obs[OBS], action (< 0: padding, obs zero), return, old value, old log-prob}.
template <int OBS, int A>
struct StagedIn {
  const TileLds<OBS, A>& L;
  XA_DEV float x(int s, int k) const { return L.sX[s * OBS + k]; }
  XA_DEV bool valid(int s) const { return L.sValid[s] != 0; }
  XA_DEV float act(int s) const { return L.sAct[s]; }
  XA_DEV float ret(int s) const { return L.sRet[s]; }
  XA_DEV float oldv(int s) const { return L.sOldV[s]; }
  XA_DEV float oldlp(int s) const { return L.sOldLp[s]; }
  XA_DEV float advin(int s) const { return L.sAdvIn[s]; }
};
template <int OBS>
struct PackedIn {
  static constexpr int R = OBS + 4;
  const float* rec;  // [S][R]
  XA_DEV float x(int s, int k) const { return rec[s * R + k]; }
  XA_DEV bool valid(int s) const { return rec[s * R + OBS] >= 0.0f; }
  XA_DEV float act(int s) const { return rec[s * R + OBS]; }
  XA_DEV float ret(int s) const { return rec[s * R + OBS + 1]; }
  XA_DEV float oldv(int s) const { return rec[s * R + OBS + 2]; }
  XA_DEV float oldlp(int s) const { return rec[s * R + OBS + 3]; }
  XA_DEV float advin(int) const { return 0.0f; }
};

// Forward + loss + backward; stamp(slot) marks the phase ends (diagnostic builds).
// TS = samples per tile: S (32), or 16 for small minibatches, where more blocks with half
// the element-wise work each shorten the latency-bound step (the persistent update).
template <int OBS, int A, class Stamp, class In, int TS = S>
XA_DEV void tile_compute(TileLds<OBS, A>& L, TileAcc<OBS, A>& acc, const LossCfg& cfg,
                         Stamp stamp, const In& in);

template <int OBS, int A, class Stamp = NoStamp>
XA_DEV void tile_compute(TileLds<OBS, A>& L, TileAcc<OBS, A>& acc, const LossCfg& cfg,
                         Stamp stamp = Stamp()) {
  tile_compute<OBS, A>(L, acc, cfg, stamp, StagedIn<OBS, A>{L});
}

template <int OBS, int A, class Stamp, class In, int TS>
XA_DEV void tile_compute(TileLds<OBS, A>& L, TileAcc<OBS, A>& acc, const LossCfg& cfg,
                         Stamp stamp, const In& in) {
  static_assert(TS == 16 || TS == 32, "tile sizes: 16 or 32 samples");
  constexpr int AH = A + 1;
  constexpr int SPW = TS / 4;  // samples per wave in the element-wise phases
  constexpr int KQ = TS / 4;   // dW2: samples per MFMA lane group (K = TS)
  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;      // MFMA lane coordinates
  const int f = tid & 63, c8 = (tid >> 6) * SPW;  // element-wise phases: feature, sample chunk
  // ---- H1 = tanh(X W1 + b1): feature f, samples c8..c8+SPW-1 ----
  {
    float hv[SPW];
#pragma unroll
    for (int ss = 0; ss < SPW; ++ss) {
      const int s = c8 + ss;
      float z = 0.0f;
#pragma unroll
      for (int k = 0; k < OBS; ++k) z = fmaf(in.x(s, k), L.sW1[k * H + f], z);
      hv[ss] = ftanh(z + L.sb1[f]);
      L.sH1[s * LDW + f] = hv[ss];
    }
#pragma unroll
    for (int q = 0; q < SPW / 4; ++q)
      *reinterpret_cast<float4*>(&L.sH1T[f * LDT + c8 + 4 * q]) =
          make_float4(hv[4 * q], hv[4 * q + 1], hv[4 * q + 2], hv[4 * q + 3]);
  }
  __syncthreads();
  stamp(50);
  // ---- Z2 = H1 W2 (MFMA): wave w owns hidden columns 16w..16w+15 ----
  {
    float bv[16];
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) {
      const float4 t4 = *reinterpret_cast<const float4*>(&L.sW2T[(16 * w + li) * LDW + 16 * lq + 4 * v4]);
      bv[4 * v4] = t4.x; bv[4 * v4 + 1] = t4.y; bv[4 * v4 + 2] = t4.z; bv[4 * v4 + 3] = t4.w;
    }
    const float bias = L.sb2[16 * w + li];
#pragma unroll
    for (int st = 0; st < TS / 16; ++st) {
      float av[16];
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const float4 t4 = *reinterpret_cast<const float4*>(&L.sH1[(16 * st + li) * LDW + 16 * lq + 4 * v4]);
        av[4 * v4] = t4.x; av[4 * v4 + 1] = t4.y; av[4 * v4 + 2] = t4.z; av[4 * v4 + 3] = t4.w;
      }
      f32x4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) d = mfma4(av[kk], bv[kk], d);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        L.sH2[(16 * st + 4 * lq + r) * LDW + 16 * w + li] = ftanh(d[r] + bias);
    }
  }
  __syncthreads();
  stamp(51);
  // ---- heads + loss + dL/dz: 8 lanes per sample (threads past TS x 8 idle) ----
  if (tid < TS * 8) {
    const int s = tid >> 3, pp = tid & 7;
    float z[AH];
#pragma unroll
    for (int a = 0; a < AH; ++a) z[a] = 0.0f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = 8 * pp + jj;
      const float hj = L.sH2[s * LDW + j];
#pragma unroll
      for (int a = 0; a < AH; ++a) z[a] = fmaf(hj, L.sW34[j * AH + a], z[a]);
    }
#pragma unroll
    for (int a = 0; a < AH; ++a) z[a] = xa_sum8(z[a]) + L.sb34[a];
    if (pp == 0) {
      float dz[AH];
#pragma unroll
      for (int a = 0; a < AH; ++a) dz[a] = 0.0f;
      if (in.valid(s)) {
        const int act = (int)in.act(s);
        float m = z[0];
#pragma unroll
        for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
        float e[A], ssum = 0.0f;
#pragma unroll
        for (int a = 0; a < A; ++a) {
          e[a] = fexp(z[a] - m);
          ssum = ssum + e[a];
        }
        const float ls = flog(ssum), rs = frcp(ssum);
        float lp[A], pr[A], ent = 0.0f, logp = 0.0f;
#pragma unroll
        for (int a = 0; a < A; ++a) {
          lp[a] = (z[a] - m) - ls;
          pr[a] = e[a] * rs;
          ent = ent - pr[a] * lp[a];
          if (a == act) logp = lp[a];
        }
        const float v = z[A];
        const float R = in.ret(s);
        const float oldv = in.oldv(s);
        const float adv_raw = R - oldv;
        const float sc = cfg.loss_scale;
        float dlogp, dv, pg, vl;
        if (cfg.is_ppo) {
          const float adv =
              cfg.has_adv_in ? in.advin(s) : (adv_raw - cfg.adv_mean) * cfg.adv_rstd;
          const float ratio = fexp(logp - in.oldlp(s));
          const float c = cfg.clip_norm;
          const float pg1 = -adv * ratio;
          const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
          pg = fmaxf(pg1, pg2);
          // tf.maximum routes the gradient to its first input when x >= y; the
          // second input's gradient passes tf.clip_by_value only inside [lo, hi]
          const bool r_in = ratio >= 1.0f - c && ratio <= 1.0f + c;
          dlogp = (pg1 >= pg2 || r_in) ? (sc * -adv) * ratio : 0.0f;
          const float dvo = v - oldv;
          const float vclip = oldv + fminf(fmaxf(dvo, -c), c);
          const float vl1 = (v - R) * (v - R);
          const float vl2 = (vclip - R) * (vclip - R);
          vl = fmaxf(vl1, vl2);
          // rounding can make oldv + (v - oldv) != v inside the clip range: the
          // clipped branch then still carries the gradient 2 (v_clip - R)
          const float kv = sc * cfg.value_coef * 0.5f * 2.0f;
          if (vl1 >= vl2) dv = kv * (v - R);
          else dv = (dvo >= -c && dvo <= c) ? kv * (vclip - R) : 0.0f;
        } else {
          pg = -(adv_raw * logp);
          dlogp = -sc * adv_raw;
          vl = (v - R) * (v - R);
          dv = sc * cfg.value_coef * 2.0f * (v - R);
        }
        const float ec = sc * cfg.entropy_coef;
#pragma unroll
        for (int a = 0; a < A; ++a)
          dz[a] = dlogp * ((a == act ? 1.0f : 0.0f) - pr[a]) + ec * pr[a] * (lp[a] + ent);
        dz[A] = dv;
        acc.l_pg += pg;
        acc.l_v += vl;
        acc.l_ent += ent;
        acc.l_cnt += 1.0f;
      }
#pragma unroll
      for (int a = 0; a < AH; ++a) L.sdZ[s * AH + a] = dz[a];
    }
  }
  __syncthreads();
  stamp(52);
  // ---- dA2 = (dZ W34^T) * (1 - H2^2); head / b2 partial grads ----
  {
    float dv8[SPW];
#pragma unroll
    for (int ss = 0; ss < SPW; ++ss) {
      const int s = c8 + ss;
      float dh = 0.0f;
#pragma unroll
      for (int a = 0; a < AH; ++a) dh = fmaf(L.sdZ[s * AH + a], L.sW34[f * AH + a], dh);
      const float hv = L.sH2[s * LDW + f];
#pragma unroll
      for (int a = 0; a < AH; ++a) acc.gW34[a] = fmaf(hv, L.sdZ[s * AH + a], acc.gW34[a]);
      const float d = dh * (1.0f - hv * hv);
      acc.gb2 = acc.gb2 + d;
      L.sdA2[s * LDW + f] = d;
      dv8[ss] = d;
    }
#pragma unroll
    for (int q = 0; q < SPW / 4; ++q)
      *reinterpret_cast<float4*>(&L.sdA2T[f * LDT + c8 + 4 * q]) =
          make_float4(dv8[4 * q], dv8[4 * q + 1], dv8[4 * q + 2], dv8[4 * q + 3]);
    if (tid < AH) {
      float t = acc.gb34;
      for (int s = 0; s < TS; ++s) t = t + L.sdZ[s * AH + tid];
      acc.gb34 = t;
    }
  }
  __syncthreads();
  stamp(53);
  // ---- dW2 += H1^T dA2 (rows 16w.., K = samples KQ q + kk) and dH1 = dA2 W2^T ----
  {
    float av[KQ];
#pragma unroll
    for (int q = 0; q < KQ / 4; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(&L.sH1T[(16 * w + li) * LDT + KQ * lq + 4 * q]);
      av[4 * q] = t.x; av[4 * q + 1] = t.y; av[4 * q + 2] = t.z; av[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      float bv[KQ];
#pragma unroll
      for (int q = 0; q < KQ / 4; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(&L.sdA2T[(16 * jt + li) * LDT + KQ * lq + 4 * q]);
        bv[4 * q] = t.x; bv[4 * q + 1] = t.y; bv[4 * q + 2] = t.z; bv[4 * q + 3] = t.w;
      }
#pragma unroll
      for (int kk = 0; kk < KQ; ++kk) acc.gW2[jt] = mfma4(av[kk], bv[kk], acc.gW2[jt]);
    }
    float wv[16];
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) {
      const float4 t4 = *reinterpret_cast<const float4*>(&L.sW2[(16 * w + li) * LDW + 16 * lq + 4 * v4]);
      wv[4 * v4] = t4.x; wv[4 * v4 + 1] = t4.y; wv[4 * v4 + 2] = t4.z; wv[4 * v4 + 3] = t4.w;
    }
#pragma unroll
    for (int st = 0; st < TS / 16; ++st) {
      float dv16[16];
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const float4 t4 = *reinterpret_cast<const float4*>(&L.sdA2[(16 * st + li) * LDW + 16 * lq + 4 * v4]);
        dv16[4 * v4] = t4.x; dv16[4 * v4 + 1] = t4.y; dv16[4 * v4 + 2] = t4.z; dv16[4 * v4 + 3] = t4.w;
      }
      f32x4 d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) d = mfma4(dv16[kk], wv[kk], d);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int s = 16 * st + 4 * lq + r;
        const float h1 = L.sH1[s * LDW + 16 * w + li];
        L.sH2[s * LDW + 16 * w + li] = d[r] * (1.0f - h1 * h1);  // dA1
      }
    }
  }
  __syncthreads();
  stamp(54);
  // ---- dW1 += X^T dA1 ; db1 ----
#pragma unroll
  for (int ss = 0; ss < SPW; ++ss) {
    const int s = c8 + ss;
    const float d = L.sH2[s * LDW + f];
    acc.gb1 = acc.gb1 + d;
#pragma unroll
    for (int k = 0; k < OBS; ++k) acc.gW1[k] = fmaf(in.x(s, k), d, acc.gW1[k]);
  }
  stamp(55);
}

// The block's gradient row: W2 straight from the MFMA accumulators, the rest after a
// fixed-order combine of the 4 sample-chunk partials per feature through L.sRed.
// put(index, value) performs each store. Contains one __syncthreads().
template <int OBS, int A, class Put>
XA_DEV void tile_write_row(TileLds<OBS, A>& L, const TileAcc<OBS, A>& acc, Put put) {
  constexpr int AH = A + 1, NSLOT = Dims<OBS, A>::NSLOT;
  const Offs o = offs(OBS, A);
  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63, li = lane & 15, lq = lane >> 4, f = tid & 63;
  {
    float* r = L.sRed + ((tid >> 6) * H + f) * NSLOT;
#pragma unroll
    for (int a = 0; a < AH; ++a) r[a] = acc.gW34[a];
    r[AH] = acc.gb2;
    r[AH + 1] = acc.gb1;
#pragma unroll
    for (int k = 0; k < OBS; ++k) r[AH + 2 + k] = acc.gW1[k];
  }
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) put(o.w2 + (16 * w + 4 * lq + r) * H + 16 * jt + li, acc.gW2[jt][r]);
  if (tid < AH) {
    if (tid < A) put(o.b3 + tid, acc.gb34);
    else put(o.b4, acc.gb34);
  }
  __syncthreads();
  for (int e = tid; e < H * NSLOT; e += 256) {
    const int ff = e / NSLOT, slot = e - ff * NSLOT;
    const float v = ((L.sRed[(0 * H + ff) * NSLOT + slot] + L.sRed[(1 * H + ff) * NSLOT + slot]) +
                     (L.sRed[(2 * H + ff) * NSLOT + slot] + L.sRed[(3 * H + ff) * NSLOT + slot]));
    if (slot < A) put(o.w3 + ff * A + slot, v);
    else if (slot == A) put(o.w4 + ff, v);
    else if (slot == AH) put(o.b2 + ff, v);
    else if (slot == AH + 1) put(o.b1 + ff, v);
    else put(o.w1 + (slot - AH - 2) * H + ff, v);
  }
}

// Block sums of the loss accumulators (pg, value, entropy, count), valid in tid < 4.
// Contains one __syncthreads().
template <int OBS, int A>
XA_DEV float tile_loss_sums(TileLds<OBS, A>& L, const TileAcc<OBS, A>& acc) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const float s0 = xa_wave_sum(acc.l_pg), s1 = xa_wave_sum(acc.l_v);
  const float s2 = xa_wave_sum(acc.l_ent), s3 = xa_wave_sum(acc.l_cnt);
  if (lane == 0) {
    L.sLoss[w][0] = s0;
    L.sLoss[w][1] = s1;
    L.sLoss[w][2] = s2;
    L.sLoss[w][3] = s3;
  }
  __syncthreads();
  return tid < 4 ? (L.sLoss[0][tid] + L.sLoss[1][tid]) + (L.sLoss[2][tid] + L.sLoss[3][tid]) : 0.0f;
}

}  // namespace xa_ac
