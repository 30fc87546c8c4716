// Per-step block work of the persistent PPO update (ppo_update.hip), laid out for latency:
// forward, clipped PPO loss and backward of one tile of TS = 16 or 32 samples
// (PPO.update_gradients' forward / loss / tape.gradient, xagents/ppo/agent.py:96-134) in
// three barrier-separated phases, with every MFMA operand that the block owns kept in
// registers.
//
// Lane map (256 threads = 4 waves, wave w, lane l = 16 lq + li): the lane works on hidden
// unit i = 16 w + li and on the samples s = 16 mt + 4 lq + r (m-tile mt < TS / 16, r < 4)
// in EVERY phase, which is the output layout of v_mfma_f32_16x16x4f32 (D[4 lq + r][li]).
//   1  H1[s][i] = tanh(x_s W1[:, i] + b1[i])     VALU -> registers + LDS (row-major and
//                                                 transposed copies: the MFMA A operands)
//   2  Z2[s][i] = H1[s] W2[:, i]                 MFMA, B operand = the lane's own W2 column
//      H2 = tanh(Z2 + b2) in registers;          (thread ownership below)
//      head partials over the wave's 16 units    DPP row sums -> LDS            | barrier
//   3  logits / value (4 wave partials + b34), the clipped PPO loss and dL/dz per sample,
//      each lane for its own samples (no broadcast); dA2 = (dz W34^T)(1 - H2^2) in
//      registers and LDS; head / b2 gradients;
//      dW2[:, i] += H1^T dA2                     MFMA, B operand = the lane's dA2   | barrier
//   4  dH1[s][i] = dA2[s] W2[i, :]^T             MFMA (A: dA2 from LDS, B: W2 row i,
//                                                 preloaded at the step top)
//      dA1 = dH1 (1 - H1^2) in registers, dW1 / b1 gradients.
// MFMA operands come as 16-byte LDS rows with the K index of lane group q remapped to a
// contiguous block (k = 16 q + kk): only the f32 summation order changes (the update is
// checked against float64 with a tolerance).
//
// Parameter ownership (PSlice): thread t = 64 w + 16 lq + li owns the W2 column
// j = 16 w + li, rows 16 lq .. 16 lq + 15 (exactly its Z2 B operand), and the remaining
// parameters t, t + 256, ... of the non-W2 list. The block's gradient row and the reduced
// gradient travel in EXCHANGE order, as value pairs (one 16-byte granule pair each): the
// W2 values (row 16 lq + kk, column 16 w + li) of thread t sit in pairs 256 h + t
// (h = kk / 2), so a thread's optimizer slice is 8 pairs that the block reads with lane-
// consecutive (coalesced) accesses, and a wave stores a dW2 accumulator tile as 16 runs of
// 256 contiguous bytes; non-W2 value number rr sits at x = H*H + rr.
#pragma once
#include "ac_tile.hpp"

namespace xa_pt {

using namespace xa_ac;

template <int OBS, int A, int TS>
struct PtLds {
  static constexpr int AH = A + 1, AHP = (AH + 3) & ~3, LDT = TS + 4;
  alignas(16) float sW2[H * LDW];   // W2 row-major [i][j] (dH1's B operand)
  alignas(16) float sH1[TS * LDW];  // [s][i]
  alignas(16) float sH1T[H * LDT];  // [i][s]
  alignas(16) float sdA2[TS * LDW]; // [s][j]
  alignas(16) float sZp[4][TS][AHP];  // per-wave partial head sums
  alignas(16) float sdz[4][TS][AHP];  // per-wave copy of dL/dz (wave-private exchange)
  alignas(16) float sW1[OBS * H];
  float sb1[H], sb2[H], sW34[H * AH], sb34[AH];
};

// exchange index -> canonical flat index (Keras trainable_variables order)
template <int OBS, int A>
XA_DEV int canon_of_exchange(int x) {
  const Offs o = offs(OBS, A);
  if (x < H * H) {
    const int pr = x >> 1, t = pr & 255, kk = 2 * (pr >> 8) + (x & 1);
    const int w = t >> 6, lq = (t >> 4) & 3, li = t & 15;
    return o.w2 + (16 * lq + kk) * H + 16 * w + li;
  }
  const int rr = x - H * H;
  return rr < o.w2 ? rr : rr + H * H;
}

// a canonical non-W2 parameter -> its exchange index
template <int OBS, int A>
XA_DEV int exchange_of_rest(int c) {
  const Offs o = offs(OBS, A);
  return H * H + (c < o.w2 ? c : c - H * H);
}

// H1 from registers (OBS = 4): the lanes of hidden unit i own its layer-1 weights, lane row
// lq the weight W1[lq][i] (rest slot 0) and row 0 also b1[i] (slot 1), so the next step's H1
// needs no LDS refresh of W1 / b1 and no barrier in front of it (pt_tile gathers the four
// rows' weights with permlane swaps); every other non-W2 parameter sits on the lanes of rows
// 1..3. The rest slots per thread stay at Dims::RPT.
#ifdef XA_NO_REGH1  // diagnostic A/B build: layer-1 weights through LDS behind a barrier
constexpr bool kRegH1On = false;
#else
constexpr bool kRegH1On = true;
#endif
template <int OBS, int A>
constexpr bool kRegH1 = kRegH1On && OBS == 4 &&
                        1 + (offs(OBS, A).P - offs(OBS, A).b2 + 191) / 192 <= Dims<OBS, A>::RPT;

template <int OBS, int A, int TS>
struct PSlice {
  static constexpr int RPT = Dims<OBS, A>::RPT, NREST = Dims<OBS, A>::NREST;
  int col, row0;  // W2 column 16 w + li, rows row0 .. row0 + 15
  int ri[RPT];    // canonical flat index of rest value q, -1 past the end
  int rx[RPT];    // its exchange index, -1 past the end
  int rdst[RPT];  // its float offset inside PtLds, -1 past the end
  // canonical index of rest slot q of thread tid (-1: none)
  XA_DEV static int rest_of(int tid, int q) {
    const Offs o = offs(OBS, A);
    if constexpr (kRegH1<OBS, A>) {
      const int w = tid >> 6, lane = tid & 63, lq = lane >> 4, li = lane & 15, i = 16 * w + li;
      if (q == 0) return o.w1 + lq * H + i;
      if (lq == 0) return q == 1 ? o.b1 + i : -1;
      const int id2 = (lq - 1) * 64 + 16 * w + li, r2 = id2 + 192 * (q - 1);
      return o.b2 + r2 < o.P ? o.b2 + r2 : -1;
    } else {
      const int r = tid + 256 * q;
      return r < NREST ? (r < o.w2 ? r : r + H * H) : -1;
    }
  }
  XA_DEV void init(int tid) {
    typedef PtLds<OBS, A, TS> T;
    constexpr int AH = A + 1;
    const Offs o = offs(OBS, A);
    const int w = tid >> 6, lane = tid & 63;
    col = 16 * w + (lane & 15);
    row0 = 16 * (lane >> 4);
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int e = rest_of(tid, q);
      ri[q] = e;
      rx[q] = e >= 0 ? exchange_of_rest<OBS, A>(e) : -1;
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
  XA_DEV int w2_canon(int kk) const { return offs(OBS, A).w2 + (row0 + kk) * H + col; }
  XA_DEV void load(const float* base, float (&w)[16], float (&r)[RPT]) const {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) w[kk] = base[w2_canon(kk)];
#pragma unroll
    for (int q = 0; q < RPT; ++q) r[q] = base[ri[q] >= 0 ? ri[q] : 0];
  }
  XA_DEV void store(float* base, const float (&w)[16], const float (&r)[RPT]) const {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) base[w2_canon(kk)] = w[kk];
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (ri[q] >= 0) base[ri[q]] = r[q];
  }
  // the slice into the LDS weight tiles (W2 row-major, W1, biases, heads)
  XA_DEV void to_lds(PtLds<OBS, A, TS>& L, const float (&w)[16], const float (&r)[RPT]) const {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) L.sW2[(row0 + kk) * LDW + col] = w[kk];
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (rdst[q] >= 0) reinterpret_cast<float*>(&L)[rdst[q]] = r[q];
  }
};

// per-thread gradient / loss accumulators of the tiles one block processes in a step
template <int OBS, int A>
struct PtAcc {
  static constexpr int AH = A + 1;
  f32x4 gW2[4];    // dW2[16 it + 4 lq + r][16 w + li]
  float gW34[AH];  // [j][a], j = 16 w + li, this lane's samples
  float gW1[OBS];  // [k][i], i = 16 w + li, this lane's samples
  float gb1, gb2;
  float gb34[AH];  // wave 0, lq == 0 lanes: this lane's samples
  float l_pg, l_v, l_ent, l_cnt;
  XA_DEV void zero() {
#pragma unroll
    for (int it = 0; it < 4; ++it) gW2[it] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int a = 0; a < AH; ++a) gW34[a] = gb34[a] = 0.0f;
#pragma unroll
    for (int k = 0; k < OBS; ++k) gW1[k] = 0.0f;
    gb1 = gb2 = 0.0f;
    l_pg = l_v = l_ent = l_cnt = 0.0f;
  }
};

// ftanh (ac_tile.hpp) on two values at once: packed f32 polynomial and Newton step
XA_DEV xa_f2 ftanh2(xa_f2 x) {
  const float c = 7.90531110763549805f;
  const xa_f2 xc = {fminf(fmaxf(x.x, -c), c), fminf(fmaxf(x.y, -c), c)};
  const xa_f2 x2 = xc * xc;
  auto k2 = [](float v) { return xa_f2{v, v}; };
  xa_f2 p = xa_fma2(x2, k2(-2.76076847742355e-16f), k2(2.00018790482477e-13f));
  p = xa_fma2(x2, p, k2(-8.60467152213735e-11f));
  p = xa_fma2(x2, p, k2(5.12229709037114e-08f));
  p = xa_fma2(x2, p, k2(1.48572235717979e-05f));
  p = xa_fma2(x2, p, k2(6.37261928875436e-04f));
  p = xa_fma2(x2, p, k2(4.89352455891786e-03f));
  p = xc * p;
  xa_f2 q = xa_fma2(x2, k2(1.19825839466702e-06f), k2(1.18534705686654e-04f));
  q = xa_fma2(x2, q, k2(2.26843463243900e-03f));
  q = xa_fma2(x2, q, k2(4.89352518554385e-03f));
  const xa_f2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  const xa_f2 rn = xa_fma2(xa_fma2(-q, r, k2(1.0f)), r, r);  // one Newton step
  return p * rn;
}

// sum over aligned 16-lane rows, every lane of a row ends with it
XA_DEV float xa_sum16(float v) {
  v = v + XA_DPP_F(v, 0xB1);   // quad_perm [1,0,3,2]
  v = v + XA_DPP_F(v, 0x4E);   // quad_perm [2,3,0,1]
  v = v + XA_DPP_F(v, 0x141);  // row_half_mirror
  return v + XA_DPP_F(v, 0x140);  // row_mirror
}

// W2 row i = 16 w + li, columns 16 lq .. 16 lq + 15 (dH1's B operand), from the LDS copy
template <int OBS, int A, int TS>
XA_DEV void load_w2_rows(const PtLds<OBS, A, TS>& L, float (&w2r)[16]) {
  const int tid = threadIdx.x, w = tid >> 6, li = tid & 15, lq = (tid & 63) >> 4;
#pragma unroll
  for (int v4 = 0; v4 < 4; ++v4) {
    const float4 t = *reinterpret_cast<const float4*>(&L.sW2[(16 * w + li) * LDW + 16 * lq + 4 * v4]);
    w2r[4 * v4] = t.x; w2r[4 * v4 + 1] = t.y; w2r[4 * v4 + 2] = t.z; w2r[4 * v4 + 3] = t.w;
  }
}

// permlane swaps between the four 16-lane rows of a wave (v_permlane16_swap /
// v_permlane32_swap on the same value): .x of swap16 holds rows (0, 0, 2, 2), .y rows
// (1, 1, 3, 3); .x of swap32 rows (0, 1, 0, 1), .y rows (2, 3, 2, 3)
XA_DEV float2 xa_swap16(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return make_float2(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
XA_DEV float2 xa_swap32(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return make_float2(__uint_as_float(a[0]), __uint_as_float(a[1]));
}

// One tile: rec = TS packed LDS records {obs[OBS], action (< 0: padding), return, old
// value, old log-prob}; w2c = the thread's W2 column slice, w2r = load_w2_rows (with
// kRegH1 loaded here, after the first barrier); w1v / b1v = the lane's own layer-1 weight
// W1[lq][i] and (row 0) b1[i] (kRegH1; unused otherwise); on the block's last tile of the
// step (last) w2_out(acc) runs right after the dW2 MFMAs. Ends after the dW1 accumulation
// (no trailing barrier; the next tile's first LDS writes come after the other waves passed
// this tile's last barrier).
template <int OBS, int A, int TS, class Stamp, class W2Out>
XA_DEV void pt_tile(PtLds<OBS, A, TS>& L, PtAcc<OBS, A>& acc, const LossCfg& cfg,
                    const float* rec, const float (&w2c)[16], float (&w2r)[16], float w1v,
                    float b1v, Stamp stamp, bool last, W2Out w2_out) {
  static_assert(TS == 16 || TS == 32, "tile sizes: 16 or 32 samples");
  constexpr int NT = TS / 16, AH = A + 1, R = OBS + 4, LDT = PtLds<OBS, A, TS>::LDT;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
  const int i = 16 * w + li;  // this lane's hidden unit
  // ---- 1: H1 ----
  float h1[NT][4];
  {
    // w1[k] = W1[k][i] (kRegH1: the weights of rows lq ^ j from the neighbouring lane rows
    // by permlane swaps, put in k order by selects -- no LDS)
    float w1[OBS];
    float b1;
    if constexpr (kRegH1<OBS, A>) {
      const float2 s16 = xa_swap16(w1v), s32 = xa_swap32(w1v);
      float vj[4];                        // vj[j] = W1[lq ^ j][i]
      vj[0] = w1v;
      vj[1] = (lq & 1) ? s16.x : s16.y;  // row lq ^ 1
      const float2 s48 = xa_swap32(vj[1]);
      vj[2] = (lq & 2) ? s32.x : s32.y;  // row lq ^ 2
      vj[3] = (lq & 2) ? s48.x : s48.y;  // row lq ^ 3
      const bool o1 = lq & 1, o2 = lq & 2;
#pragma unroll
      for (int k = 0; k < OBS; ++k) {  // j = k ^ lq
        const float e0 = ((k & 1) != 0) != o1 ? vj[1] : vj[0];
        const float e1 = ((k & 1) != 0) != o1 ? vj[3] : vj[2];
        w1[k] = ((k & 2) != 0) != o2 ? e1 : e0;
      }
      b1 = xa_swap32(xa_swap16(b1v).x).x;  // row 0's b1[i] on every row
    } else {
#pragma unroll
      for (int k = 0; k < OBS; ++k) w1[k] = L.sW1[k * H + i];
      b1 = L.sb1[i];
    }
    stamp(47);  // (diagnostic) the weights are in registers
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) {
      // two samples per packed op
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int s = 16 * mt + 4 * lq + r;
        xa_f2 z = {0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < OBS; ++k)
          z = xa_fma2(xa_f2{rec[s * R + k], rec[(s + 1) * R + k]}, xa_f2{w1[k], w1[k]}, z);
        const xa_f2 h = ftanh2(z + xa_f2{b1, b1});
        h1[mt][r] = h.x;
        h1[mt][r + 1] = h.y;
      }
      stamp(48);  // (diagnostic) H1 computed
#pragma unroll
      for (int r = 0; r < 4; ++r) L.sH1[(16 * mt + 4 * lq + r) * LDW + i] = h1[mt][r];
      *reinterpret_cast<float4*>(&L.sH1T[i * LDT + 16 * mt + 4 * lq]) =
          make_float4(h1[mt][0], h1[mt][1], h1[mt][2], h1[mt][3]);
    }
  }
  stamp(49);  // this wave's H1 is done (before waiting for the others)
  __syncthreads();
  if constexpr (kRegH1<OBS, A>) load_w2_rows(L, w2r);  // refreshed by every thread by now
  stamp(50);
  // ---- 2: Z2 = H1 W2 on MFMA (two accumulator chains), H2, head partials ----
  float h2[NT][4];
  float w34[AH];
#pragma unroll
  for (int a = 0; a < AH; ++a) w34[a] = L.sW34[i * AH + a];
  {
    const float b2 = L.sb2[i];
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) {
      float av[16];
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const float4 t = *reinterpret_cast<const float4*>(&L.sH1[(16 * mt + li) * LDW + 16 * lq + 4 * v4]);
        av[4 * v4] = t.x; av[4 * v4 + 1] = t.y; av[4 * v4 + 2] = t.z; av[4 * v4 + 3] = t.w;
      }
      f32x4 d0 = {0.0f, 0.0f, 0.0f, 0.0f}, d1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        d0 = mfma4(av[kk], w2c[kk], d0);
        d1 = mfma4(av[kk + 1], w2c[kk + 1], d1);
      }
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const xa_f2 h = ftanh2(xa_f2{d0[r], d0[r + 1]} + xa_f2{d1[r], d1[r + 1]} + xa_f2{b2, b2});
        h2[mt][r] = h.x;
        h2[mt][r + 1] = h.y;
      }
    }
  }
  stamp(51);
#pragma unroll
  for (int mt = 0; mt < NT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int a = 0; a < AH; ++a) {
        const float p = xa_sum16(h2[mt][r] * w34[a]);
        if (li == 0) L.sZp[w][16 * mt + 4 * lq + r][a] = p;
      }
  __syncthreads();
  stamp(52);
  // ---- 3: loss + dL/dz, one sample per lane (lane li: sample 16 mt + li; the lane groups
  // lq repeat it), handed to the lanes that need it through a wave-private LDS copy; dA2,
  // head grads, dW2 ----
  constexpr int AHP = PtLds<OBS, A, TS>::AHP;
  const bool tally = w == 0 && lq == 0;  // one lane per sample accumulates the sums
#pragma unroll
  for (int mt = 0; mt < NT; ++mt) {
    const int s = 16 * mt + li;
    float z[AHP];
#pragma unroll
    for (int a4 = 0; a4 < AHP; a4 += 4) {
      float4 zp[4];
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) zp[ww] = *reinterpret_cast<const float4*>(&L.sZp[ww][s][a4]);
      z[a4] = (zp[0].x + zp[1].x) + (zp[2].x + zp[3].x);
      z[a4 + 1] = (zp[0].y + zp[1].y) + (zp[2].y + zp[3].y);
      z[a4 + 2] = (zp[0].z + zp[1].z) + (zp[2].z + zp[3].z);
      z[a4 + 3] = (zp[0].w + zp[1].w) + (zp[2].w + zp[3].w);
    }
#pragma unroll
    for (int a = 0; a < AH; ++a) z[a] = z[a] + L.sb34[a];
    const float* rs = rec + s * R;
    const float act_f = rs[OBS];
    float dz[AHP];
#pragma unroll
    for (int a = 0; a < AHP; ++a) dz[a] = 0.0f;
    if (act_f >= 0.0f) {
      const int act = (int)act_f;
      float m = z[0];
#pragma unroll
      for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
      float e[A], ssum = 0.0f;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        e[a] = fexp(z[a] - m);
        ssum = ssum + e[a];
      }
      const float ls = flog(ssum), rsum = frcp(ssum);
      float lp[A], pr[A], ent = 0.0f, logp = 0.0f;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        lp[a] = (z[a] - m) - ls;
        pr[a] = e[a] * rsum;
        ent = ent - pr[a] * lp[a];
        if (a == act) logp = lp[a];
      }
      const float v = z[A], R_ = rs[OBS + 1], oldv = rs[OBS + 2];
      const float adv = ((R_ - oldv) - cfg.adv_mean) * cfg.adv_rstd;
      const float ratio = fexp(logp - rs[OBS + 3]);
      const float c = cfg.clip_norm, sc = cfg.loss_scale;
      const float pg1 = -adv * ratio;
      const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      const float pg = fmaxf(pg1, pg2);
      // tf.maximum routes the gradient to its first input when x >= y; the second
      // input's gradient passes tf.clip_by_value only inside [lo, hi]
      const bool r_in = ratio >= 1.0f - c && ratio <= 1.0f + c;
      const float dlogp = (pg1 >= pg2 || r_in) ? (sc * -adv) * ratio : 0.0f;
      const float dvo = v - oldv;
      const float vclip = oldv + fminf(fmaxf(dvo, -c), c);
      const float vl1 = (v - R_) * (v - R_);
      const float vl2 = (vclip - R_) * (vclip - R_);
      const float vl = fmaxf(vl1, vl2);
      // rounding can make oldv + (v - oldv) != v inside the clip range: the clipped
      // branch then still carries the gradient 2 (v_clip - R)
      const float kv = sc * cfg.value_coef * 0.5f * 2.0f;
      float dv;
      if (vl1 >= vl2) dv = kv * (v - R_);
      else dv = (dvo >= -c && dvo <= c) ? kv * (vclip - R_) : 0.0f;
      const float ec = sc * cfg.entropy_coef;
#pragma unroll
      for (int a = 0; a < A; ++a)
        dz[a] = dlogp * ((a == act ? 1.0f : 0.0f) - pr[a]) + ec * pr[a] * (lp[a] + ent);
      dz[A] = dv;
      if (tally) {
        acc.l_pg += pg;
        acc.l_v += vl;
        acc.l_ent += ent;
        acc.l_cnt += 1.0f;
#pragma unroll
        for (int a = 0; a < AH; ++a) acc.gb34[a] += dz[a];
      }
    }
    if (lq == 0) {
#pragma unroll
      for (int a4 = 0; a4 < AHP; a4 += 4)
        *reinterpret_cast<float4*>(&L.sdz[w][s][a4]) = make_float4(dz[a4], dz[a4 + 1], dz[a4 + 2], dz[a4 + 3]);
    }
  }
  // the wave's own LDS writes are done before its reads (in-order LDS queue); keep the
  // compiler from moving the reads above them
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  float da2[NT][4];
#pragma unroll
  for (int mt = 0; mt < NT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * mt + 4 * lq + r;
      float dz[AHP];
#pragma unroll
      for (int a4 = 0; a4 < AHP; a4 += 4) {
        const float4 t = *reinterpret_cast<const float4*>(&L.sdz[w][s][a4]);
        dz[a4] = t.x; dz[a4 + 1] = t.y; dz[a4 + 2] = t.z; dz[a4 + 3] = t.w;
      }
      // dA2 = (dz W34^T) (1 - H2^2), this lane's unit j = i
      float dh = 0.0f;
#pragma unroll
      for (int a = 0; a < AH; ++a) dh = fmaf(dz[a], w34[a], dh);
      const float hv = h2[mt][r];
#pragma unroll
      for (int a = 0; a < AH; ++a) acc.gW34[a] = fmaf(hv, dz[a], acc.gW34[a]);
      const float d = dh * (1.0f - hv * hv);
      acc.gb2 = acc.gb2 + d;
      da2[mt][r] = d;
      L.sdA2[s * LDW + i] = d;
    }
  }
  stamp(53);
  // dW2[:, j = i] += H1^T dA2: output i-tile it, K = samples (step (mt, r): lane group lq
  // is sample 16 mt + 4 lq + r)
#pragma unroll
  for (int it = 0; it < 4; ++it)
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) {
      const float4 t = *reinterpret_cast<const float4*>(&L.sH1T[(16 * it + li) * LDT + 16 * mt + 4 * lq]);
      acc.gW2[it] = mfma4(t.x, da2[mt][0], acc.gW2[it]);
      acc.gW2[it] = mfma4(t.y, da2[mt][1], acc.gW2[it]);
      acc.gW2[it] = mfma4(t.z, da2[mt][2], acc.gW2[it]);
      acc.gW2[it] = mfma4(t.w, da2[mt][3], acc.gW2[it]);
    }
  // the block's dW2 is complete after its last tile: hand it out now, so the stores drain
  // while the dH1 phase runs
  if (last) w2_out(acc);
  __syncthreads();
  stamp(54);
  // ---- 4: dH1 = dA2 W2^T (unit i, K = 64), dA1, dW1 ----
#pragma unroll
  for (int mt = 0; mt < NT; ++mt) {
    float av[16];
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) {
      const float4 t = *reinterpret_cast<const float4*>(&L.sdA2[(16 * mt + li) * LDW + 16 * lq + 4 * v4]);
      av[4 * v4] = t.x; av[4 * v4 + 1] = t.y; av[4 * v4 + 2] = t.z; av[4 * v4 + 3] = t.w;
    }
    f32x4 d0 = {0.0f, 0.0f, 0.0f, 0.0f}, d1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int kk = 0; kk < 16; kk += 2) {
      d0 = mfma4(av[kk], w2r[kk], d0);
      d1 = mfma4(av[kk + 1], w2r[kk + 1], d1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * mt + 4 * lq + r;
      const float hv = h1[mt][r];
      const float d = (d0[r] + d1[r]) * (1.0f - hv * hv);
      acc.gb1 = acc.gb1 + d;
#pragma unroll
      for (int k = 0; k < OBS; ++k) acc.gW1[k] = fmaf(rec[s * R + k], d, acc.gW1[k]);
    }
  }
  stamp(55);
}

// The block's gradient row in exchange order: W2 straight from the MFMA accumulators
// through put_pair(pair, v0, v1) (the accumulator rows r = 0, 1 and r = 2, 3 of lane
// (lq, li) in tile it belong to thread 64 w + 16 it + li, slice pairs 2 lq and 2 lq + 1),
// the other parameters after a fixed-order sum over the lane groups lq (xor 16 / 32
// butterfly) through put(x, v). Also returns the block's loss sums (pg, value, entropy, count) in the
// wave-0 lanes lq == 0 (lane 0 holds the totals). No barrier inside. pt_write_row_w2
// is the W2 part alone (pt_tile calls it after the last tile's dW2, so the stores
// overlap the dH1 phase), pt_write_row_rest the other parameters.
template <int OBS, int A, class PutPair>
XA_DEV void pt_write_row_w2(const PtAcc<OBS, A>& acc, PutPair put_pair) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int t = 64 * w + 16 * it + li;
    put_pair(256 * (2 * lq) + t, acc.gW2[it][0], acc.gW2[it][1]);
    put_pair(256 * (2 * lq + 1) + t, acc.gW2[it][2], acc.gW2[it][3]);
  }
}

// the rest of the row (pt_write_row without its W2 part, which pt_tile stored early)
template <int OBS, int A, class Put>
XA_DEV void pt_write_row_rest(PtAcc<OBS, A>& acc, Put put, bool loss_sums = true) {
  constexpr int AH = A + 1;
  const Offs o = offs(OBS, A);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
  const int i = 16 * w + li;
  // sum over the lane groups lq in the fixed order (lq0 + lq1) + (lq2 + lq3), every lane:
  // v_permlane16_swap / v_permlane32_swap exchange rows 0 <-> 1, 2 <-> 3 and halves
  auto red = [](float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(c[0]) + __uint_as_float(c[1]);
  };
#pragma unroll
  for (int a = 0; a < AH; ++a) acc.gW34[a] = red(acc.gW34[a]);
#pragma unroll
  for (int k = 0; k < OBS; ++k) acc.gW1[k] = red(acc.gW1[k]);
  acc.gb1 = red(acc.gb1);
  acc.gb2 = red(acc.gb2);
  if (w == 0) {  // the tally lanes: wave 0, lq == 0, one sample each
#pragma unroll
    for (int a = 0; a < AH; ++a) acc.gb34[a] = xa_sum16(acc.gb34[a]);
    if (loss_sums) {  // (wave 0 is the last to reach the row barrier: skipped when unused)
      acc.l_pg = xa_sum16(acc.l_pg);
      acc.l_v = xa_sum16(acc.l_v);
      acc.l_ent = xa_sum16(acc.l_ent);
      acc.l_cnt = xa_sum16(acc.l_cnt);
    }
  }
  if (lq == 0) {
#pragma unroll
    for (int a = 0; a < A; ++a) put(exchange_of_rest<OBS, A>(o.w3 + i * A + a), acc.gW34[a]);
    put(exchange_of_rest<OBS, A>(o.w4 + i), acc.gW34[A]);
    put(exchange_of_rest<OBS, A>(o.b2 + i), acc.gb2);
    put(exchange_of_rest<OBS, A>(o.b1 + i), acc.gb1);
#pragma unroll
    for (int k = 0; k < OBS; ++k) put(exchange_of_rest<OBS, A>(o.w1 + k * H + i), acc.gW1[k]);
    if (w == 0 && li == 0) {
#pragma unroll
      for (int a = 0; a < A; ++a) put(exchange_of_rest<OBS, A>(o.b3 + a), acc.gb34[a]);
      put(exchange_of_rest<OBS, A>(o.b4), acc.gb34[A]);
    }
  }
}

}  // namespace xa_pt
