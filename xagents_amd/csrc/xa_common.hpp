// Shared device helpers for the xagents_amd HIP kernels (gfx950 / CDNA4 only).
//
// * Deterministic f32 math (xa_expf / xa_logf / xa_tanhf): built only from IEEE
//   +,-,*,/ and fmaf so that the CPU oracle (oracle/xa_oracle.c) can restate the
//   exact same operation sequence and integer action indices come out bit-exact.
//   All kernels are compiled with -ffp-contract=off; every fused multiply-add is
//   written explicitly as fmaf.
// * Philox4x32-10 counter RNG (stateless; counters live in device memory so that
//   hipGraph replays draw fresh numbers).
// * Wave64 butterfly reductions.
// * Thread-local error string for the C ABI (include/xagents_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define XA_DEV __device__ __forceinline__

// ----------------------------------------------------------------------------
// error plumbing (host)
// ----------------------------------------------------------------------------
void xa_set_error(const char* fmt, ...);

#define XA_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      xa_set_error(__VA_ARGS__);           \
      return -1;                           \
    }                                      \
  } while (0)

#define XA_CHECK_LAUNCH(name)                                              \
  do {                                                                     \
    hipError_t e_ = hipGetLastError();                                     \
    if (e_ != hipSuccess) {                                                \
      xa_set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return -2;                                                           \
    }                                                                      \
  } while (0)

// ----------------------------------------------------------------------------
// diagnostic in-kernel stamps (only in the -DXA_STAMPS build, tools/diag): thread 0
// of block 0 accumulates s_memtime deltas per phase slot; read back with
// xa_diag_read_stamps. Production builds compile every XA_STAMP to nothing.
// ----------------------------------------------------------------------------
#ifdef XA_STAMPS
static __device__ unsigned long long xa_stamp_acc[64];
// one reader per translation unit (no relocatable device code)
#define XA_DIAG_READER(name)                                                         \
  extern "C" int name(unsigned long long* host) {                                    \
    unsigned long long zero[64] = {0};                                               \
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(xa_stamp_acc), sizeof(zero)) != hipSuccess) \
      return -1;                                                                     \
    return hipMemcpyToSymbol(HIP_SYMBOL(xa_stamp_acc), zero, sizeof(zero)) == hipSuccess ? 0 : -1; \
  }
#define XA_STAMP_DECL \
  unsigned long long xa_t_last_ = 0; \
  bool xa_stamp_on_ = threadIdx.x == 0 && blockIdx.x == 0;
// a kernel whose logical block ids differ from blockIdx.x names the stamping block
#define XA_STAMP_BLOCK(is_zero) xa_stamp_on_ = threadIdx.x == 0 && (is_zero);
#define XA_STAMP(slot)                                                              \
  do {                                                                              \
    if (xa_stamp_on_) {                                                             \
      unsigned long long t_;                                                        \
      __builtin_amdgcn_sched_barrier(0);                                            \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");    \
      __builtin_amdgcn_sched_barrier(0);                                            \
      if (xa_t_last_) xa_stamp_acc[slot] += t_ - xa_t_last_;                        \
      xa_t_last_ = t_;                                                              \
    }                                                                               \
  } while (0)
#else
#define XA_DIAG_READER(name)
#define XA_STAMP_DECL
#define XA_STAMP_BLOCK(is_zero)
#define XA_STAMP(slot) \
  do {                 \
  } while (0)
#endif

// ----------------------------------------------------------------------------
// deterministic f32 math
// ----------------------------------------------------------------------------
typedef float xa_f2 __attribute__((ext_vector_type(2)));
// two IEEE fmas in one v_pk_fma_f32 (each lane rounds exactly like fmaf)
XA_DEV xa_f2 xa_fma2(xa_f2 a, xa_f2 b, xa_f2 c) { return __builtin_elementwise_fma(a, b, c); }

XA_DEV float xa_as_float(uint32_t u) { return __uint_as_float(u); }
XA_DEV uint32_t xa_as_uint(float f) { return __float_as_uint(f); }

// exp(x): Cody-Waite reduction by ln2, degree-7 Taylor on |r| <= ln2/2, exact
// two-step scaling by 2^n (no intermediate underflow).
// Branch-free: the core runs on the input clamped to the finite range and the
// special cases are fixed up with selects (no exec-mask branches in the callers).
XA_DEV float xa_expf(float x) {
  const float xin = x;
  x = fminf(fmaxf(x, -104.0f), 89.0f);
  float n = rintf(x * 1.44269502162933349609375f);
  float r = fmaf(n, -0.693145751953125f, x);
  r = fmaf(n, -1.428606765330187045e-06f, r);
  float p = 1.98412698e-4f;
  p = fmaf(p, r, 1.38888889e-3f);
  p = fmaf(p, r, 8.33333333e-3f);
  p = fmaf(p, r, 4.16666667e-2f);
  p = fmaf(p, r, 1.66666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  int ni = (int)n;
  int n1 = ni / 2;
  int n2 = ni - n1;
  float s1 = xa_as_float((uint32_t)(n1 + 127) << 23);
  float s2 = xa_as_float((uint32_t)(n2 + 127) << 23);
  float y = (p * s1) * s2;
  y = xin > 88.72283935546875f ? __builtin_inff() : y;
  y = xin < -103.97208404541015625f ? 0.0f : y;
  return xin != xin ? xin : y;
}

// log(x): FreeBSD e_logf reduction (mantissa in [sqrt(.5), sqrt(2))), s = f/(2+f).
// Branch-free like xa_expf: the core runs on a sanitised input.
XA_DEV float xa_logf(float x) {
  const float xin = x;
  const bool ok = x > 0.0f && x < __builtin_inff();
  x = ok ? x : 1.0f;
  uint32_t hx = xa_as_uint(x);
  const bool sub = hx < 0x00800000u;  // subnormal: scale by 2^25
  x = sub ? x * 33554432.0f : x;
  hx = xa_as_uint(x);
  int k = sub ? -25 : 0;
  k += (int)((hx >> 23) & 0xffu) - 127;
  hx &= 0x007fffffu;
  uint32_t i = (hx + (0x95f64u << 3)) & 0x800000u;
  float m = xa_as_float(hx | (i ^ 0x3f800000u));
  k += (int)(i >> 23);
  float f = m - 1.0f;
  float s = f / (2.0f + f);
  float z = s * s;
  float w = z * z;
  float t1 = w * (4.0000972152e-01f + w * 2.4279078841e-01f);
  float t2 = z * (6.6666662693e-01f + w * 2.8498786688e-01f);
  float R = t2 + t1;
  float hfsq = (0.5f * f) * f;
  float dk = (float)k;
  float r = dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
  r = xin == __builtin_inff() ? xin : r;
  r = xin == 0.0f ? -__builtin_inff() : r;
  r = xin < 0.0f ? __builtin_nanf("") : r;
  return xin != xin ? xin : r;
}

// tanh(x): branch-free odd rational minimax x*P(x^2)/Q(x^2) (13/6) on the input
// clamped to +-7.905311 (where tanh rounds to +-1); <= 5 ulp, no exp, no divergence,
// no division.
XA_DEV float xa_tanhf(float x) {
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
  // p / q without the IEEE division sequence (v_div_scale / rcp / div_fmas / div_fixup):
  // q lies in [0.00489, 0.903], so a bit-trick seed (<= 5.1% relative error), two
  // Newton steps (6.4e-6) and one residual correction of the quotient give tanh within
  // the same 4.5 ulp bound in 8 dependent full-rate ops. Integer and fmaf only, so the
  // C oracle restates it bit for bit.
  float r = __int_as_float(0x7EF311C3 - __float_as_int(q));
  r = fmaf(r, fmaf(-q, r, 1.0f), r);
  r = fmaf(r, fmaf(-q, r, 1.0f), r);
  const float t = p * r;
  return fmaf(r, fmaf(-q, t, p), t);
}

// b^t for integer t >= 0 by binary exponentiation in f64 (deterministic: the
// oracle restates the same multiply sequence). Keras forms beta^t with tf.pow.
__host__ __device__ inline double xa_powi(double b, int t) {
  double r = 1.0;
  while (t > 0) {
    if (t & 1) r *= b;
    b *= b;
    t >>= 1;
  }
  return r;
}

// ----------------------------------------------------------------------------
// Philox4x32-10
// ----------------------------------------------------------------------------
struct xa_u4 {
  uint32_t x, y, z, w;
};

XA_DEV xa_u4 xa_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                       uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return xa_u4{c0, c1, c2, c3};
}

// uniform in [0, 1) with 24 random bits
XA_DEV float xa_u01(uint32_t v) { return (float)(v >> 8) * 5.9604644775390625e-08f; }

// ----------------------------------------------------------------------------
// wave64 butterfly reduction: lane l adds lane l^m for m = 1,2,4,...,32.
// f32 addition is commutative, so every lane ends with the identical value and
// the order is the fixed pairwise tree the oracle restates.
// ----------------------------------------------------------------------------
// Partners come from DPP / permlane swaps instead of ds_bpermute (VALU latency, no
// LDS round trip): quad_perm gives exact xor-1/xor-2, row_half_mirror/row_mirror pair
// each lane with the other half of its 8/16-lane group (after the previous levels
// every lane of a group holds the same value, so this equals xor-4/xor-8), and the
// row broadcasts finish the xor-16/xor-32 levels in lane 63, read back as a scalar.
#define XA_DPP_F(v, ctrl) \
  __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))

XA_DEV float xa_wave_sum(float v) {
  v = v + XA_DPP_F(v, 0xB1);   // quad_perm [1,0,3,2]
  v = v + XA_DPP_F(v, 0x4E);   // quad_perm [2,3,0,1]
  v = v + XA_DPP_F(v, 0x141);  // row_half_mirror
  v = v + XA_DPP_F(v, 0x140);  // row_mirror: every lane of row r holds S_r
  // row_bcast:15 into rows 1,3 then row_bcast:31 into rows 2,3: lane 63 ends with
  // (S2 + S3) + (S0 + S1), bitwise equal to the xor-16 / xor-32 butterfly
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// f64 DPP move: the two 32-bit halves take the same lane permutation
template <int CTRL, int ROW_MASK = 0xF>
XA_DEV double xa_dpp_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}

// same tree as xa_wave_sum, in f64; the result is wave-uniform
XA_DEV double xa_wave_sum_f64(double v) {
  v = v + xa_dpp_f64<0xB1>(v);
  v = v + xa_dpp_f64<0x4E>(v);
  v = v + xa_dpp_f64<0x141>(v);
  v = v + xa_dpp_f64<0x140>(v);
  v = v + xa_dpp_f64<0x142, 0xA>(v);
  v = v + xa_dpp_f64<0x143, 0xC>(v);
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// sum over aligned 8-lane groups (xor 1, 2, 4), every lane of a group ends with it
XA_DEV float xa_sum8(float v) {
  v = v + XA_DPP_F(v, 0xB1);
  v = v + XA_DPP_F(v, 0x4E);
  return v + XA_DPP_F(v, 0x141);
}

// ----------------------------------------------------------------------------
// Feistel pseudo-random permutation on [0, n) (cycle walking), used for the
// device-side minibatch shuffle that replaces tf.random.shuffle
// (ppo/agent.py:149-154) when no host permutation is supplied.
// ----------------------------------------------------------------------------
XA_DEV uint32_t xa_feistel_round(uint32_t v, uint32_t key, uint32_t mask) {
  uint32_t h = v * 0x9E3779B1u ^ key;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & mask;
}

XA_DEV uint32_t xa_permute(uint32_t i, uint32_t n, uint32_t half_bits, uint32_t k0, uint32_t k1,
                           uint32_t k2, uint32_t k3) {
  const uint32_t mask = (1u << half_bits) - 1u;
  uint32_t v = i;
  do {
    uint32_t l = v >> half_bits, r = v & mask;
    l ^= xa_feistel_round(r, k0, mask); { uint32_t t = l; l = r; r = t; }
    l ^= xa_feistel_round(r, k1, mask); { uint32_t t = l; l = r; r = t; }
    l ^= xa_feistel_round(r, k2, mask); { uint32_t t = l; l = r; r = t; }
    l ^= xa_feistel_round(r, k3, mask); { uint32_t t = l; l = r; r = t; }
    v = (l << half_bits) | r;
  } while (v >= n);
  return v;
}
