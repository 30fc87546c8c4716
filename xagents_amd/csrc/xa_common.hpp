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
// deterministic f32 math
// ----------------------------------------------------------------------------
XA_DEV float xa_as_float(uint32_t u) { return __uint_as_float(u); }
XA_DEV uint32_t xa_as_uint(float f) { return __float_as_uint(f); }

// exp(x): Cody-Waite reduction by ln2, degree-7 Taylor on |r| <= ln2/2, exact
// two-step scaling by 2^n (no intermediate underflow).
XA_DEV float xa_expf(float x) {
  if (x != x) return x;
  if (x > 88.72283935546875f) return __builtin_inff();
  if (x < -103.97208404541015625f) return 0.0f;
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
  return (p * s1) * s2;
}

// log(x): FreeBSD e_logf reduction (mantissa in [sqrt(.5), sqrt(2))), s = f/(2+f).
XA_DEV float xa_logf(float x) {
  if (x != x) return x;
  if (x < 0.0f) return __builtin_nanf("");
  if (x == 0.0f) return -__builtin_inff();
  if (x == __builtin_inff()) return x;
  int k = 0;
  uint32_t hx = xa_as_uint(x);
  if (hx < 0x00800000u) {  // subnormal
    x = x * 33554432.0f;
    hx = xa_as_uint(x);
    k = -25;
  }
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
  return dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
}

// tanh(x): odd minimax polynomial on |x| < 0.625, 1 - 2/(e^{2|x|}+1) above.
XA_DEV float xa_tanhf(float x) {
  float ax = fabsf(x);
  if (ax < 0.625f) {
    float z = x * x;
    float p = fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f);
    p = fmaf(p, z, -5.37397155531e-2f);
    p = fmaf(p, z, 1.33314422036e-1f);
    p = fmaf(p, z, -3.33332819422e-1f);
    return fmaf(p * z, x, x);
  }
  float r;
  if (ax > 9.0f) {
    r = 1.0f;
  } else {
    float e = xa_expf(ax + ax);
    r = 1.0f - 2.0f / (e + 1.0f);
  }
  return x < 0.0f ? -r : r;
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
// gfx950 permlane16/32 swaps give exact xor-16/xor-32.
#define XA_DPP_F(v, ctrl) \
  __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))

XA_DEV float xa_wave_sum(float v) {
  v = v + XA_DPP_F(v, 0xB1);   // quad_perm [1,0,3,2]
  v = v + XA_DPP_F(v, 0x4E);   // quad_perm [2,3,0,1]
  v = v + XA_DPP_F(v, 0x141);  // row_half_mirror
  v = v + XA_DPP_F(v, 0x140);  // row_mirror
  const int lane = __lane_id();
  {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false,
                                                    false);
    v = v + __int_as_float(((lane >> 4) & 1) ? s[0] : s[1]);
  }
  {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false,
                                                    false);
    v = v + __int_as_float((lane >> 5) ? s[0] : s[1]);
  }
  return v;
}

XA_DEV double xa_wave_sum_f64(double v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v = v + __shfl_xor(v, m, 64);
  return v;
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
