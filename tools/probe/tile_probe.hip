// Probe: cycles per phase of the persistent update's per-step block work, in isolation
// (one workgroup per CU, no hand-offs): the 16-sample tile (ac_tile.hpp tile_compute),
// the gradient-row combine into LDS (tile_write_row), and Keras Adam on the register
// slices + the LDS weight refresh. s_memtime stamps in thread 0, accumulated over
// `iters` repetitions; a second pass without stamps gives the unstamped total.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tile_probe.hip -o tile_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "../../xagents_amd/csrc/ppo_tile.hpp"

using namespace xa_ac;

// the per-pair Keras Adam of the probe's optimizer-step stand-in (the product update folds
// b1 m / b2 v in ahead of its gradient poll; the arithmetic cost here is the same)
__device__ inline void adam_pk(xa_f2 g, float& th0, float& th1, float& m0, float& m1, float& v0,
                               float& v1, float alpha, float omb1, float omb2, float eps) {
  const xa_f2 m = {m0, m1}, v = {v0, v1};
  const xa_f2 mn = xa_fma2(g - m, xa_f2{omb1, omb1}, m);
  const xa_f2 vn = xa_fma2(g * g - v, xa_f2{omb2, omb2}, v);
  const xa_f2 step = mn * xa_f2{alpha, alpha};
  th0 = th0 - step.x * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vn.x) + eps);
  th1 = th1 - step.y * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vn.y) + eps);
  m0 = mn.x;
  m1 = mn.y;
  v0 = vn.x;
  v1 = vn.y;
}
constexpr int OBS = 4, A = 2;

XA_DEV unsigned long long rnow() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
XA_DEV unsigned long long now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

struct Stamper {
  unsigned long long* acc;
  unsigned long long* last;
  XA_DEV void operator()(int slot) const {
    if (threadIdx.x == 0 && slot >= 50) {
      const unsigned long long t = now();
      acc[slot - 50] += t - *last;
      *last = t;
    }
  }
};

template <int TS, bool STAMPS>
__global__ __launch_bounds__(256) void probe(const float* theta, const float* recs, int iters,
                                             unsigned long long* cyc, float* sink) {
  constexpr int RPT = Dims<OBS, A>::RPT;
  __shared__ __attribute__((aligned(16))) TileLds<OBS, A> L;
  __shared__ __attribute__((aligned(16))) float row[(offs(OBS, A).P + 3) & ~3];
  __shared__ float pre[TS * (OBS + 4)];
  const int tid = threadIdx.x;
  ParamSlice<OBS, A> ps;
  ps.init(tid);
  float wv[16], rv[RPT], mw[16], mr[RPT], vw[16], vr[RPT];
  ps.load(theta, wv, rv);
  for (int i = 0; i < 16; ++i) mw[i] = vw[i] = 0.0f;
  for (int i = 0; i < RPT; ++i) mr[i] = vr[i] = 0.0f;
  ps.to_lds(L, wv, rv);
  for (int i = tid; i < TS * (OBS + 4); i += 256) pre[i] = recs[(blockIdx.x * TS) * (OBS + 4) + i];
  __syncthreads();
  LossCfg cfg;
  cfg.is_ppo = true;
  cfg.has_adv_in = false;
  cfg.clip_norm = 0.1f;
  cfg.value_coef = 0.5f;
  cfg.entropy_coef = 0.01f;
  cfg.adv_eps = 1e-8f;
  cfg.adv_mean = 0.1f;
  cfg.adv_std = 1.2f;
  cfg.adv_rstd = 1.0f / 1.2f;
  cfg.loss_scale = 1.0f / 512.0f;
  unsigned long long acc_c[16] = {0}, last = 0;
  Stamper st{acc_c, &last};
  TileAcc<OBS, A> acc;
  float chk = 0.0f;
  const unsigned long long t_begin = now();
  for (int it = 0; it < iters; ++it) {
    __syncthreads();
    acc.zero();
    if (STAMPS && tid == 0) last = now();
    tile_compute<OBS, A, Stamper, PackedIn<OBS>, TS>(L, acc, cfg, st, PackedIn<OBS>{pre});
    if (STAMPS) st(56);  // tile end
    tile_write_row<OBS, A>(L, acc, [&](int i, float v) { row[i] = v; });
    __syncthreads();
    if (STAMPS) st(57);  // row combine into LDS
    // Adam on the register slices with a gradient read from the row, then the LDS refresh
    float gw[16], gr[RPT];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int c = 0; c < 4; ++c) gw[4 * rr + c] = row[ps.w2_off(rr) + c];
#pragma unroll
    for (int q = 0; q < RPT; ++q) gr[q] = ps.ri[q] >= 0 ? row[ps.ri[q]] : 0.0f;
    const float alpha = 1e-4f, omb1 = 0.1f, omb2 = 0.001f, eps = 1e-7f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      mw[i] = mw[i] + (gw[i] - mw[i]) * omb1;
      vw[i] = vw[i] + (gw[i] * gw[i] - vw[i]) * omb2;
      wv[i] = wv[i] - (mw[i] * alpha) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vw[i]) + eps);
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      mr[q] = mr[q] + (gr[q] - mr[q]) * omb1;
      vr[q] = vr[q] + (gr[q] * gr[q] - vr[q]) * omb2;
      rv[q] = rv[q] - (mr[q] * alpha) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vr[q]) + eps);
    }
    if (STAMPS) st(58);  // Adam
    ps.to_lds(L, wv, rv);
    if (STAMPS) st(59);  // LDS refresh (before the loop-top barrier)
  }
  __syncthreads();
  const unsigned long long t_end = now();
  chk = wv[0] + rv[0];
  if (tid == 0) {
    for (int i = 0; i < 10; ++i) cyc[blockIdx.x * 16 + i] = acc_c[i];
    cyc[blockIdx.x * 16 + 15] = t_end - t_begin;
  }
  sink[blockIdx.x * 256 + tid] = chk;
}

// the same loop on the latency-laid-out tile (ppo_tile.hpp)
template <int TS, bool STAMPS>
__global__ __launch_bounds__(256) void probe2(const float* theta, const float* recs, int iters,
                                              unsigned long long* cyc, float* sink, float* row_out) {
  using namespace xa_pt;
  constexpr int RPT = Dims<OBS, A>::RPT;
  constexpr int P = offs(OBS, A).P;
  __shared__ __attribute__((aligned(16))) PtLds<OBS, A, TS> L;
  __shared__ __attribute__((aligned(16))) float row[(P + 3) & ~3];
  __shared__ __attribute__((aligned(16))) float pre[TS * (OBS + 4)];
  const int tid = threadIdx.x;
  PSlice<OBS, A, TS> ps;
  ps.init(tid);
  float wv[16], rv[RPT], mw[16], mr[RPT], vw[16], vr[RPT];
  ps.load(theta, wv, rv);
  for (int i = 0; i < 16; ++i) mw[i] = vw[i] = 0.0f;
  for (int i = 0; i < RPT; ++i) mr[i] = vr[i] = 0.0f;
  ps.to_lds(L, wv, rv);
  for (int i = tid; i < TS * (OBS + 4); i += 256) pre[i] = recs[(blockIdx.x * TS) * (OBS + 4) + i];
  LossCfg cfg;
  cfg.is_ppo = true;
  cfg.has_adv_in = false;
  cfg.clip_norm = 0.1f;
  cfg.value_coef = 0.5f;
  cfg.entropy_coef = 0.01f;
  cfg.adv_eps = 1e-8f;
  cfg.adv_mean = 0.1f;
  cfg.adv_std = 1.2f;
  cfg.adv_rstd = 1.0f / 1.2f;
  cfg.loss_scale = 1.0f / 512.0f;
  unsigned long long acc_c[16] = {0}, last = 0;
  Stamper st{acc_c, &last};
  PtAcc<OBS, A> acc;
  float w2r[16];
  const unsigned long long r_begin = rnow();
  const unsigned long long t_begin = now();
  for (int it = 0; it < iters; ++it) {
    __syncthreads();
    load_w2_rows(L, w2r);
    acc.zero();
    if (STAMPS && tid == 0) last = now();
    auto put_pair = [&](int pr, float v0, float v1) {
      row[canon_of_exchange<OBS, A>(2 * pr)] = v0;
      row[canon_of_exchange<OBS, A>(2 * pr + 1)] = v1;
    };
    pt_tile<OBS, A, TS>(L, acc, cfg, pre, wv, w2r, rv[0], rv[1], st, true,
                        [&](const PtAcc<OBS, A>& a) { pt_write_row_w2<OBS, A>(a, put_pair); });
    if (STAMPS) st(56);  // tile end
    pt_write_row_rest<OBS, A>(acc, [&](int x, float v) { row[canon_of_exchange<OBS, A>(x)] = v; });
    __syncthreads();
    if (STAMPS) st(57);  // row into LDS
    float gw[16], gr[RPT];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) gw[kk] = row[ps.w2_canon(kk)];
#pragma unroll
    for (int q = 0; q < RPT; ++q) gr[q] = ps.ri[q] >= 0 ? row[ps.ri[q]] : 0.0f;
    if (row_out && it == 0) {
      for (int q = tid; q < P; q += 256) row_out[blockIdx.x * P + q] = row[q];
    }
    const float alpha = 1e-4f, omb1 = 0.1f, omb2 = 0.001f, eps = 1e-7f;
#pragma unroll
    for (int i = 0; i < 16; i += 2)
      adam_pk(xa_f2{gw[i], gw[i + 1]}, wv[i], wv[i + 1], mw[i], mw[i + 1], vw[i], vw[i + 1], alpha,
              omb1, omb2, eps);
#pragma unroll
    for (int q = 0; q + 1 < RPT; q += 2)
      adam_pk(xa_f2{gr[q], gr[q + 1]}, rv[q], rv[q + 1], mr[q], mr[q + 1], vr[q], vr[q + 1], alpha,
              omb1, omb2, eps);
    if (RPT % 2) {
      float t0 = 0.f, m0 = 0.f, v0 = 0.f;
      adam_pk(xa_f2{gr[RPT - 1], 0.0f}, rv[RPT - 1], t0, mr[RPT - 1], m0, vr[RPT - 1], v0, alpha,
              omb1, omb2, eps);
    }
    if (STAMPS) st(58);  // Adam
    ps.to_lds(L, wv, rv);
    if (STAMPS) st(59);  // LDS refresh
  }
  __syncthreads();
  const unsigned long long t_end = now();
  const unsigned long long r_end = rnow();
  if (tid == 0) {
    for (int i = 0; i < 10; ++i) cyc[blockIdx.x * 16 + i] = acc_c[i];
    cyc[blockIdx.x * 16 + 14] = r_end - r_begin;
    cyc[blockIdx.x * 16 + 15] = t_end - t_begin;
  }
  sink[blockIdx.x * 256 + tid] = wv[0] + rv[0] + acc.l_pg;
}

// the old tile's gradient row (canonical order) of one iteration, for the comparison
template <int TS>
__global__ __launch_bounds__(256) void ref_row(const float* theta, const float* recs, float* row_out) {
  constexpr int RPT = Dims<OBS, A>::RPT;
  constexpr int P = offs(OBS, A).P;
  __shared__ __attribute__((aligned(16))) TileLds<OBS, A> L;
  __shared__ __attribute__((aligned(16))) float row[(P + 3) & ~3];
  __shared__ float pre[TS * (OBS + 4)];
  const int tid = threadIdx.x;
  ParamSlice<OBS, A> ps;
  ps.init(tid);
  float wv[16], rv[RPT];
  ps.load(theta, wv, rv);
  ps.to_lds(L, wv, rv);
  for (int i = tid; i < TS * (OBS + 4); i += 256) pre[i] = recs[(blockIdx.x * TS) * (OBS + 4) + i];
  __syncthreads();
  LossCfg cfg;
  cfg.is_ppo = true;
  cfg.has_adv_in = false;
  cfg.clip_norm = 0.1f;
  cfg.value_coef = 0.5f;
  cfg.entropy_coef = 0.01f;
  cfg.adv_eps = 1e-8f;
  cfg.adv_mean = 0.1f;
  cfg.adv_std = 1.2f;
  cfg.adv_rstd = 1.0f / 1.2f;
  cfg.loss_scale = 1.0f / 512.0f;
  TileAcc<OBS, A> acc;
  acc.zero();
  tile_compute<OBS, A, NoStamp, PackedIn<OBS>, TS>(L, acc, cfg, NoStamp(), PackedIn<OBS>{pre});
  tile_write_row<OBS, A>(L, acc, [&](int i, float v) { row[i] = v; });
  __syncthreads();
  for (int q = tid; q < P; q += 256) row_out[blockIdx.x * P + q] = row[q];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int P = offs(OBS, A).P;
  const int nblk = 32;
  std::vector<float> th(P), rec(nblk * 32 * (OBS + 4));
  srand(1);
  auto u = [] { return (float)rand() / RAND_MAX - 0.5f; };
  for (auto& x : th) x = 0.4f * u();
  for (int s = 0; s < nblk * 32; ++s) {
    float* r = &rec[s * (OBS + 4)];
    for (int k = 0; k < OBS; ++k) r[k] = 2.0f * u();
    r[OBS] = (float)(rand() % A);
    r[OBS + 1] = u();
    r[OBS + 2] = u();
    r[OBS + 3] = -0.7f + 0.2f * u();
  }
  float *dth, *drec, *dsink;
  unsigned long long* dcyc;
  hipMalloc(&dth, P * 4);
  hipMalloc(&drec, rec.size() * 4);
  hipMalloc(&dsink, nblk * 256 * 4);
  hipMalloc(&dcyc, nblk * 16 * 8);
  hipMemcpy(dth, th.data(), P * 4, hipMemcpyHostToDevice);
  hipMemcpy(drec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice);
  const char* names[] = {"H1 (VALU tanh)", "Z2 = H1 W2 (MFMA) + tanh", "heads + loss + dz",
                         "dA2 + head grads", "dW2, dH1 (MFMA)", "dW1", "tile end",
                         "row combine into LDS", "Adam (registers)", "LDS weight refresh"};
  for (int ts = 16; ts <= 32; ts += 16) {
    for (int stamps = 1; stamps >= 0; --stamps) {
      hipMemset(dcyc, 0, nblk * 16 * 8);
      auto k = ts == 16 ? (stamps ? probe<16, true> : probe<16, false>)
                        : (stamps ? probe<32, true> : probe<32, false>);
      hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, dth, drec, 10, dcyc, dsink);  // warm
      hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, dth, drec, iters, dcyc, dsink);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
      }
      std::vector<unsigned long long> c(nblk * 16);
      hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
      printf("TS %d, %s: total %.0f cycles per iteration (block 0)\n", ts,
             stamps ? "stamped" : "no stamps", (double)c[15] / iters);
      if (stamps)
        for (int i = 0; i < 10; ++i) printf("  %-28s %8.0f\n", names[i], (double)c[i] / iters);
    }
  }
  float *drow1, *drow2;
  hipMalloc(&drow1, nblk * P * 4);
  hipMalloc(&drow2, nblk * P * 4);
  for (int ts = 16; ts <= 32; ts += 16) {
    for (int stamps = 1; stamps >= 0; --stamps) {
      hipMemset(dcyc, 0, nblk * 16 * 8);
      auto k = ts == 16 ? (stamps ? probe2<16, true> : probe2<16, false>)
                        : (stamps ? probe2<32, true> : probe2<32, false>);
      hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, dth, drec, 10, dcyc, dsink, (float*)nullptr);
      hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, dth, drec, iters, dcyc, dsink, (float*)nullptr);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
      }
      std::vector<unsigned long long> c(nblk * 16);
      hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
      printf("NEW TS %d, %s: total %.0f cycles per iteration (block 0), clock %.2f GHz\n", ts,
             stamps ? "stamped" : "no stamps", (double)c[15] / iters,
             (double)c[15] / (double)c[14] * 0.1);
      const char* n2[] = {"H1 (VALU tanh)", "Z2 (MFMA) + tanh", "head partials (DPP) + barrier",
                          "loss + dz + dA2", "dW2 (MFMA) + barrier", "dH1 (MFMA) + dA1 + dW1",
                          "tile end", "row (W2 direct, rest reduced)", "Adam (registers)",
                          "LDS weight refresh"};
      if (stamps)
        for (int i = 0; i < 10; ++i) printf("  %-30s %8.0f\n", n2[i], (double)c[i] / iters);
    }
    // parity: one iteration of each tile from the same weights and records
    auto kr = ts == 16 ? ref_row<16> : ref_row<32>;
    hipLaunchKernelGGL(kr, dim3(nblk), dim3(256), 0, 0, dth, drec, drow1);
    auto kn = ts == 16 ? probe2<16, false> : probe2<32, false>;
    hipLaunchKernelGGL(kn, dim3(nblk), dim3(256), 0, 0, dth, drec, 1, dcyc, dsink, drow2);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
    std::vector<float> r1(nblk * P), r2(nblk * P);
    hipMemcpy(r1.data(), drow1, r1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), drow2, r2.size() * 4, hipMemcpyDeviceToHost);
    double num = 0, den = 0, mx = 0;
    for (size_t q = 0; q < r1.size(); ++q) {
      const double d = (double)r1[q] - r2[q];
      num += d * d;
      den += (double)r1[q] * r1[q];
      mx = fmax(mx, fabs(d));
    }
    printf("TS %d parity new vs old tile: rel %.3e, max abs %.3e, |ref| %.3e\n", ts,
           sqrt(num / den), mx, sqrt(den));
  }
  return 0;
}
