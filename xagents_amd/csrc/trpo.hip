// TRPO pieces around the layer-executor GEMMs (xagents/trpo/agent.py):
//   * xa_trpo_head     per-sample surrogate gain / KL / entropy of Categorical(logits)
//                      and the gradient of surrogate_loss w.r.t. the new logits
//                      (calculate_losses, trpo/agent.py:200-223)
//   * xa_categorical_fisher  the categorical Fisher metric applied to a logit tangent,
//                      (diag(p) - p p^T) t: the middle of the Fisher-vector product
//                      (calculate_fvp, trpo/agent.py:121-148, as J^T M J v at the
//                      point where the actor equals the old actor)
//   * xa_vec_dot / xa_axpby  the conjugate-gradient vector algebra
//                      (conjugate_gradients, trpo/agent.py:150-177)
// Sums are fixed-order (per-block partials in f64, then one block), so every launch
// is deterministic.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int kMaxA = 32;
constexpr int kHeadThreads = 256;

// log-softmax of one row (max-shifted, exp/log from xa_common for determinism)
XA_DEV void log_softmax_row(const float* z, int A, float* lp) {
  float mx = z[0];
  for (int a = 1; a < A; ++a) mx = fmaxf(mx, z[a]);
  float s = 0.0f;
  for (int a = 0; a < A; ++a) s = s + xa_expf(z[a] - mx);
  const float ls = xa_logf(s);
  for (int a = 0; a < A; ++a) lp[a] = (z[a] - mx) - ls;
}

__global__ __launch_bounds__(kHeadThreads) void trpo_head_kernel(XaTrpoHeadArgs h) {
  __shared__ double red[3][kHeadThreads];
  const int i = blockIdx.x * kHeadThreads + threadIdx.x;
  double gain = 0.0, kl = 0.0, ent = 0.0;
  if (i < h.n) {
    const int A = h.n_actions;
    float lpn[kMaxA], lpo[kMaxA];
    log_softmax_row(h.logits_new + (int64_t)i * h.ld_logits, A, lpn);
    log_softmax_row(h.logits_old + (int64_t)i * h.ld_logits, A, lpo);
    const int act = min(max(h.actions[i], 0), A - 1);  // in range by construction; never read out of bounds
    // ratio = exp(new log_prob(a) - old log_prob(a)); H = -sum p log p; KL(old || new)
    const float ratio = xa_expf(lpn[act] - lpo[act]);
    const float adv = h.advantages[i];
    float H = 0.0f, K = 0.0f;
    for (int a = 0; a < A; ++a) {
      const float pn = xa_expf(lpn[a]), po = xa_expf(lpo[a]);
      H = H - pn * lpn[a];
      K = K + po * (lpo[a] - lpn[a]);
    }
    gain = (double)(ratio * adv);
    kl = (double)K;
    ent = (double)H;
    if (h.dlogits) {
      // d/dz_a of [ratio adv + c H] / n:  ratio adv (1[a = act] - p_a) - c p_a (log p_a + H)
      const float inv_n = h.inv_n, c = h.entropy_coef;
      for (int a = 0; a < A; ++a) {
        const float pn = xa_expf(lpn[a]);
        const float d_ratio = ratio * adv * ((a == act ? 1.0f : 0.0f) - pn);
        const float d_ent = -pn * (lpn[a] + H);
        h.dlogits[(int64_t)i * h.ld_dlogits + a] = (d_ratio + c * d_ent) * inv_n;
      }
    }
  }
  red[0][threadIdx.x] = gain;
  red[1][threadIdx.x] = kl;
  red[2][threadIdx.x] = ent;
  __syncthreads();
  for (int s = kHeadThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 3 && h.partials) h.partials[(int64_t)blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// fixed-order sum of the per-block (gain, kl, entropy) partials -> out[3] = means,
// out[0] = mean(ratio adv) + c mean(H) (surrogate_loss), out[1] = mean KL, out[2] = mean H
__global__ void trpo_head_finalize_kernel(const double* partials, int nblocks, double inv_n,
                                          float c, float* out) {
  if (threadIdx.x != 0) return;
  double g = 0.0, k = 0.0, e = 0.0;
  for (int b = 0; b < nblocks; ++b) {
    g += partials[3 * b];
    k += partials[3 * b + 1];
    e += partials[3 * b + 2];
  }
  const float ent = (float)(e * inv_n);
  out[0] = (float)(g * inv_n) + c * ent;
  out[1] = (float)(k * inv_n);
  out[2] = ent;
}

__global__ __launch_bounds__(256) void categorical_fisher_kernel(const float* logits, int64_t ld,
                                                                 const float* tangent,
                                                                 int64_t ld_t, int n, int A,
                                                                 float scale, float* out,
                                                                 int64_t ld_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float lp[kMaxA], p[kMaxA];
  log_softmax_row(logits + (int64_t)i * ld, A, lp);
  float pt = 0.0f;
  for (int a = 0; a < A; ++a) {
    p[a] = xa_expf(lp[a]);
    pt = fmaf(p[a], tangent[(int64_t)i * ld_t + a], pt);
  }
  for (int a = 0; a < A; ++a)
    out[(int64_t)i * ld_out + a] = scale * (p[a] * (tangent[(int64_t)i * ld_t + a] - pt));
}

constexpr int kDotThreads = 1024;

// one block: f64 sum of x y in a fixed order (thread-strided partials, tree in LDS)
__global__ __launch_bounds__(kDotThreads) void vec_dot_kernel(const float* x, const float* y,
                                                              int64_t n, double* out) {
  __shared__ double red[kDotThreads];
  double s = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += kDotThreads) s += (double)x[e] * (double)y[e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = kDotThreads / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

__global__ __launch_bounds__(256) void axpby_kernel(float a, const float* x, float b,
                                                    const float* y, float* out, int64_t n) {
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    out[e] = a * x[e] + b * y[e];
}

// adv = ((ret - val) - mean) / (std + eps), population std, one block (f64 sums in a
// fixed order, the arithmetic on the differences in f32)
__global__ __launch_bounds__(kDotThreads) void norm_adv_kernel(const float* ret, const float* val,
                                                               int n, float eps, float* adv) {
  __shared__ double r1[kDotThreads], r2[kDotThreads];
  double s1 = 0.0, s2 = 0.0;
  for (int e = threadIdx.x; e < n; e += kDotThreads) {
    const double d = (double)(ret[e] - val[e]);
    s1 += d;
    s2 += d * d;
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int k = kDotThreads / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) {
      r1[threadIdx.x] += r1[threadIdx.x + k];
      r2[threadIdx.x] += r2[threadIdx.x + k];
    }
    __syncthreads();
  }
  const double mean = r1[0] / n;
  const double var = fmax(r2[0] / n - mean * mean, 0.0);
  const float m = (float)mean, sd = (float)sqrt(var) + eps;
  for (int e = threadIdx.x; e < n; e += kDotThreads) adv[e] = ((ret[e] - val[e]) - m) / sd;
}

int blocks_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 4096 ? b : 4096);
}

}  // namespace

extern "C" int xa_trpo_head_blocks(int n) { return (n + kHeadThreads - 1) / kHeadThreads; }

extern "C" int xa_trpo_head(const XaTrpoHeadArgs* p, float* out, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_trpo_head: null args");
  const XaTrpoHeadArgs& h = *p;
  XA_CHECK_ARG(h.n > 0 && h.n_actions >= 2 && h.n_actions <= kMaxA,
               "xa_trpo_head: n > 0 and 2 <= n_actions <= %d required", kMaxA);
  XA_CHECK_ARG(h.logits_new && h.logits_old && h.actions && h.advantages && h.partials &&
                   h.ld_logits >= h.n_actions && (!h.dlogits || h.ld_dlogits >= h.n_actions),
               "xa_trpo_head: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int nb = xa_trpo_head_blocks(h.n);
  hipLaunchKernelGGL(trpo_head_kernel, dim3(nb), dim3(kHeadThreads), 0, s, h);
  XA_CHECK_LAUNCH("xa_trpo_head");
  if (out) {
    hipLaunchKernelGGL(trpo_head_finalize_kernel, dim3(1), dim3(64), 0, s, h.partials, nb,
                       1.0 / h.n, h.entropy_coef, out);
    XA_CHECK_LAUNCH("xa_trpo_head (finalize)");
  }
  return 0;
}

extern "C" int xa_categorical_fisher(const float* logits, int64_t ld_logits, const float* tangent,
                                     int64_t ld_tangent, int n, int n_actions, float scale,
                                     float* out, int64_t ld_out, void* stream) {
  XA_CHECK_ARG(logits && tangent && out && n > 0 && n_actions >= 2 && n_actions <= kMaxA &&
                   ld_logits >= n_actions && ld_tangent >= n_actions && ld_out >= n_actions,
               "xa_categorical_fisher: bad arguments");
  hipLaunchKernelGGL(categorical_fisher_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, logits, ld_logits, tangent, ld_tangent, n, n_actions,
                     scale, out, ld_out);
  XA_CHECK_LAUNCH("xa_categorical_fisher");
  return 0;
}

extern "C" int xa_vec_dot(const float* x, const float* y, int64_t n, double* out, void* stream) {
  XA_CHECK_ARG(x && y && out && n > 0, "xa_vec_dot: bad arguments");
  hipLaunchKernelGGL(vec_dot_kernel, dim3(1), dim3(kDotThreads), 0, (hipStream_t)stream, x, y, n,
                     out);
  XA_CHECK_LAUNCH("xa_vec_dot");
  return 0;
}

extern "C" int xa_axpby(float a, const float* x, float b, const float* y, float* out, int64_t n,
                        void* stream) {
  XA_CHECK_ARG(x && y && out && n > 0, "xa_axpby: bad arguments");
  hipLaunchKernelGGL(axpby_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, a, x,
                     b, y, out, n);
  XA_CHECK_LAUNCH("xa_axpby");
  return 0;
}

extern "C" int xa_normalized_advantages(const float* returns, const float* values, int n,
                                        float eps, float* adv, void* stream) {
  XA_CHECK_ARG(returns && values && adv && n > 0, "xa_normalized_advantages: bad arguments");
  hipLaunchKernelGGL(norm_adv_kernel, dim3(1), dim3(kDotThreads), 0, (hipStream_t)stream,
                     returns, values, n, eps, adv);
  XA_CHECK_LAUNCH("xa_normalized_advantages");
  return 0;
}
