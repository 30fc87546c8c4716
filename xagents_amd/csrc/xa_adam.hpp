// tf.clip_by_global_norm + Keras Adam element arithmetic, shared by the standalone
// xa_clip_adam kernel and the optimizer tails that the gradient reduce
// (ac_update.hip) and the peer all-reduce (comm.hip) run in their last workgroup.
// Keras OptimizerV2 Adam (utils/common.py:476, training_ops ApplyAdam), clip as
// a2c/agent.py:217 / ppo/agent.py:135-136.
#pragma once
#include <math.h>

#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

// tf.clip_by_global_norm scale: clip * min(1/gn, 1/clip)
XA_DEV float clip_scale(double total, float clip) {
  const float gn = (float)sqrt(total);
  return clip > 0.0f ? clip * fminf(1.0f / gn, 1.0f / clip) : 1.0f;
}

// Keras OptimizerV2 Adam step size, computed as training_ops ApplyAdam receives it
XA_DEV float adam_alpha(float lr, float b1, float b2, int t) {
  const float b1p = (float)xa_powi((double)b1, t);
  const float b2p = (float)xa_powi((double)b2, t);
  return lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
}

// one ApplyAdam element: m += (g-m)(1-b1); v += (g^2-v)(1-b2); theta -= m*alpha/(sqrt(v)+eps)
XA_DEV void adam_elem(float g, float& th, float& m, float& v, float alpha, float omb1,
                      float omb2, float eps) {
  m = m + (g - m) * omb1;
  v = v + (g * g - v) * omb2;
  th = th - (m * alpha) / (sqrtf(v) + eps);
}

// Sum of squares of g * grad_scale in the order of the one-pass xa_clip_adam kernel
// (256 threads, thread i takes i, i + 256, ...; f64 wave sums; (w0 + w1) + (w2 + w3)),
// so a tail reproduces xa_clip_adam bit for bit. Every thread of the block calls it;
// red = 4 doubles of LDS. Contains a __syncthreads().
XA_DEV double clip_norm_sumsq(const float* g, int P, float grad_scale, double* red) {
  constexpr int kBatch = 16;  // loads issued together, then summed in index order
  const int tid = threadIdx.x;
  if (tid < 256) {
    double acc = 0.0;
    for (int i0 = tid; i0 < P; i0 += 256 * kBatch) {
      float x[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int i = i0 + 256 * j;
        x[j] = i < P ? g[i] : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        if (i0 + 256 * j >= P) break;
        const float y = x[j] * grad_scale;
        acc += (double)y * (double)y;
      }
    }
    acc = xa_wave_sum_f64(acc);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
  }
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// The optimizer tail: every thread of the last-arriving block calls it after an
// acquire fence, with the complete gradient g[P] visible. In place on theta/m/v.
XA_DEV void adam_tail_apply(const XaAdamTail& t, const float* g, int P) {
  __shared__ double red[4];
  __shared__ float s_alpha;
  const int tid = threadIdx.x;
  const XaAdam& a = t.adam;
  if (tid == 0) {
    int step = *t.adam_step;
    if (t.bump) {
      step += 1;
      *t.adam_step = step;
    }
    s_alpha = adam_alpha(a.lr, a.beta1, a.beta2, step);
  }
  const bool need_norm = a.clip_norm > 0.0f || t.gnorm_out != nullptr;
  double total = 0.0;
  if (need_norm) total = clip_norm_sumsq(g, P, a.grad_scale, red);
  else __syncthreads();
  if (tid == 0 && t.gnorm_out) t.gnorm_out[0] = (float)sqrt(total);
  const float sc = need_norm ? clip_scale(total, a.clip_norm) : 1.0f;
  const float alpha = s_alpha, omb1 = 1.0f - a.beta1, omb2 = 1.0f - a.beta2;
  constexpr int kBatch = 8;  // every load of a batch issued before the first update
  for (int i0 = tid; i0 < P; i0 += blockDim.x * kBatch) {
    float gg[kBatch], th[kBatch], mm[kBatch], vv[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = min(i0 + (int)blockDim.x * j, P - 1);
      gg[j] = g[i];
      th[j] = t.theta[i];
      mm[j] = t.m[i];
      vv[j] = t.v[i];
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = i0 + (int)blockDim.x * j;
      if (i >= P) break;
      adam_elem((gg[j] * a.grad_scale) * sc, th[j], mm[j], vv[j], alpha, omb1, omb2, a.eps);
      t.theta[i] = th[j];
      t.m[i] = mm[j];
      t.v[i] = vv[j];
    }
  }
}

// Last-block election: every thread has stored its share of the result; returns true
// in the one block that arrives last (which then sees every block's stores) and resets
// the arrival counter for the next launch. Only thread 0 fences (an agent-scope fence
// writes back / invalidates the XCD's L2, far too costly per wave); the other waves
// first drain their own stores (s_waitcnt 0), so thread 0's release covers them.
// Contains __syncthreads().
XA_DEV bool last_block_arrived(unsigned* arrivals) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(arrivals, 1u);
    s_last = prev == gridDim.x - 1;
    if (s_last) {
      *arrivals = 0u;
      __threadfence();  // acquire for the whole block (same CU, same L2)
    }
  }
  __syncthreads();
  return s_last != 0;
}
