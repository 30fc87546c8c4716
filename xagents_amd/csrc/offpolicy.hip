// Off-policy hot path pieces around the GEMMs (gemm.hip):
//   * Conv1D input gradient (col2im as a gather, deterministic) with the ReLU gate of
//     the layer below,
//   * DQN epsilon-greedy action selection and TD targets + MSE gradient
//     (xagents/dqn/agent.py:107-171),
//   * replay rings on device: ReplayBuffer1 (deque + random.sample,
//     xagents/utils/buffers.py:59-98) and ReplayBuffer2 (row-0 overwrite when full,
//     buffers.py:101-148) append / gather. The ring position arithmetic that
//     reproduces the reference's index semantics lives on the host; the kernels move
//     the bytes.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

// dAct[row][q][c] = sum_t dcol[(row P + (q - t) / s) (k C) + t C + c] over taps t with
// (q - t) >= 0, (q - t) % s == 0, (q - t) / s < P; then * [gate > 0]
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcol, int rows,
                                                     int P, int k, int s, int C, int W_in,
                                                     const float* __restrict__ gate,
                                                     float* __restrict__ out) {
  const int64_t total = (int64_t)rows * W_in * C;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    // 32-bit index arithmetic (rows * W_in * C < 2^31, checked on the host)
    const unsigned ue = (unsigned)e;
    const unsigned rq = ue / (unsigned)C;
    const int c = (int)(ue - rq * (unsigned)C);
    const unsigned row_u = rq / (unsigned)W_in;
    const int q = (int)(rq - row_u * (unsigned)W_in);
    const int64_t row = row_u;
    float acc = 0.0f;
    for (int t = 0; t < k; ++t) {
      const int d = q - t;
      if (d < 0 || d % s != 0) continue;
      const int p = d / s;
      if (p >= P) continue;
      acc = acc + dcol[((row * P + p) * k + t) * C + c];
    }
    if (gate && !(gate[e] > 0.0f)) acc = 0.0f;
    out[e] = acc;
  }
}

// argmax (first max, tf.argmax) of each row of q [n x A]; rows flagged random take the
// host-drawn action (np.random.randint, dqn/agent.py:114-116)
__global__ void dqn_act_kernel(const float* __restrict__ q, int n, int A,
                               const int* __restrict__ random_actions, int use_random,
                               int* __restrict__ actions) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (use_random) {
    actions[i] = random_actions[i];
    return;
  }
  const float* r = q + (size_t)i * A;
  int best = 0;
  float bv = r[0];
  for (int a = 1; a < A; ++a)
    if (r[a] > bv) {
      bv = r[a];
      best = a;
    }
  actions[i] = best;
}

// DQN.get_targets + the MSE gradient (dqn/agent.py:118-171):
//   v' = double ? Qt(s')[argmax Q(s')] : max_a Qt(s');  v' = 0 where done
//   y_b = v' gamma + r_b;   L = sum_b mean_a (y - Q)^2 (minimize on a [B] loss sums)
//   dQ[b][a_b] = -2 (y_b - Q[b][a_b]) / A, zero elsewhere (y copies Q off the action)
__global__ void dqn_td_kernel(const float* __restrict__ q, const float* __restrict__ q_next_t,
                              const float* __restrict__ q_next_o, const int* __restrict__ act,
                              const float* __restrict__ rew, const float* __restrict__ done,
                              int B, int A, float gamma, float huber, float* __restrict__ dq,
                              float* __restrict__ loss, int* __restrict__ adam_step) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (adam_step && b == 0) adam_step[0] += 1;  // the update's t += 1, one launch fewer
  if (b >= B) return;
  const float* qt = q_next_t + (size_t)b * A;
  float v;
  if (q_next_o) {
    const float* qo = q_next_o + (size_t)b * A;
    int best = 0;
    float bv = qo[0];
    for (int a = 1; a < A; ++a)
      if (qo[a] > bv) {
        bv = qo[a];
        best = a;
      }
    v = qt[best];
  } else {
    v = qt[0];
    for (int a = 1; a < A; ++a) v = fmaxf(v, qt[a]);
  }
  if (done[b] != 0.0f) v = 0.0f;
  const float y = v * gamma + rew[b];
  const int ab = act[b];
  const float diff = y - q[(size_t)b * A + ab];
  float dqa, l;
  if (huber > 0.0f) {
    // tf.keras.losses.Huber(delta): 0.5 x^2 if |x| <= delta else delta (|x| - 0.5 delta)
    const float ad = fabsf(diff);
    dqa = -fminf(fmaxf(diff, -huber), huber) / (float)A;
    l = (ad <= huber ? 0.5f * (diff * diff) : huber * (ad - 0.5f * huber)) / (float)A;
  } else {
    dqa = (-2.0f * diff) / (float)A;
    l = (diff * diff) / (float)A;
  }
  for (int a = 0; a < A; ++a) dq[(size_t)b * A + a] = a == ab ? dqa : 0.0f;
  if (loss) loss[b] = l;
}

// ring[slot[i]] <- src[i] for n_items items of item_bytes each (append)
__global__ __launch_bounds__(256) void ring_scatter_kernel(const uint8_t* __restrict__ src,
                                                           uint8_t* __restrict__ ring,
                                                           const int64_t* __restrict__ slots,
                                                           int n_items, int64_t item_bytes) {
  const int i = blockIdx.y;
  if (i >= n_items) return;
  const uint8_t* s = src + (int64_t)i * item_bytes;
  uint8_t* d = ring + slots[i] * item_bytes;
  if ((item_bytes & 15) == 0 && ((uintptr_t)s & 15) == 0 && ((uintptr_t)d & 15) == 0) {
    const int64_t n16 = item_bytes >> 4;
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n16; e += (int64_t)gridDim.x * 256)
      reinterpret_cast<uint4*>(d)[e] = reinterpret_cast<const uint4*>(s)[e];
  } else {
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < item_bytes; e += (int64_t)gridDim.x * 256)
      d[e] = s[e];
  }
}

// dst[i] <- ring[slot[i]] (sample gather, env-major batch order)
__global__ __launch_bounds__(256) void ring_gather_kernel(const uint8_t* __restrict__ ring,
                                                          uint8_t* __restrict__ dst,
                                                          const int64_t* __restrict__ slots,
                                                          int n_items, int64_t item_bytes) {
  const int i = blockIdx.y;
  if (i >= n_items) return;
  const uint8_t* s = ring + slots[i] * item_bytes;
  uint8_t* d = dst + (int64_t)i * item_bytes;
  if ((item_bytes & 15) == 0 && ((uintptr_t)s & 15) == 0 && ((uintptr_t)d & 15) == 0) {
    const int64_t n16 = item_bytes >> 4;
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n16; e += (int64_t)gridDim.x * 256)
      reinterpret_cast<uint4*>(d)[e] = reinterpret_cast<const uint4*>(s)[e];
  } else {
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < item_bytes; e += (int64_t)gridDim.x * 256)
      d[e] = s[e];
  }
}

// every field of a sampled batch in one launch: blockIdx.z = field (wave-uniform), the
// field's bytes spread over blockIdx.x as ring_gather_kernel does
__global__ __launch_bounds__(256) void ring_gather_fields_kernel(XaGatherArgs a) {
  const int i = blockIdx.y, f = blockIdx.z;
  if (i >= a.n_items || f >= a.n_fields) return;
  const int64_t nb = a.field[f].item_bytes;
  const uint8_t* s = static_cast<const uint8_t*>(a.field[f].ring) + a.slots[i] * nb;
  uint8_t* d = static_cast<uint8_t*>(a.field[f].dst) + (int64_t)i * nb;
  if ((nb & 15) == 0 && ((uintptr_t)s & 15) == 0 && ((uintptr_t)d & 15) == 0) {
    const int64_t n16 = nb >> 4;
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n16; e += (int64_t)gridDim.x * 256)
      reinterpret_cast<uint4*>(d)[e] = reinterpret_cast<const uint4*>(s)[e];
  } else {
    for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < nb; e += (int64_t)gridDim.x * 256)
      d[e] = s[e];
  }
}

// y = (1 - tau) y + tau x (DDPG.sync_target_models, ddpg/agent.py:73-85); tau = 1: copy
__global__ __launch_bounds__(256) void polyak_kernel(const float* __restrict__ x,
                                                     float* __restrict__ y, int64_t n,
                                                     float tau) {
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    y[e] = tau == 1.0f ? x[e] : (1.0f - tau) * y[e] + tau * x[e];
}

__global__ void step_bump_kernel(int* step) { step[0] += 1; }

// dz = dy * act'(y) from the layer output y (relu: y > 0; tanh: 1 - y^2)
__global__ __launch_bounds__(256) void act_grad_kernel(const float* __restrict__ y,
                                                       const float* __restrict__ dy, int64_t n,
                                                       int act, float* __restrict__ dz) {
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const float v = y[e];
    float d = dy[e];
    if (act == XA_ACT_RELU) d = v > 0.0f ? d : 0.0f;
    else if (act == XA_ACT_TANH) d = d * (1.0f - v * v);
    dz[e] = d;
  }
}

// ---- off-policy replay env step + ring store (BaseAgent.step_envs with
// store_in_buffers, xagents/base.py:388-426) -----------------------------------------
XA_DEV int64_t ring_slot(const XaReplayStepArgs& a, int i) {
  const int64_t cnt = a.ring_count[i];
  // RB1 deque: the append lands after the newest element; RB2: row current_size % size,
  // current_size saturating at size -> row 0 once full (buffers.py:133-135)
  return a.ring_kind == XA_RING_RB2 ? (cnt % a.capacity) : (cnt % a.capacity);
}

XA_DEV void copy_bytes(uint8_t* d, const uint8_t* s, int64_t n, int64_t lo, int64_t hi) {
  for (int64_t e = lo + threadIdx.x; e < hi && e < n; e += blockDim.x) d[e] = s[e];
}

// phase 1: frames (grid: byte chunks x envs); every block reads and writes only its own
// byte range of its env, so reading the old state and overwriting it is race-free
__global__ __launch_bounds__(256) void replay_step_frames_kernel(XaReplayStepArgs a,
                                                                 int64_t chunk) {
  const int i = blockIdx.y;
  const int64_t lo = blockIdx.x * chunk, hi = lo + chunk;
  const int64_t ob = a.obs_bytes;
  const int c = a.cursor[i];
  const uint8_t* s_new = (const uint8_t*)a.rep_obs + ((int64_t)i * a.t_rec + c) * ob;
  const uint8_t* s_post = (const uint8_t*)a.rep_state + ((int64_t)i * a.t_rec + c) * ob;
  uint8_t* st = (uint8_t*)a.state + (int64_t)i * ob;
  // stage this chunk of the old state (register per byte slot: <= 16 per thread)
  const bool vec = (ob & 15) == 0 && (chunk & 15) == 0;
  if (vec) {
    const int64_t lo16 = lo >> 4, hi16 = (hi < ob ? hi : ob) >> 4;
    for (int64_t e = lo16 + threadIdx.x; e < hi16; e += blockDim.x) {
      const uint4 old = reinterpret_cast<const uint4*>(st)[e];
      const uint4 nw = reinterpret_cast<const uint4*>(s_new)[e];
      const uint4 post = reinterpret_cast<const uint4*>(s_post)[e];
      if (a.ring_states) {
        const int64_t slot = (int64_t)i * a.capacity + ring_slot(a, i);
        reinterpret_cast<uint4*>((uint8_t*)a.ring_states + slot * ob)[e] = old;
        reinterpret_cast<uint4*>((uint8_t*)a.ring_new_states + slot * ob)[e] = nw;
      }
      if (a.out_states) reinterpret_cast<uint4*>((uint8_t*)a.out_states + (int64_t)i * ob)[e] = old;
      if (a.out_new_states)
        reinterpret_cast<uint4*>((uint8_t*)a.out_new_states + (int64_t)i * ob)[e] = nw;
      reinterpret_cast<uint4*>(st)[e] = post;
    }
  } else {
    for (int64_t e = lo + threadIdx.x; e < hi && e < ob; e += blockDim.x) {
      const uint8_t old = st[e], nw = s_new[e], post = s_post[e];
      if (a.ring_states) {
        const int64_t slot = (int64_t)i * a.capacity + ring_slot(a, i);
        ((uint8_t*)a.ring_states)[slot * ob + e] = old;
        ((uint8_t*)a.ring_new_states)[slot * ob + e] = nw;
      }
      if (a.out_states) ((uint8_t*)a.out_states)[(int64_t)i * ob + e] = old;
      if (a.out_new_states) ((uint8_t*)a.out_new_states)[(int64_t)i * ob + e] = nw;
      st[e] = post;
    }
  }
}

// phase 2: per-env scalars, ring scalars, cursor / counters (one thread per env)
__global__ void replay_step_scalars_kernel(XaReplayStepArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_envs) return;
  const int c = a.cursor[i];
  const float r = a.rep_rew[(int64_t)i * a.t_rec + c];
  const float d = a.rep_done[(int64_t)i * a.t_rec + c];
  if (a.ring_states) {
    const int64_t slot = (int64_t)i * a.capacity + ring_slot(a, i);
    const uint8_t* src = (const uint8_t*)a.actions + (int64_t)i * a.act_bytes;
    uint8_t* dst = (uint8_t*)a.ring_actions + slot * a.act_bytes;
    for (int64_t e = 0; e < a.act_bytes; ++e) dst[e] = src[e];
    a.ring_rewards[slot] = r;
    a.ring_dones[slot] = d;
    const int64_t cnt = a.ring_count[i];
    a.ring_count[i] = a.ring_kind == XA_RING_RB2 ? (cnt < a.capacity ? cnt + 1 : cnt) : cnt + 1;
  }
  const int64_t o = (int64_t)i * (a.out_ld > 0 ? a.out_ld : 1);
  if (a.out_rewards) a.out_rewards[o] = r;
  if (a.out_dones) a.out_dones[o] = d;
  float ep = a.ep_return[i] + r;
  if (a.done_epret) a.done_epret[o] = d != 0.0f ? ep : 0.0f;
  if (d != 0.0f) ep = 0.0f;
  a.ep_return[i] = ep;
  a.done[i] = d;
  a.cursor[i] = c + 1 < a.t_rec ? c + 1 : 0;
}

// small observations (vector envs): both phases in ONE launch, one workgroup per env -- the
// frame bytes of env i by its workgroup, then its scalars by thread 0 (the cursor is read
// by every thread before thread 0 advances it behind the barrier)
__global__ __launch_bounds__(256) void replay_step_small_kernel(XaReplayStepArgs a) {
  const int i = blockIdx.x;
  const int64_t ob = a.obs_bytes;
  const int c = a.cursor[i];
  const uint8_t* s_new = (const uint8_t*)a.rep_obs + ((int64_t)i * a.t_rec + c) * ob;
  const uint8_t* s_post = (const uint8_t*)a.rep_state + ((int64_t)i * a.t_rec + c) * ob;
  uint8_t* st = (uint8_t*)a.state + (int64_t)i * ob;
  const int64_t slot = a.ring_states ? (int64_t)i * a.capacity + ring_slot(a, i) : 0;
  const uintptr_t bases = (uintptr_t)a.state | (uintptr_t)a.rep_obs | (uintptr_t)a.rep_state |
                          (uintptr_t)a.ring_states | (uintptr_t)a.ring_new_states |
                          (uintptr_t)a.out_states | (uintptr_t)a.out_new_states;
  if ((ob & 15) == 0 && (bases & 15) == 0) {
    // 16-B moves (frames: 7056 B = 441 per env): every address is a 16-B aligned base plus
    // a multiple of ob
    const int64_t n16 = ob >> 4;
    for (int64_t e = threadIdx.x; e < n16; e += blockDim.x) {
      const uint4 old = reinterpret_cast<const uint4*>(st)[e];
      const uint4 nw = reinterpret_cast<const uint4*>(s_new)[e];
      const uint4 post = reinterpret_cast<const uint4*>(s_post)[e];
      if (a.ring_states) {
        reinterpret_cast<uint4*>((uint8_t*)a.ring_states + slot * ob)[e] = old;
        reinterpret_cast<uint4*>((uint8_t*)a.ring_new_states + slot * ob)[e] = nw;
      }
      if (a.out_states) reinterpret_cast<uint4*>((uint8_t*)a.out_states + (int64_t)i * ob)[e] = old;
      if (a.out_new_states)
        reinterpret_cast<uint4*>((uint8_t*)a.out_new_states + (int64_t)i * ob)[e] = nw;
      reinterpret_cast<uint4*>(st)[e] = post;
    }
  } else {
    for (int64_t e = threadIdx.x; e < ob; e += blockDim.x) {
      const uint8_t old = st[e], nw = s_new[e], post = s_post[e];
      if (a.ring_states) {
        ((uint8_t*)a.ring_states)[slot * ob + e] = old;
        ((uint8_t*)a.ring_new_states)[slot * ob + e] = nw;
      }
      if (a.out_states) ((uint8_t*)a.out_states)[(int64_t)i * ob + e] = old;
      if (a.out_new_states) ((uint8_t*)a.out_new_states)[(int64_t)i * ob + e] = nw;
      st[e] = post;
    }
  }
  __syncthreads();  // (ring_slot and the cursor above were read before the scalars advance them)
  if (threadIdx.x != 0) return;
  const float r = a.rep_rew[(int64_t)i * a.t_rec + c];
  const float d = a.rep_done[(int64_t)i * a.t_rec + c];
  if (a.ring_states) {
    const uint8_t* src = (const uint8_t*)a.actions + (int64_t)i * a.act_bytes;
    uint8_t* dst = (uint8_t*)a.ring_actions + slot * a.act_bytes;
    for (int64_t e = 0; e < a.act_bytes; ++e) dst[e] = src[e];
    a.ring_rewards[slot] = r;
    a.ring_dones[slot] = d;
    const int64_t cnt = a.ring_count[i];
    a.ring_count[i] = a.ring_kind == XA_RING_RB2 ? (cnt < a.capacity ? cnt + 1 : cnt) : cnt + 1;
  }
  const int64_t o = (int64_t)i * (a.out_ld > 0 ? a.out_ld : 1);
  if (a.out_rewards) a.out_rewards[o] = r;
  if (a.out_dones) a.out_dones[o] = d;
  float ep = a.ep_return[i] + r;
  if (a.done_epret) a.done_epret[o] = d != 0.0f ? ep : 0.0f;
  if (d != 0.0f) ep = 0.0f;
  a.ep_return[i] = ep;
  a.done[i] = d;
  a.cursor[i] = c + 1 < a.t_rec ? c + 1 : 0;
}

// dst[r][c] = src[r][c] for a rows x cols block (concat / column slices of [B, n] rows)
__global__ __launch_bounds__(256) void copy_block_kernel(const float* __restrict__ src,
                                                         int64_t ld_src, float* __restrict__ dst,
                                                         int64_t ld_dst, int rows, int cols) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / cols, c = e % cols;
    dst[r * ld_dst + c] = src[r * ld_src + c];
  }
}

// standard normal from Philox4x32-10 (Box-Muller on two 24-bit uniforms in (0, 1])
XA_DEV float philox_normal(uint32_t i, uint32_t j, uint64_t ctr, uint64_t seed) {
  const xa_u4 r = xa_philox(i, j, (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)seed,
                            (uint32_t)(seed >> 32));
  const float u1 = ((float)(r.x >> 8) + 1.0f) * 5.9604644775390625e-08f;
  const float u2 = (float)(r.y >> 8) * 5.9604644775390625e-08f;
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// out[b][a] = clip(x[b][a] + clip(sigma N(0,1), -noise_clip, noise_clip), lo, hi)
// TD3 target smoothing (td3/agent.py:83-91) and DDPG exploration (ddpg/agent.py:60-71)
__global__ void noisy_actions_kernel(const float* __restrict__ x, int64_t ld_x, int rows,
                                     int cols, float sigma, float noise_clip, float lo, float hi,
                                     const uint64_t* __restrict__ ctr, uint64_t seed,
                                     float* __restrict__ out, int64_t ld_out,
                                     float* __restrict__ noise_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * cols) return;
  const int b = e / cols, a = e % cols;
  float n = 0.0f;
  if (sigma != 0.0f) {
    n = philox_normal((uint32_t)b, (uint32_t)a, ctr ? *ctr : 0ull, seed) * sigma;
    n = fminf(fmaxf(n, -noise_clip), noise_clip);
  }
  if (noise_out) noise_out[e] = n;
  out[(int64_t)b * ld_out + a] = fminf(fmaxf(x[(int64_t)b * ld_x + a] + n, lo), hi);
}

// DDPG / TD3 critic targets and MSE gradients (ddpg/agent.py:104-127, td3/agent.py:66-110):
//   y = r + ((1 - d) gamma) min(tv1, tv2);  dv_i = 2 (v_i - y)  (MSE over a size-1 axis,
//   minimize sums over the batch); loss_i[b] = (v_i - y)^2
__global__ void critic_td_kernel(const float* __restrict__ v1, const float* __restrict__ v2,
                                 const float* __restrict__ tv1, const float* __restrict__ tv2,
                                 const float* __restrict__ rew, const float* __restrict__ done,
                                 int B, float gamma, float huber, float* __restrict__ dv1,
                                 float* __restrict__ dv2, float* __restrict__ loss) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float tv = tv2 ? fminf(tv1[b], tv2[b]) : tv1[b];
  const float y = rew[b] + ((1.0f - done[b]) * gamma) * tv;
  // MSE (the reference): d = 2 e, l = e^2; Huber(delta) opt-in: d = clip(e, +-delta),
  // l = 0.5 e^2 if |e| <= delta else delta (|e| - 0.5 delta)
  auto term = [huber](float e, float& d) {
    if (huber > 0.0f) {
      d = fminf(fmaxf(e, -huber), huber);
      const float ae = fabsf(e);
      return ae <= huber ? 0.5f * (e * e) : huber * (ae - 0.5f * huber);
    }
    d = 2.0f * e;
    return e * e;
  };
  float d1;
  float l = term(v1[b] - y, d1);
  dv1[b] = d1;
  if (v2) {
    float d2;
    l = l + term(v2[b] - y, d2);
    dv2[b] = d2;
  }
  if (loss) loss[b] = l;
}

int grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

// workgroups per item: one 256-thread pass of 16-B chunks each, at most 64
int ring_grid_x(int64_t item_bytes) {
  const int64_t g = ((item_bytes + 15) / 16 + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 64 ? 64 : g));
}

}  // namespace

extern "C" int xa_conv1d_input_grad(const float* dcol, int rows, int positions, int kernel,
                                    int stride, int channels, int width_in, const float* gate,
                                    float* dinput, void* stream) {
  XA_CHECK_ARG(dcol && dinput && rows > 0 && positions > 0 && kernel > 0 && stride > 0 &&
                   channels > 0 && width_in >= (positions - 1) * stride + kernel,
               "xa_conv1d_input_grad: bad arguments");
  const int64_t total = (int64_t)rows * width_in * channels;
  XA_CHECK_ARG(total < (1ll << 31), "xa_conv1d_input_grad: rows * width * channels >= 2^31");
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     dcol, rows, positions, kernel, stride, channels, width_in, gate, dinput);
  XA_CHECK_LAUNCH("xa_conv1d_input_grad");
  return 0;
}

extern "C" int xa_dqn_act(const float* q, int n, int n_actions, const int* random_actions,
                          int use_random, int* actions, void* stream) {
  XA_CHECK_ARG(actions && n > 0 && n_actions > 0 && (use_random ? random_actions != nullptr : q != nullptr),
               "xa_dqn_act: bad arguments");
  hipLaunchKernelGGL(dqn_act_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, q, n,
                     n_actions, random_actions, use_random, actions);
  XA_CHECK_LAUNCH("xa_dqn_act");
  return 0;
}

extern "C" int xa_dqn_td_grad(const float* q, const float* q_next_target,
                              const float* q_next_online, const int* actions,
                              const float* rewards, const float* dones, int batch, int n_actions,
                              float gamma, float huber_delta, float* dq, float* loss,
                              int* adam_step, void* stream) {
  XA_CHECK_ARG(q && q_next_target && actions && rewards && dones && dq && batch > 0 &&
                   n_actions > 0,
               "xa_dqn_td_grad: bad arguments");
  hipLaunchKernelGGL(dqn_td_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream, q,
                     q_next_target, q_next_online, actions, rewards, dones, batch, n_actions,
                     gamma, huber_delta, dq, loss, adam_step);
  XA_CHECK_LAUNCH("xa_dqn_td_grad");
  return 0;
}

extern "C" int xa_ring_scatter(const void* src, void* ring, const int64_t* slots, int n_items,
                               int64_t item_bytes, void* stream) {
  XA_CHECK_ARG(src && ring && slots && n_items > 0 && item_bytes > 0,
               "xa_ring_scatter: bad arguments");
  const int gx = ring_grid_x(item_bytes);
  hipLaunchKernelGGL(ring_scatter_kernel, dim3(gx, n_items), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)src, (uint8_t*)ring, slots, n_items, item_bytes);
  XA_CHECK_LAUNCH("xa_ring_scatter");
  return 0;
}

extern "C" int xa_ring_gather(const void* ring, void* dst, const int64_t* slots, int n_items,
                              int64_t item_bytes, void* stream) {
  XA_CHECK_ARG(dst && ring && slots && n_items > 0 && item_bytes > 0,
               "xa_ring_gather: bad arguments");
  const int gx = ring_grid_x(item_bytes);
  hipLaunchKernelGGL(ring_gather_kernel, dim3(gx, n_items), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)ring, (uint8_t*)dst, slots, n_items, item_bytes);
  XA_CHECK_LAUNCH("xa_ring_gather");
  return 0;
}

extern "C" int xa_ring_gather_fields(const XaGatherArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_ring_gather_fields: null args");
  const XaGatherArgs& a = *p;
  XA_CHECK_ARG(a.n_fields > 0 && a.n_fields <= XA_GATHER_MAX_FIELDS && a.n_items > 0 && a.slots,
               "xa_ring_gather_fields: need 1..%d fields, n_items > 0 and slots",
               XA_GATHER_MAX_FIELDS);
  int gx = 1;
  for (int f = 0; f < a.n_fields; ++f) {
    XA_CHECK_ARG(a.field[f].ring && a.field[f].dst && a.field[f].item_bytes > 0,
                 "xa_ring_gather_fields: field %d: null ring / dst or item_bytes <= 0", f);
    const int g = ring_grid_x(a.field[f].item_bytes);
    gx = g > gx ? g : gx;
  }
  hipLaunchKernelGGL(ring_gather_fields_kernel, dim3(gx, a.n_items, a.n_fields), dim3(256), 0,
                     (hipStream_t)stream, a);
  XA_CHECK_LAUNCH("xa_ring_gather_fields");
  return 0;
}

extern "C" int xa_polyak(const float* src, float* dst, int64_t n, float tau, void* stream) {
  XA_CHECK_ARG(src && dst && n > 0, "xa_polyak: bad arguments");
  hipLaunchKernelGGL(polyak_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src,
                     dst, n, tau);
  XA_CHECK_LAUNCH("xa_polyak");
  return 0;
}

extern "C" int xa_adam_step_bump(int* adam_step, void* stream) {
  XA_CHECK_ARG(adam_step != nullptr, "xa_adam_step_bump: null step");
  hipLaunchKernelGGL(step_bump_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, adam_step);
  XA_CHECK_LAUNCH("xa_adam_step_bump");
  return 0;
}

extern "C" int xa_activation_grad(const float* y, const float* dy, int64_t n, int act,
                                  float* dz, void* stream) {
  XA_CHECK_ARG(y && dy && dz && n > 0, "xa_activation_grad: bad arguments");
  hipLaunchKernelGGL(act_grad_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, y,
                     dy, n, act, dz);
  XA_CHECK_LAUNCH("xa_activation_grad");
  return 0;
}

extern "C" int xa_replay_env_step(const XaReplayStepArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_replay_env_step: null args");
  const XaReplayStepArgs& a = *p;
  XA_CHECK_ARG(a.n_envs > 0 && a.t_rec > 0 && a.obs_bytes > 0 && a.rep_obs && a.rep_state &&
                   a.rep_rew && a.rep_done && a.state && a.cursor && a.ep_return && a.done,
               "xa_replay_env_step: bad env arguments");
  XA_CHECK_ARG(!a.ring_states || (a.ring_new_states && a.ring_actions && a.ring_rewards &&
                                  a.ring_dones && a.ring_count && a.capacity > 0 &&
                                  a.actions && a.act_bytes > 0),
               "xa_replay_env_step: incomplete replay ring");
  hipStream_t s = (hipStream_t)stream;
  const int64_t chunk = 4096;
  dim3 grid((unsigned)((a.obs_bytes + chunk - 1) / chunk), a.n_envs);
  // vector observations and single frames up to 32 KB (C3's 84 x 84 frames: 7056 B): one
  // launch, one workgroup per env
  if (a.obs_bytes <= 4096 || (a.obs_bytes <= 32768 && (a.obs_bytes & 15) == 0)) {
    hipLaunchKernelGGL(replay_step_small_kernel, dim3(a.n_envs), dim3(256), 0, s, a);
    XA_CHECK_LAUNCH("xa_replay_env_step (small)");
    return 0;
  }
  hipLaunchKernelGGL(replay_step_frames_kernel, grid, dim3(256), 0, s, a, chunk);
  XA_CHECK_LAUNCH("xa_replay_env_step (frames)");
  hipLaunchKernelGGL(replay_step_scalars_kernel, dim3((a.n_envs + 63) / 64), dim3(64), 0, s, a);
  XA_CHECK_LAUNCH("xa_replay_env_step (scalars)");
  return 0;
}

// tf.keras.losses.MSE(y, pred) over the last axis, gradient of its batch sum
// (optimizer.minimize on a [B] loss, dqn/agent.py:158-171): d = 2 (pred - y) / A
__global__ void mse_grad_kernel(const float* __restrict__ pred, const float* __restrict__ y,
                                int B, int A, float* __restrict__ d, float* __restrict__ loss) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc = 0.0f;
  for (int a = 0; a < A; ++a) {
    const float e = pred[(size_t)b * A + a] - y[(size_t)b * A + a];
    d[(size_t)b * A + a] = (2.0f * e) / (float)A;
    acc = acc + e * e;
  }
  if (loss) loss[b] = acc / (float)A;
}

extern "C" int xa_mse_grad(const float* pred, const float* target, int batch, int n_out,
                           float* dpred, float* loss, void* stream) {
  XA_CHECK_ARG(pred && target && dpred && batch > 0 && n_out > 0, "xa_mse_grad: bad arguments");
  hipLaunchKernelGGL(mse_grad_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     pred, target, batch, n_out, dpred, loss);
  XA_CHECK_LAUNCH("xa_mse_grad");
  return 0;
}

extern "C" int xa_copy_block(const float* src, int64_t ld_src, float* dst, int64_t ld_dst,
                             int rows, int cols, void* stream) {
  XA_CHECK_ARG(src && dst && rows > 0 && cols > 0 && ld_src >= cols && ld_dst >= cols,
               "xa_copy_block: bad arguments");
  hipLaunchKernelGGL(copy_block_kernel, dim3(grid_for((int64_t)rows * cols)), dim3(256), 0,
                     (hipStream_t)stream, src, ld_src, dst, ld_dst, rows, cols);
  XA_CHECK_LAUNCH("xa_copy_block");
  return 0;
}

extern "C" int xa_noisy_actions(const float* x, int64_t ld_x, int rows, int cols, float sigma,
                                float noise_clip, float lo, float hi, const uint64_t* rng_counter,
                                uint64_t seed, float* out, int64_t ld_out, float* noise_out,
                                void* stream) {
  XA_CHECK_ARG(x && out && rows > 0 && cols > 0, "xa_noisy_actions: bad arguments");
  hipLaunchKernelGGL(noisy_actions_kernel, dim3((rows * cols + 63) / 64), dim3(64), 0,
                     (hipStream_t)stream, x, ld_x, rows, cols, sigma, noise_clip, lo, hi,
                     rng_counter, seed, out, ld_out, noise_out);
  XA_CHECK_LAUNCH("xa_noisy_actions");
  return 0;
}

extern "C" int xa_critic_td_grad(const float* v1, const float* v2, const float* tv1,
                                 const float* tv2, const float* rewards, const float* dones,
                                 int batch, float gamma, float huber_delta, float* dv1,
                                 float* dv2, float* loss, void* stream) {
  XA_CHECK_ARG(v1 && tv1 && rewards && dones && dv1 && batch > 0 && (!v2 || dv2),
               "xa_critic_td_grad: bad arguments");
  hipLaunchKernelGGL(critic_td_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     v1, v2, tv1, tv2, rewards, dones, batch, gamma, huber_delta, dv1, dv2, loss);
  XA_CHECK_LAUNCH("xa_critic_td_grad");
  return 0;
}
