// GAE (PPO.calculate_returns, xagents/ppo/agent.py:48-94) and n-step returns
// (A2C.calculate_returns, xagents/a2c/agent.py:141-171) over env-major [N, T]
// rollout buffers.
//
// Layout / schedule: a workgroup owns 64 envs. Its 256 threads stage the 64
// contiguous [T]-rows of rewards, values and dones into LDS with coalesced loads
// (row stride T+1 floats so the per-env column walk is bank-conflict free), one
// lane per env then runs the reverse recurrence out of LDS (it is a sequential
// recurrence in the reference and must stay one so the f32 rounding is
// identical), writes returns back into LDS, and the 256 threads store the tile
// coalesced. T is chunked when 64 rows do not fit the LDS budget.
//
// Arithmetic (numpy f32 with Python-float scalars, ppo/agent.py:84-92):
//   nnt   = 1 - d[t+1]
//   delta = (r[t] + (gamma * V[t+1]) * nnt) - V[t]
//   A     = delta + ((gamma_lam * nnt) * A)        A starts at 0
//   ret   = A + V[t]
// compiled with -ffp-contract=off so nothing is fused.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int kEnvsPerBlock = 64;
constexpr int kThreads = 256;
constexpr int kMaxChunk = 96;  // time steps per LDS chunk: 3 arrays x 64 x 97 x 4 B = 74 KiB

template <bool GAE>
__global__ __launch_bounds__(kThreads) void returns_kernel(const float* __restrict__ rew,
                                                           const float* __restrict__ val,
                                                           const float* __restrict__ done,
                                                           const float* __restrict__ next_val,
                                                           float* __restrict__ ret, int N, int T,
                                                           float gamma, float gamma_lam) {
  __shared__ float s_rew[kEnvsPerBlock * (kMaxChunk + 1)];
  __shared__ float s_val[kEnvsPerBlock * (kMaxChunk + 1)];
  __shared__ float s_done[kEnvsPerBlock * (kMaxChunk + 1)];
  const int env0 = blockIdx.x * kEnvsPerBlock;
  const int nenv = min(kEnvsPerBlock, N - env0);
  const int tid = threadIdx.x;
  const int my_env = env0 + tid;
  // carried recurrence state for lane `tid` (< nenv)
  float carry = 0.0f;   // GAE: last_lam; n-step: R_{t+1}
  float v_next = 0.0f;  // GAE: V[t+1]
  if (tid < nenv) {
    v_next = next_val[my_env];
    if (!GAE) carry = v_next;
  }
  // chunks from the end of the horizon backwards
  for (int t_hi = T; t_hi > 0; t_hi -= kMaxChunk) {
    const int t_lo = max(0, t_hi - kMaxChunk);
    const int L = t_hi - t_lo;
    const int stride = L + 1;
    __syncthreads();
    // coalesced stage: element (e, j) of the chunk, j in [0, L)
    for (int idx = tid; idx < nenv * L; idx += kThreads) {
      const int e = idx / L, j = idx - e * L;
      const size_t g = (size_t)(env0 + e) * T + t_lo + j;
      s_rew[e * stride + j] = rew[g];
      if (GAE) s_val[e * stride + j] = val[g];
      // dones[t+1] for t in [t_lo, t_hi)
      s_done[e * stride + j] = done[(size_t)(env0 + e) * (T + 1) + t_lo + j + 1];
    }
    __syncthreads();
    if (tid < nenv) {
      float* r = s_rew + tid * stride;
      const float* v = s_val + tid * stride;
      const float* d = s_done + tid * stride;
      for (int j = L - 1; j >= 0; --j) {
        const float nnt = 1.0f - d[j];
        if (GAE) {
          const float vt = v[j];
          const float delta = (r[j] + (gamma * v_next) * nnt) - vt;
          carry = delta + ((gamma_lam * nnt) * carry);
          r[j] = carry + vt;  // return overwrites the reward slot
          v_next = vt;
        } else {
          carry = r[j] + (gamma * carry) * nnt;
          r[j] = carry;
        }
      }
    }
    __syncthreads();
    for (int idx = tid; idx < nenv * L; idx += kThreads) {
      const int e = idx / L, j = idx - e * L;
      ret[(size_t)(env0 + e) * T + t_lo + j] = s_rew[e * stride + j];
    }
  }
}

int launch_returns(bool gae, const float* rew, const float* val, const float* done,
                   const float* next_val, float* ret, int N, int T, float gamma,
                   float gamma_lam, void* stream, const char* name) {
  XA_CHECK_ARG(N > 0 && T > 0, "%s: n_envs and n_steps must be > 0 (got %d, %d)", name, N, T);
  XA_CHECK_ARG(rew && done && next_val && ret && (!gae || val), "%s: null pointer", name);
  dim3 grid((N + kEnvsPerBlock - 1) / kEnvsPerBlock);
  if (gae)
    hipLaunchKernelGGL(returns_kernel<true>, grid, dim3(kThreads), 0, (hipStream_t)stream, rew,
                       val, done, next_val, ret, N, T, gamma, gamma_lam);
  else
    hipLaunchKernelGGL(returns_kernel<false>, grid, dim3(kThreads), 0, (hipStream_t)stream, rew,
                       val, done, next_val, ret, N, T, gamma, gamma_lam);
  XA_CHECK_LAUNCH(name);
  return 0;
}

}  // namespace

extern "C" int xa_gae(const float* rewards, const float* values, const float* dones,
                      const float* next_values, float* returns, int n_envs, int n_steps,
                      float gamma, float gamma_lam, void* stream) {
  return launch_returns(true, rewards, values, dones, next_values, returns, n_envs, n_steps,
                        gamma, gamma_lam, stream, "xa_gae");
}

extern "C" int xa_nstep_returns(const float* rewards, const float* dones,
                                const float* next_values, float* returns, int n_envs,
                                int n_steps, float gamma, void* stream) {
  return launch_returns(false, rewards, nullptr, dones, next_values, returns, n_envs, n_steps,
                        gamma, 0.0f, stream, "xa_nstep_returns");
}
