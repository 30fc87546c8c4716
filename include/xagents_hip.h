/*
 * xagents_hip.h -- C ABI of libxagents_hip.so, the MI355X (gfx950) hot path of an
 * xagents-compatible RL training core.
 *
 * Conventions:
 *   - Caller owns all memory. Every pointer is a device pointer (hipMalloc /
 *     torch tensor data_ptr) unless stated. The library never allocates or frees.
 *   - Every function is asynchronous on `stream` (a hipStream_t, NULL = default)
 *     and may be captured into a hipGraph (no sync, no malloc inside).
 *   - Return 0 on success, negative on error; xa_last_error() gives the message
 *     (thread-local).
 *   - Rollout and batch tensors are env-major: [n_envs, n_steps, ...]. The flat
 *     index i = env * n_steps + t is exactly the order the reference produces with
 *     BaseAgent.concat_step_batches (xagents/base.py:549-564, swapaxes(0,1).reshape).
 *   - Actor-critic MLP parameters live in ONE flat f32 buffer laid out in Keras
 *     trainable_variables order for the .cfg topology
 *       dense-0 (obs->64, tanh), dense-1 (64->64, tanh, common), dense-2 (64->A
 *       logits), dense-3 (64->1 value)     (xagents/ppo/models/ann-actor-critic.cfg)
 *     i.e. W1[obs][64], b1[64], W2[64][64], b2[64], W3[64][A], b3[A], W4[64][1], b4[1]
 *     (Keras Dense kernel is (in, out), y = x @ W + b; xagents/utils/common.py:239-258).
 *     Gradients and Adam moments use the same layout.
 */
#ifndef XAGENTS_HIP_H
#define XAGENTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XA_ABI_VERSION 2
#define XA_MLP_HIDDEN 64

/* environment kinds for the fused rollout */
#define XA_ENV_REPLAY 0   /* synthetic pre-recorded observation replay (BASELINE config 2) */
#define XA_ENV_CARTPOLE 1 /* CartPole-v1 dynamics on device (gym classic_control semantics) */

/* return kinds computed at the end of the fused rollout */
#define XA_RETURNS_NONE 0
#define XA_RETURNS_GAE 1   /* PPO.calculate_returns, xagents/ppo/agent.py:48-94 */
#define XA_RETURNS_NSTEP 2 /* A2C.calculate_returns, xagents/a2c/agent.py:141-171 */

/* action distributions of the actor-critic heads (A2C.get_distribution, a2c/agent.py:54-63) */
#define XA_DIST_CATEGORICAL 0
#define XA_DIST_DIAG_GAUSSIAN 1

/* loss kinds of the fused actor-critic gradient */
#define XA_LOSS_PPO 0 /* PPO.update_gradients, xagents/ppo/agent.py:96-137 */
#define XA_LOSS_A2C 1 /* A2C.train_step, xagents/a2c/agent.py:190-218 */

int xa_abi_version(void);
const char* xa_last_error(void);
/* Hash of the sources the library was built from (xagents_amd/_build.py source_hash()). */
const char* xa_build_hash(void);

/* Number of parameters of the actor-critic MLP (obs -> 64 -> 64 -> {A, 1}). */
int xa_mlp_param_count(int obs_dim, int n_actions);

/* Increment a device-side u64 counter (RNG stream position) by one. */
int xa_counter_bump(uint64_t* counter, void* stream);

/*
 * GAE returns. Replaces PPO.calculate_returns (xagents/ppo/agent.py:48-94).
 *   rewards [N,T], values [N,T], dones [N,T+1] (dones[:,0] = carried-in flags,
 *   dones[:,t+1] = done returned by step t, as A2C.get_batch records them,
 *   xagents/a2c/agent.py:116,129,138), next_values [N] = V(get_states()).
 *   returns [N,T] = GAE advantages + values.
 *   gamma_lam must be (float)((double)gamma * (double)lam): the reference forms
 *   gamma*lam as a Python float product before the f32 multiply.
 * Bit-exact with the reference numpy f32 arithmetic (LDS-staged, one lane per env).
 */
int xa_gae(const float* rewards, const float* values, const float* dones,
           const float* next_values, float* returns, int n_envs, int n_steps, float gamma,
           float gamma_lam, void* stream);

/*
 * n-step discounted returns. Replaces A2C.calculate_returns
 * (xagents/a2c/agent.py:141-171): R_T = V(s_T); R_t = r_t + gamma*R_{t+1}*(1-d_{t+1}).
 * Same layouts as xa_gae. Bit-exact with the reference f32 arithmetic.
 */
int xa_nstep_returns(const float* rewards, const float* dones, const float* next_values,
                     float* returns, int n_envs, int n_steps, float gamma, void* stream);

/*
 * Fused vectorized rollout: n_steps x (policy forward -> Categorical sample ->
 * log-prob/entropy/value -> env step -> store) for every env, plus the bootstrap
 * value V(s_T) and (optionally) the returns. One wave64 per env.
 * Replaces: A2C.get_batch (xagents/a2c/agent.py:96-139), A2C.get_model_outputs
 * (a2c/agent.py:65-94), BaseAgent.step_envs (xagents/base.py:388-426) and the
 * return computation (ppo/agent.py:48-94 or a2c/agent.py:141-171).
 * Reference quirks reproduced: the policy input of step t+1 is the PRE-reset
 * observation returned by step t (a2c/agent.py:132-136); the carried state
 * (env_state) and the bootstrap use the POST-reset state (base.py:424,
 * ppo/agent.py:72).
 * Sampling: action = first a with u * sum_k e_k < cumsum(e)_a, e_k =
 * exp(logit_k - max), u from `uniforms` [N,T] if given, else Philox4x32-10 keyed
 * by seed at counter (env, t, *rng_counter).
 */
typedef struct XaRolloutArgs {
  int n_envs, n_steps, obs_dim, n_actions;
  const float* theta; /* flat actor-critic parameters */

  int env_kind;           /* XA_ENV_REPLAY / XA_ENV_CARTPOLE */
  float* env_state;       /* [N,obs] post-reset current observation (BaseAgent.states) */
  double* env_state64;    /* [N,4]   CartPole internal f64 state (cartpole only) */
  float* env_done;        /* [N]     last done flags (BaseAgent.dones) */
  int* env_cursor;        /* [N]     replay position / elapsed episode steps */
  float* ep_return;       /* [N]     running episode return (BaseAgent.episode_rewards) */
  const float* rep_obs;   /* [N,t_rec,obs] obs returned by env.step at replay position p */
  const float* rep_state; /* [N,t_rec,obs] state after step p (post-reset if done) */
  const float* rep_rew;   /* [N,t_rec] */
  const float* rep_done;  /* [N,t_rec] 0/1 */
  int t_rec;
  int max_episode_steps;  /* CartPole TimeLimit (500 for v1) */

  const float* uniforms;  /* [N,T] or NULL */
  uint64_t seed;
  const uint64_t* rng_counter; /* device u64, read-only here */

  float* obs_out;   /* [N,T,obs] policy inputs (A2C.get_batch `states`) */
  int* act_out;     /* [N,T] */
  float* logp_out;  /* [N,T] */
  float* val_out;   /* [N,T] */
  float* ent_out;   /* [N,T] or NULL */
  float* rew_out;   /* [N,T] */
  float* done_out;  /* [N,T+1] */
  float* epret_out; /* [N,T] running episode return after step t, or NULL */
  float* next_val;  /* [N] V(post-reset s_T) */
  float* ret_out;   /* [N,T] or NULL */
  int return_kind;  /* XA_RETURNS_* */
  float gamma, gamma_lam;
} XaRolloutArgs;

int xa_mlp_rollout(const XaRolloutArgs* args, void* stream);

/*
 * Batched actor-critic forward (A2C.get_model_outputs, a2c/agent.py:65-94) over
 * an arbitrary batch: logits, value, and either the log-prob of given actions
 * (actions_in != NULL) or a sampled action (uniforms [B] required).
 * Same arithmetic as the rollout. Outputs may be NULL when not wanted.
 */
int xa_mlp_forward(const float* theta, const float* obs, int batch, int obs_dim, int n_actions,
                   const int* actions_in, const float* uniforms, int* actions_out, float* logp,
                   float* value, float* entropy, float* logits, void* stream);

/*
 * Minibatch shuffle spec (replaces tf.random.shuffle + slicing,
 * ppo/agent.py:139-155). If perm != NULL it holds epochs x batch indices (host
 * permutations, parity mode). Otherwise a keyed Feistel permutation of [0,batch)
 * per epoch, keyed by (seed, *rng_counter, epoch).
 */
typedef struct XaShuffle {
  const int* perm;
  uint64_t seed;
  const uint64_t* rng_counter;
} XaShuffle;

/*
 * PPO minibatch preparation for a whole train step (ppo/agent.py:139-155, 180-183):
 * for every (epoch e, minibatch m) the shuffled sample indices, and
 *  - stats[((e*n_mb + m)*n_chunks + c)*2 + {0,1}] = f64 (sum adv, sum adv^2) of
 *    1024-sample chunk c, adv = returns - values, n_chunks = ceil(mb_size/1024)
 *    (xa_ppo_adv_stats_size doubles). The sums are linear: all-reduce the array
 *    across ranks for exact global normalisation.
 *  - if mb_obs != NULL, the gather: row e*batch + m*mb_size + q of mb_* holds
 *    sample q of minibatch (e, m) (all minibatches materialised up front, as the
 *    reference's get_mini_batches does).
 */
typedef struct XaMinibatchArgs {
  int batch, mb_size, epochs, obs_dim;
  XaShuffle shuffle;
  const float* returns; /* [batch] */
  const float* values;  /* [batch] */
  const float* obs;     /* [batch, obs] (gather sources, NULL for stats only) */
  const int* actions;
  const float* old_logp;
  double* stats;
  float* mb_obs;       /* [epochs*batch, obs] */
  int* mb_actions;     /* [epochs*batch] */
  float* mb_old_logp;
  float* mb_values;
  float* mb_returns;
} XaMinibatchArgs;

int xa_ppo_adv_stats_size(int batch, int mb_size, int epochs);
int xa_ppo_minibatches(const XaMinibatchArgs* args, void* stream);

/* Keras Adam hyper-parameters + tf.clip_by_global_norm (a2c/agent.py:217,
 * ppo/agent.py:135-137, utils/common.py:476). grad_scale multiplies the gradient
 * before the norm (1 when the loss is already scaled by the global count). */
typedef struct XaAdam {
  float lr, beta1, beta2, eps;
  float clip_norm; /* <= 0: no clipping */
  float grad_scale;
} XaAdam;

/*
 * Fused [pending optimizer step] + minibatch gather + actor-critic forward + loss +
 * backward. Writes per-block partial gradients [n_blocks, P] (reduce with
 * xa_grad_reduce) and per-block loss sums [n_blocks, 4] (pg, value, entropy, count)
 * when loss_partials != NULL.
 * Pending step (pend_grad != NULL): every block first applies clip + Keras Adam with
 * t = *adam_step to (theta, pend_m, pend_v, pend_grad) -- identical arithmetic in
 * every block -- trains on the result, and block 0 stores it to theta_out / m_out /
 * v_out (ping-pong buffers, never aliasing the inputs). This folds minibatch k-1's
 * optimizer step into minibatch k's launch.
 */
typedef struct XaAcGradArgs {
  int obs_dim, n_actions;
  int loss_kind; /* XA_LOSS_PPO / XA_LOSS_A2C */
  const float* theta;
  int batch;    /* rollout batch N*T (flat, env-major) */
  int mb_size;  /* minibatch size (PPO) or batch (A2C) */
  int epoch, mb_index;
  XaShuffle shuffle; /* ignored for A2C (identity order) and when gathered */
  int gathered;      /* 1: inputs are xa_ppo_minibatches' mb_* rows */
  const float* obs;        /* [batch, obs] */
  const int* actions;      /* [batch] */
  const float* old_logp;   /* [batch] (PPO) */
  const float* old_values; /* [batch] */
  const float* returns;    /* [batch] */
  const double* adv_stats; /* xa_ppo_minibatches stats (PPO) */
  double adv_count;        /* number of samples the stats were summed over (global) */
  const float* adv_in;     /* [batch] precomputed (already normalised) advantages, or NULL */
  float clip_norm, entropy_coef, value_coef, adv_eps;
  float loss_scale; /* 1 / global minibatch size */
  int n_blocks;
  float* partials;      /* [n_blocks, P] */
  float* loss_partials; /* [n_blocks, 4] or NULL */
  const float* pend_grad; /* pending optimizer step, or NULL */
  const float* pend_m;
  const float* pend_v;
  float* theta_out;
  float* m_out;
  float* v_out;
  const int* adam_step;
  XaAdam adam;
} XaAcGradArgs;

int xa_ac_grad(const XaAcGradArgs* args, void* stream);
int xa_ac_grad_blocks(int mb_size);

/* grad[p] = sum_b partials[b*P + p] (f64 accumulation, fixed order). If adam_step
 * != NULL it is incremented by one (Keras `iterations`): the following optimizer
 * step (xa_clip_adam or a peer all-reduce tail) uses the new value as t. */
int xa_grad_reduce(const float* partials, int n_parts, int n_params, float* grad,
                   int* adam_step, void* stream);

/*
 * Optimizer tail run by the LAST workgroup of a gradient-producing kernel (elected
 * with the self-resetting `arrivals` counter, a zeroed u32): clip + Keras Adam of the
 * complete gradient, in place on theta/m/v, with exactly xa_clip_adam's arithmetic
 * and norm order (so bit-identical to xa_grad_reduce + xa_clip_adam). t = *adam_step,
 * incremented first when bump != 0. n_params <= XA_ADAM_TAIL_MAX_PARAMS.
 */
#define XA_ADAM_TAIL_MAX_PARAMS 65536
typedef struct XaAdamTail {
  float* theta;
  float* m;
  float* v;
  int* adam_step;
  int bump;
  unsigned* arrivals;
  float* gnorm_out; /* optional pre-clip global norm */
  XaAdam adam;
} XaAdamTail;

/* xa_grad_reduce whose last block applies `tail` (one launch per optimizer step). */
int xa_grad_reduce_adam(const float* partials, int n_parts, int n_params, float* grad,
                        const XaAdamTail* tail, void* stream);

/*
 * g' = grad * grad_scale; if clip_norm > 0: tf.clip_by_global_norm(g', clip_norm)
 * (a2c/agent.py:217, ppo/agent.py:135-136); then Keras Adam (OptimizerV2,
 * training_ops ApplyAdam): m += (g-m)(1-b1); v += (g^2-v)(1-b2);
 * theta -= (m*alpha)/(sqrt(v)+eps), alpha = lr*sqrt(1-b2^t)/(1-b1^t), t = *adam_step.
 * Results go to theta_out/m_out/v_out (NULL = in place). workspace: >= 1024 doubles
 * (used when n_params > 65536). gnorm_out (device f32, optional): pre-clip norm.
 */
int xa_clip_adam(float* theta, float* adam_m, float* adam_v, const float* grad, int n_params,
                 float grad_scale, float clip_norm, float lr, float beta1, float beta2,
                 float eps, const int* adam_step, double* workspace, float* gnorm_out,
                 float* theta_out, float* m_out, float* v_out, void* stream);

/*
 * Persistent PPO update: EVERY optimizer step of one train step in ONE launch.
 * Replaces PPO.get_mini_batches + run_ppo_epochs + update_gradients
 * (xagents/ppo/agent.py:96-191): for epoch e, minibatch m (k = e*n_mb + m, n_mb =
 * ceil(batch/mb_size), ragged last minibatch as range(0, batch, mb_size) slices it;
 * E*n_mb <= 128):
 * the shuffled samples (XaShuffle, the same permutation as xa_ppo_minibatches),
 * advantage normalisation with the minibatch's mean / population std
 * (ppo/agent.py:180-183), clipped PPO loss + backward (as xa_ac_grad), global-norm clip
 * and Keras Adam with t = *adam_step + k + 1 -- the arithmetic of the per-minibatch
 * chain xa_ppo_minibatches -> [xa_ac_grad -> xa_grad_reduce] x E*M -> xa_clip_adam,
 * up to the f64 summation order of the gradient and advantage sums.
 * In place on theta / adam_m / adam_v; *adam_step += E*M. Data parallel (dp_world > 1,
 * below): the cross-rank exchange runs inside the launch.
 * n_blocks: xa_ppo_update_blocks(obs_dim, n_actions, mb_size) (every block must be
 * resident at once: the blocks exchange gradient rows inside the launch), at most one
 * per 16 samples of a minibatch. More blocks than 32-sample tiles select 16-sample
 * tiles (the default for minibatches of <= 512 samples). Grids of < 64 blocks run
 * XCD-local when 8 x n_blocks blocks fit the device: 8 x n_blocks workgroups are
 * launched, the n_blocks that land first on one XCD do the update and keep every
 * hand-off in that XCD's L2, the rest leave at once (placement: XA_PPO_PLACE_*).
 * workspace: device memory, 256-byte aligned, >= xa_ppo_update_workspace_bytes(...),
 * owned by the caller, ZEROED ONCE at allocation and then reused by every launch
 * (nothing in it is reset between launches: a launch counter kept in it numbers the
 * launches, and the exchange words carry tags unique per launch and step).
 * loss_out (optional) [E*n_mb, n_blocks, 4]: per-block (pg, value, entropy, count) sums.
 * grad_out (optional) [P]: the last optimizer step's reduced gradient (before the clip).
 * status (optional device int): set to 1 if an in-launch exchange timed out (10 s per
 * hop); the parameters are then invalid. adam.grad_scale is not used (must be 1).
 * theta_trace / grad_trace (optional, diagnostic) [E*n_mb, P]: theta at the start of
 * every optimizer step k and step k's reduced gradient (before the clip).
 */
#define XA_PPO_DP_MAX 16
#define XA_PPO_STATS_SLOTS 16 /* host slots of the in-launch episode statistics */
#define XA_PPO_PLACE_AUTO 0   /* XCD-local when eligible; not for data-parallel launches */
#define XA_PPO_PLACE_SPREAD 1 /* never XCD-local */
#define XA_PPO_PLACE_LOCAL 2  /* XCD-local when eligible, data parallel included (every
                                 rank on its own GPU) */
typedef struct XaPpoUpdateArgs {
  int obs_dim, n_actions;
  int batch, mb_size, epochs;
  XaShuffle shuffle;
  const float* obs;        /* [batch, obs] env-major rollout (concat_step_batches order) */
  const int* actions;      /* [batch] */
  const float* old_logp;   /* [batch] */
  const float* old_values; /* [batch] */
  const float* returns;    /* [batch] */
  float clip_norm, entropy_coef, value_coef, adv_eps;
  float* theta;
  float* adam_m;
  float* adam_v;
  int* adam_step;
  XaAdam adam;
  void* workspace;
  size_t workspace_bytes;
  float* loss_out;
  float* grad_out;
  int* status;
  int n_blocks;
  int bump_counter; /* nonzero: the launch ends with *shuffle.rng_counter += 1 (the
                       xa_counter_bump that follows the update in a train step) */
  /* data parallel (dp_world > 1; one process per GPU, each with its own env shard and
   * batch): per minibatch the advantage sums, and per optimizer step every workgroup's
   * reduced gradient slice, are exchanged inside the launch through the ranks' exchange
   * blocks (uncached, IPC-mapped into every rank, zeroed once; dp_blocks[r] = rank r's,
   * each >= xa_ppo_update_dp_block_bytes) and summed in rank order, so every rank applies
   * the step of the union of the ranks' minibatches (the all_reduce(SUM) of SURVEY 8e).
   * Every rank must launch with the same shapes and n_blocks, and all ranks' workgroups
   * must be resident at once. */
  int dp_world, dp_rank;
  void* dp_blocks[XA_PPO_DP_MAX];
  int placement;      /* XA_PPO_PLACE_* */
  float* theta_trace; /* optional diagnostic outputs (above) */
  float* grad_trace;
  /* episode statistics to the host inside the launch (replaces the xa_copy_to_host launch
   * of a train step): stats_words (> 0) 32-bit words of stats_src (device: the rollout's
   * done flags / running returns / this status word, as the caller packs them) are
   * stored into stats_dst[g % XA_PPO_STATS_SLOTS] (device pointers of mapped pinned host
   * buffers of stats_words + 1 words), g = the launch number kept in the workspace (0 for
   * the first launch on a zeroed workspace), and word stats_words of that buffer receives
   * g. The words are copied when the launch starts (the status word as the previous
   * launches left it). stats_words = 0: nothing. The host may keep up to
   * XA_PPO_STATS_SLOTS - 1 launches in flight before it folds the oldest slot (several
   * train steps per hipGraph replay). */
  const void* stats_src;
  void* stats_dst[XA_PPO_STATS_SLOTS];
  int stats_words;
} XaPpoUpdateArgs;

int xa_ppo_update_blocks(int obs_dim, int n_actions, int mb_size);
size_t xa_ppo_update_workspace_bytes(int obs_dim, int n_actions, int batch, int mb_size,
                                     int epochs, int n_blocks);
size_t xa_ppo_update_dp_block_bytes(int obs_dim, int n_actions, int batch, int mb_size,
                                    int epochs, int n_blocks, int world);
int xa_ppo_update(const XaPpoUpdateArgs* args, void* stream);

/* ------------------------------------------------------------------------- */
/* Dense / Conv1D building blocks (CNN cfgs: xagents/dqn/models/cnn.cfg,      */
/* xagents/ppo/models/cnn-actor-critic.cfg; TD3/DDPG MLPs in td3/models)     */
/* ------------------------------------------------------------------------- */
#define XA_ACT_NONE 0
#define XA_ACT_RELU 1
#define XA_ACT_TANH 2

/*
 * f32 GEMM with grouped-affine operand addressing (gemm.hip):
 *   C(m, n) = [C(m, n) +] act(sum_k A(m, k) B(k, n) + bias[n]) * [gate(m, n) > 0]
 *   A(m, k) = a[f(m) + g(k)], f(m) = (m / a_pm) a_rm + (m % a_pm) a_sm,
 *                             g(k) = (k / a_pk) a_rk + (k % a_pk) a_sk
 *   B(k, n) = b[k b_ks + n b_ns];  C(m, n) = c[m ldc + n];  gate(m, n) = gate[m ld_gate + n]
 * a == NULL means A = 1 (column sums of B, e.g. bias gradients). a_u8: A holds uint8
 * pixels scaled as f32(x) / 255 (xagents/base.py:505-506). Keras Conv1D on (B,H,W,C)
 * input is a_pm = W_out, a_rm = W_in C, a_sm = stride C, g(k) = k.
 * splits > 1 splits K over workgroups; partials (>= xa_gemm_workspace_floats) holds
 * the split sums, reduced in fixed order (deterministic).
 */
typedef struct XaGemmArgs {
  int M, N, K;
  const void* a;
  int a_u8;
  int64_t a_pm, a_rm, a_sm, a_pk, a_rk, a_sk;
  const float* b;
  int64_t b_ks, b_ns;
  float* c;
  int64_t ldc;
  int splits;
  float* partials;
  const float* bias;
  int act;
  const float* gate;
  int64_t ld_gate;
  int beta;
  int force_small; /* 1: always the 64 x 64 small-tile kernel; 2: the generic tile kernels,
                     never the small-M ones; 3: every path but the few-column row-dot one
                     (tests / A-B timing) */
  int a_ones_row; /* 1: A's last row (m = M - 1) is all ones and is not read: a weight
                     gradient X^T dZ and its bias gradient 1^T dZ as ONE GEMM into the
                     contiguous [W; b] block (the 64 x 64 kernel only: xa_gemm_shape) */
} XaGemmArgs;

int xa_gemm(const XaGemmArgs* args, void* stream);

/* Keras Adam (training_ops ApplyAdam, utils/common.py:476) applied in a weight-gradient
 * GEMM's epilogue: DQN's update minimizes the MSE with no gradient clip
 * (dqn/agent.py:158-171), so a layer's Adam step needs only its own gradient and the
 * gradient never has to leave the GEMM. Element (m, n) of C, at offset e = m ldc + n, is
 * the gradient of the parameter theta[e] with moments m[e], v[e]; t = *step (already
 * bumped, xa_adam_step_bump), g scaled by grad_scale. */
typedef struct XaAdamApply {
  float* theta;
  float* m;
  float* v;
  const int* step;
  float lr, beta1, beta2, eps, grad_scale;
} XaAdamApply;

/* C = A B as xa_gemm (the 64 x 64 kernel, one K split: a dense layer's [W; b] weight
 * gradient X^T dZ with a_ones_row, A m-major, B n-major f32, N and ldc multiples of 4, no
 * bias / activation / gate / beta), then the Adam step of every element in the epilogue;
 * args->c (optional, may be NULL) receives the raw gradient. Replaces the dense layer's
 * share of tape.gradient + Adam.apply_gradients (dqn/agent.py:170-171). */
int xa_gemm_adam(const XaGemmArgs* args, const XaAdamApply* adam, void* stream);

/* The backward of a row-dot-shaped head (the last Dense of the DQN / actor-critic cfgs, A <= 8
 * outputs over K <= 4096 hidden units, utils/common.py:239-258) in ONE launch: its input
 * gradient dx[m][k] = (sum_a dz[m][a] W[k][a]) * [gate[m][k] > 0] (xa_gemm's few-k path:
 * the same k-order fmaf chain, so the same values; += when beta) and its [W; b] gradient
 * gw[k][a] (+)= sum_m x[m][k] dz[m][a], gb[a] (+)= sum_m dz[m][a] (m-order fmaf chains; gw,
 * gb = NULL: none). x, dz, dx rows of K / A / K floats (ld = K / A / K), W (K, A) in Keras
 * layout, gate rows of K (NULL: none). */
int xa_head_bwd(const float* x, const float* dz, const float* W, const float* gate, int M, int K,
                int A, float* dx, int beta, float* gw, float* gb, int accumulate, void* stream);

/* The NatureCNN convolution stack's forward in one launch (the three Conv1D layers of
 * the cnn .cfg models (xagents/dqn/models/cnn.cfg, the ppo / a2c / acer
 * cnn-actor-critic.cfg) as built by xagents/utils/common.py:225-240 over (84, 84, 1)
 * frames: 32 x 8 / 4, 64 x 4 / 2, 64 x 3 / 1, ReLU; Keras convolves each 84-pixel frame row
 * separately). rows = frames x 84; x [rows][84] uint8 (/ 255, x_u8) or f32; w1 [8][32],
 * w2 [4][32][64], w3 [3][64][64] (Keras kernel order), biases; outputs h1 [rows][20][32],
 * h2 [rows][9][64] (optional, NULL skips: kept for the backward) and h3 [rows][7][64]
 * (the flattened 37632-float features per frame). Same values as three xa_gemm launches
 * up to f32 association. */
typedef struct XaConvStackArgs {
  const void* x;
  int x_u8;
  int rows;
  const float *w1, *b1, *w2, *b2, *w3, *b3;
  float *h1, *h2, *h3;
} XaConvStackArgs;
int xa_conv_stack_fwd(const XaConvStackArgs* args, void* stream);

/* The stack's backward in one launch + a fixed-order reduce: from dz3 = dL/d(conv3
 * pre-activation) [rows][7][64] (h3's ReLU gate applied), the forward's h1 / h2 and the
 * frames, the gradient of the stack's 20896 parameters [w1 b1 w2 b2 w3 b3] (Keras variable
 * order, contiguous in theta) into grad (+= when accumulate); no input gradient (the input
 * is the frame). ws: xa_conv_stack_bwd_workspace_floats(rows) floats. Same values as the
 * per-layer weight-gradient / transposed-conv GEMMs up to f32 association. */
typedef struct XaConvStackBwdArgs {
  const void* x;
  int x_u8;
  int rows;
  const float *w2, *w3;
  const float *h1, *h2, *dz3;
  float* ws;
  size_t ws_floats;
  float* grad;
  int accumulate;
  /* optional, for an update without a gradient clip (DQN, dqn/agent.py:158-171): adam_on = 1
   * applies Keras Adam (`adam`: theta / m / v / step of the stack's first parameter, t already
   * bumped) to the stack's parameters inside the reduce launch, the raw gradient written to
   * grad only when write_grad (accumulate must be 0); n_rest > 0 also applies Adam (`rest`)
   * to n_rest more parameters whose gradient rest_grad is final when this launch runs (the
   * Q head's): the xa_clip_adam launches of those ranges folded into the reduce */
  int adam_on;
  int write_grad;
  XaAdamApply adam;
  XaAdamApply rest;
  const float* rest_grad;
  int n_rest;
} XaConvStackBwdArgs;
size_t xa_conv_stack_bwd_workspace_floats(int rows);
int xa_conv_stack_bwd(const XaConvStackBwdArgs* args, void* stream);
int xa_gemm_splits(int M, int N, int K);
/* the kernel shape xa_gemm picks for a tile-path GEMM with `splits` K splits (0 = the
 * 64 x 64 kernel, the only one that takes a_ones_row) */
int xa_gemm_shape(int M, int N, int K, int splits);
size_t xa_gemm_workspace_floats(int M, int N, int K, int splits);

/* Keras Conv1D input gradient (col2im as a fixed-order gather):
 *   dinput[row][q][c] = sum over taps t, positions p with s p + t = q of
 *                       dcol[(row P + p) (k C) + t C + c],  times [gate[row][q][c] > 0]
 * dcol = dY W^T in im2col layout [rows P, k C]; gate = the ReLU output of the layer that
 * produced the input (NULL: no gate). */
int xa_conv1d_input_grad(const float* dcol, int rows, int positions, int kernel, int stride,
                         int channels, int width_in, const float* gate, float* dinput,
                         void* stream);

/* Keras Conv1D input gradient in one launch (an implicit transposed-convolution GEMM; the
 * tape.gradient through the Conv1D layers built at xagents/utils/common.py:231-237):
 *   dinput[row][q][c] = (sum over taps t, positions p with s p + t = q, filters f of
 *                        dy[row][p][f] kernel[t][c][f]) * [gate[row][q][c] > 0]
 * dy [rows, P, F], kernel [k, C, F] (the Keras Conv1D kernel layout), dinput [rows, W_in, C].
 * Same value as xa_gemm (dY W^T) + xa_conv1d_input_grad without the im2col buffer. Needs
 * F % 4 == 0 and 16-byte aligned dy / kernel. */
int xa_conv1d_dgrad(const float* dy, const float* kernel, int rows, int positions, int ksize,
                    int stride, int channels, int filters, int width_in, const float* gate,
                    float* dinput, void* stream);

/* Keras Conv1D weight and bias gradient of a narrow layer (ksize * channels <= 8, filters a
 * power of two in [4, 64]; NatureCNN's first layer on single-channel frames) in one pass
 * over dY (the gradient tape of common.py:231-237):
 *   dw[t][c][f] (+)= sum_{row, p} x[row][p stride + t][c] dy[row][p][f],
 *   db[f]       (+)= sum_{row, p} dy[row][p][f]
 * x [rows, width_in, channels] f32 or uint8 (x_u8: scaled f32(x) / 255, base.py:505-506),
 * dy [rows, positions, filters] (16-byte aligned). accumulate = 1 adds to dw / db.
 * workspace: xa_conv1d_wgrad_workspace_floats(...) floats (0 = shape not supported). */
size_t xa_conv1d_wgrad_workspace_floats(int ksize, int channels, int filters);
int xa_conv1d_wgrad(const void* x, int x_u8, const float* dy, int rows, int width_in,
                    int channels, int positions, int ksize, int stride, int filters, float* dw,
                    float* db, int accumulate, float* workspace, size_t workspace_floats,
                    void* stream);

/* TRPO (xagents/trpo/agent.py). xa_trpo_head: per sample of Categorical(logits_new) vs
 * Categorical(logits_old) (calculate_losses / calculate_kl_divergence, trpo/agent.py:179-223):
 * ratio = exp(logp_new(a) - logp_old(a)), KL(old || new), entropy H(new); with dlogits, the
 * gradient of surrogate_loss = mean(ratio adv) + entropy_coef mean(H) w.r.t. logits_new
 * (times inv_n = 1 / n). partials: [xa_trpo_head_blocks(n), 3] f64 block sums; out (optional)
 * receives [surrogate_loss, mean KL, mean H] as f32. */
typedef struct XaTrpoHeadArgs {
  int n, n_actions;
  const float* logits_new;
  const float* logits_old;
  int64_t ld_logits;
  const int* actions;
  const float* advantages;
  float entropy_coef, inv_n;
  float* dlogits;
  int64_t ld_dlogits;
  double* partials;
} XaTrpoHeadArgs;

int xa_trpo_head_blocks(int n);
int xa_trpo_head(const XaTrpoHeadArgs* args, float* out, void* stream);

/* out[i][a] = scale p_a (t_a - sum_b p_b t_b), p = softmax(logits[i]): the Categorical Fisher
 * metric on a logit tangent, the middle factor of the Fisher-vector product
 * (TRPO.calculate_fvp, trpo/agent.py:121-148, evaluated where actor == old actor). */
int xa_categorical_fisher(const float* logits, int64_t ld_logits, const float* tangent,
                          int64_t ld_tangent, int n, int n_actions, float scale, float* out,
                          int64_t ld_out, void* stream);

/* Conjugate-gradient vector algebra (TRPO.conjugate_gradients, trpo/agent.py:150-177):
 * *out = sum x y (f64, fixed order); out = a x + b y (f32, out may alias x or y). */
int xa_vec_dot(const float* x, const float* y, int64_t n, double* out, void* stream);
int xa_axpby(float a, const float* x, float b, const float* y, float* out, int64_t n,
             void* stream);

/* adv = ((returns - values) - mean) / (std + eps) over the whole batch, population std
 * (TRPO.train_step, trpo/agent.py:321-324: tf.reduce_mean / tf.math.reduce_std, eps 0). */
int xa_normalized_advantages(const float* returns, const float* values, int n, float eps,
                             float* adv, void* stream);

/* DQN.get_actions (xagents/dqn/agent.py:107-116): actions[i] = tf.argmax(q[i]) (first max),
 * or random_actions[i] when use_random (the host draws np.random.random() < epsilon and
 * np.random.randint(0, A, n) exactly as the reference). */
int xa_dqn_act(const float* q, int n, int n_actions, const int* random_actions, int use_random,
               int* actions, void* stream);

/* DQN.get_targets + update_gradients loss (dqn/agent.py:118-171): y = v' gamma + r with
 * v' = max_a Qt(s') (or Qt(s')[argmax Q(s')] when q_next_online != NULL), 0 where done;
 * MSE over actions, summed over the batch by minimize: dq[b][a_b] = -2 (y - q[b][a_b]) / A,
 * 0 elsewhere; loss[b] (optional) = (y - q[b][a_b])^2 / A.
 * huber_delta > 0 (opt-in, not in the reference -- BASELINE north_star's Huber-TD loss):
 * tf.keras.losses.Huber(delta) in place of MSE, x = y - q[b][a_b]:
 * dq[b][a_b] = -clip(x, -delta, delta) / A, loss[b] = huber(x) / A. <= 0: MSE (parity).
 * adam_step (optional): the Keras optimizer's iteration counter, bumped by one in the same
 * launch (the update's t += 1 before its Adam step, without a launch of its own). */
int xa_dqn_td_grad(const float* q, const float* q_next_target, const float* q_next_online,
                   const int* actions, const float* rewards, const float* dones, int batch,
                   int n_actions, float gamma, float huber_delta, float* dq, float* loss,
                   int* adam_step, void* stream);

/* The Q head (the last dense layer, N <= 8 actions: xa_gemm's row-dot shape) with DQN's
 * per-row step fused into the same launch. mode 0: actions[m] = first argmax of row m
 * (xa_dqn_act's greedy branch); mode 1: the head is the TARGET network's over s', and row b
 * finishes xa_dqn_td_grad's arithmetic for sample b (q = the online Q [B][A], q_next_online
 * for double DQN or NULL, act / rewards / dones, gamma, huber, dq / loss outputs, adam_step
 * bumped). args->c still receives the head's Q values. */
typedef struct XaDqnHeadArgs {
  int mode;
  int* actions;
  const float* q;
  const float* q_next_online;
  const int* act;
  const float* rewards;
  const float* dones;
  float gamma, huber;
  float* dq;
  float* loss;
  int* adam_step;
} XaDqnHeadArgs;
int xa_dqn_head(const XaGemmArgs* head, const XaDqnHeadArgs* dqn, void* stream);

/* A split-K dense layer and the row-dot head that reads its output (Keras Dense -> Dense,
 * utils/common.py:239-258: the NatureCNN cfgs' 512-unit hidden layer and their Q head), with
 * DQN's per-row step (dqn = NULL: the plain head; else xa_dqn_head's mode 0 / 1) -- the split
 * partials as xa_gemm launches them, then ONE launch for the split reduce, the dense epilogue
 * (its rows stored to dense->c), the head and the DQN step: the same values as xa_gemm(dense)
 * followed by xa_gemm(head) / xa_dqn_head, bit for bit. Shapes xa_gemm_head_ok accepts (1):
 * dense on xa_gemm's wide split reduce (M N <= 65536, >= 64 splits), N <= 512, no gate /
 * beta; head a row-dot shape (xa_dqn_head's) with head->a == dense->c, lda = dense->ldc,
 * K = dense N, the same M. */
int xa_gemm_head(const XaGemmArgs* dense, const XaGemmArgs* head, const XaDqnHeadArgs* dqn,
                 void* stream);
int xa_gemm_head_ok(const XaGemmArgs* dense, const XaGemmArgs* head);

/* Replay rings (ReplayBuffer1 xagents/utils/buffers.py:59-98, ReplayBuffer2 101-148):
 * ring[slots[i]] = src[i] / dst[i] = ring[slots[i]] for items of item_bytes. The host
 * computes slots with the reference's index semantics (deque order + random.sample for
 * RB1, current_size % size with the row-0 overwrite + np.random.randint for RB2). */
int xa_ring_scatter(const void* src, void* ring, const int64_t* slots, int n_items,
                    int64_t item_bytes, void* stream);
int xa_ring_gather(const void* ring, void* dst, const int64_t* slots, int n_items,
                   int64_t item_bytes, void* stream);

/* Every field of one sampled batch in one launch: dst_f[i] = ring_f[slots[i]] for the
 * n_fields (<= XA_GATHER_MAX_FIELDS) rings of concat_buffer_samples' [states, actions,
 * rewards, dones, new_states] (xagents/base.py:344-368), one slot list for all of them. */
#define XA_GATHER_MAX_FIELDS 8
typedef struct XaGatherField {
  const void* ring;
  void* dst;
  int64_t item_bytes;
} XaGatherField;
typedef struct XaGatherArgs {
  XaGatherField field[XA_GATHER_MAX_FIELDS];
  int n_fields;
  int n_items;
  const int64_t* slots;
} XaGatherArgs;
int xa_ring_gather_fields(const XaGatherArgs* args, void* stream);

/* dst = (1 - tau) dst + tau src (DDPG.sync_target_models, xagents/ddpg/agent.py:73-85);
 * tau = 1 copies (DQN.sync_target_model, dqn/agent.py:97-105). */
int xa_polyak(const float* src, float* dst, int64_t n, float tau, void* stream);

/*
 * Off-policy device env step over a pre-recorded transition stream, fused with the
 * replay-ring append: BaseAgent.step_envs(actions, store_in_buffers=True)
 * (xagents/base.py:388-426). Per env i with cursor c:
 *   new_state = rep_obs[i][c] (pre-reset obs), reward / done = rep_rew / rep_done[i][c],
 *   ring[i][slot] <- (state[i], actions[i], reward, done, new_state), then
 *   state[i] = rep_state[i][c] (post-reset), cursor = (c + 1) % t_rec.
 * slot: RB1 (deque, buffers.py:59-98) = count % capacity, count += 1;
 *       RB2 (buffers.py:101-148)      = current_size % size, current_size saturating at
 *       size (every append lands on row 0 once full -- the reference's behaviour).
 * Bytes are moved verbatim (uint8 frames or f32 vectors). out_* (optional) receive this
 * step's transition; done_epret[i] = the finished episode's return where done, else 0.
 */
#define XA_RING_DEQUE 0
#define XA_RING_RB2 1

typedef struct XaReplayStepArgs {
  int n_envs, t_rec;
  int64_t obs_bytes;
  const void* rep_obs;
  const void* rep_state;
  const float* rep_rew;
  const float* rep_done;
  void* state;
  int* cursor;
  float* ep_return;
  float* done;
  const void* actions;
  int64_t act_bytes;
  int64_t capacity;
  int ring_kind;
  int64_t* ring_count;
  void* ring_states;
  void* ring_new_states;
  void* ring_actions;
  float* ring_rewards;
  float* ring_dones;
  void* out_states;
  void* out_new_states;
  float* out_rewards;
  float* out_dones;
  float* done_epret;
  int64_t out_ld; /* element stride between envs of out_rewards / out_dones / done_epret
                     (0 = 1; n_steps writes env-major [N, T] rollout rows) */
} XaReplayStepArgs;

int xa_replay_env_step(const XaReplayStepArgs* args, void* stream);

/* AtariWrapper.step / reset on device (xagents/utils/common.py:67-142, the per-env
 * `env.step` + `env.reset` of BaseAgent.step_envs, base.py:388-426, for Atari envs).
 * Raw RGB frames [n_envs, t_raw, height, width, 3] u8; stepping into frame t yields
 * raw_rew[t], raw_done[t]; the frame after a done frame is the env.reset() frame.
 * A step walks `skips` frames from raw_cursor (reward summed, stop at a done), takes the
 * pixelwise max with the previous raw frame when max_frame (the 2-deep frame_buffer),
 * then cv2.cvtColor(COLOR_BGR2GRAY) and cv2.resize(dsize = (out_w, out_h), INTER_LINEAR)
 * in OpenCV's 8-bit fixed point (xofs / alpha / yofs / beta: cv::resize's tables, built by
 * the host). out_step = frame returned by step (pre-reset), out_post = state after
 * step_envs (the reset frame, processed alone, when done). reset_only = 1 processes
 * frames[raw_cursor] alone into out_post (AtariWrapper.reset). */
typedef struct XaAtariStepArgs {
  int n_envs, t_raw, height, width, out_h, out_w;
  const uint8_t* frames;
  const float* raw_rew;
  const float* raw_done;
  int* raw_cursor;
  int skips, max_frame, reset_only;
  const int* xofs;
  const short* alpha;
  const int* yofs;
  const short* beta;
  uint8_t* out_step;
  uint8_t* out_post;
  float* out_rew;
  float* out_done;
} XaAtariStepArgs;

int xa_atari_step(const XaAtariStepArgs* args, void* stream);

/* BipedalWalker-v3 device stand-in: gym's env.step / env.reset of
 * BaseAgent.step_envs (xagents/base.py:388-426, gym call base.py:408) for BipedalWalker ids,
 * with the real env's 24-value observation, 4 motor commands in [-1, 1], reward formula and
 * termination, over a planar kinematic walker on flat ground (not Box2D; csrc/walker.hip).
 * state [n_envs][XA_WALKER_STATE] f32 and episode [n_envs] int are the env's own memory
 * (zeroed, then one reset_only call). A step reads actions [n_envs] rows of 4 f32 at row
 * stride act_ld floats and writes the returned obs (pre-reset) to out_obs, reward and done,
 * and the post-step state's obs (the reset obs when done) to out_post -- the one-step
 * record xa_replay_env_step consumes. reset_only = 1 resets every env into out_post. */
#define XA_WALKER_STATE 18
#define XA_WALKER_OBS 24
typedef struct XaWalkerStepArgs {
  int n_envs;
  float* state;
  int* episode;
  const float* actions;
  int64_t act_ld;
  uint64_t seed;
  int reset_only;
  float* out_obs;
  float* out_post;
  float* out_rew;
  float* out_done;
} XaWalkerStepArgs;

int xa_walker_step(const XaWalkerStepArgs* args, void* stream);

/* Episode statistics to the host (BaseAgent.step_envs bookkeeping, xagents/base.py:388-426):
 * copies n_segments device buffers (bytes a multiple of 4) into pinned host memory in ONE
 * launch on `stream`. dst[i] are the DEVICE addresses of the pinned host buffers, from
 * xa_host_device_pointer. Completion = the stream's next event. */
#define XA_HOST_COPY_MAX 4
typedef struct XaHostCopyArgs {
  int n_segments;
  const void* src[XA_HOST_COPY_MAX];
  void* dst[XA_HOST_COPY_MAX];
  int64_t bytes[XA_HOST_COPY_MAX];
} XaHostCopyArgs;

int xa_copy_to_host(const XaHostCopyArgs* args, void* stream);

/* *dev = the device address of pinned host memory `host` (hipHostGetDevicePointer). */
int xa_host_device_pointer(void* host, void** dev);

/* tf.keras.losses.MSE(target, pred) per row, gradient of the batch sum (minimize on a
 * [B] loss): dpred = 2 (pred - target) / n_out; loss[b] (optional). */
int xa_mse_grad(const float* pred, const float* target, int batch, int n_out, float* dpred,
                float* loss, void* stream);

/* dst[r][c] = src[r][c], rows x cols f32 block (tf.concat([states, actions], 1) and
 * column slices of it). */
int xa_copy_block(const float* src, int64_t ld_src, float* dst, int64_t ld_dst, int rows,
                  int cols, void* stream);

/* out = clip(x + clip(sigma N(0,1), -noise_clip, noise_clip), lo, hi) per element, the
 * normals from Philox4x32-10 (counter *rng_counter, key seed) by Box-Muller; sigma = 0
 * only clips. TD3 target smoothing (td3/agent.py:83-91: sigma 0.2, clip 0.5, [-1, 1]) and
 * DDPG exploration (ddpg/agent.py:60-71: sigma 0.1). TF's RNG stream is not reproduced;
 * noise_out (optional) receives the noise drawn. */
int xa_noisy_actions(const float* x, int64_t ld_x, int rows, int cols, float sigma,
                     float noise_clip, float lo, float hi, const uint64_t* rng_counter,
                     uint64_t seed, float* out, int64_t ld_out, float* noise_out, void* stream);

/* Critic targets + MSE gradients (ddpg/agent.py:104-127; TD3 twin critics
 * td3/agent.py:66-110 when v2/tv2 != NULL): y = r + ((1 - d) gamma) min(tv1, tv2),
 * dv_i = 2 (v_i - y), loss[b] = sum_i (v_i - y)^2.
 * huber_delta > 0 (opt-in Huber-TD, not in the reference): dv_i = clip(v_i - y, +-delta),
 * loss[b] = sum_i huber(v_i - y). <= 0: MSE (parity). */
int xa_critic_td_grad(const float* v1, const float* v2, const float* tv1, const float* tv2,
                      const float* rewards, const float* dones, int batch, float gamma,
                      float huber_delta, float* dv1, float* dv2, float* loss, void* stream);

/* One network of the fused TD3 / DDPG gradient step: the flat Keras-order parameters of a
 * 3-layer .cfg MLP (W1 [in][h1], b1, W2 [h1][h2], b2, W3 [h2][out], b3) and, for the
 * networks that learn, their Keras Adam state (t = *step + 1 this step; the launch adds 1). */
typedef struct XaTdNet {
  float* theta;
  float* m;
  float* v;
  int* step;
  float lr, beta1, beta2, eps;
} XaTdNet;

/* A whole DDPG / TD3 gradient step (DDPG.update_weights' body, ddpg/agent.py:129-147:
 * update_critic_weights 104-127, update_actor_weights 87-102, sync_target_models 73-85;
 * TD3's twin critics + target smoothing, td3/agent.py:66-110) in ONE persistent launch of
 * n_blocks resident workgroups (0: the default) with grid barriers between its phases.
 * Batch rows are the ring rows `slots` [batch] (concat_buffer_samples order) of the f32
 * replay rings (states / new_states [.][obs_dim], actions [.][act_dim], rewards, dones).
 * twin: TD3 (critic 2 + target critic 2); smooth: TD3 target smoothing (Philox normals at
 * (row, column, *rng_counter), key seed, times noise_sigma, clipped to +-noise_clip, the
 * counter advanced by 1 -- the draw of xa_noisy_actions); actor_update: this step updates the
 * actor through the updated critic 1 and Polyak-averages every target (tau). Critic loss
 * Sum_b (v - y)^2 per critic (huber_delta > 0: opt-in Huber-TD), actor loss -mean Q.
 * Outputs: the sampled batch (out_s, out_a, out_r, out_d, out_s2), noise_out [batch][act]
 * (optional), dv1 / dv2 [batch] and the raw gradients g_* (before Adam), loss_out [batch]
 * (optional); parameters, moments and step counters in place. workspace: zeroed once by
 * the caller (xa_td3_update_workspace_bytes), reused by every launch without a reset; a
 * barrier that times out (10 s) sets *status = 1 and the workspace must be re-zeroed;
 * while *status != 0 every launch returns without touching anything.
 * stage 0: the whole step. Data parallel (ranks all-reduce the raw gradients between
 * launches, ddpg/agent.py:104-127 + the rank sum): stage 1 writes the critics' raw gradients
 * (and the sampled batch, the noise, the actor forward on policy steps); stage 2 applies the
 * critics' Adam to g_critic* x critic_grad_scale (+ Polyak of the critic targets on policy
 * steps) and on policy steps writes the actor's raw gradient through the updated critic 1;
 * stage 3 (actor_update = 1) applies the actor's Adam to g_actor x actor_grad_scale + the
 * Polyak of the target actor. Each stage bumps the counters it owns (1: the noise counter,
 * 2: the critics' steps, 3: the actor's step). */
typedef struct XaTd3UpdateArgs {
  int batch, obs_dim, act_dim, h1, h2;
  int twin, smooth, actor_update;
  float gamma, tau, noise_sigma, noise_clip, huber_delta;
  const float* ring_states;
  const float* ring_new_states;
  const float* ring_actions;
  const float* ring_rewards;
  const float* ring_dones;
  const int64_t* slots;
  uint64_t* rng_counter;
  uint64_t seed;
  XaTdNet actor, critic1, critic2, target_actor, target_critic1, target_critic2;
  float* out_s;
  float* out_a;
  float* out_r;
  float* out_d;
  float* out_s2;
  float* noise_out;
  float* dv1;
  float* dv2;
  float* loss_out;
  float* g_actor;
  float* g_critic1;
  float* g_critic2;
  void* workspace;
  size_t workspace_bytes;
  int n_blocks;
  int* status;
  int stage;
  float critic_grad_scale, actor_grad_scale;
} XaTd3UpdateArgs;

size_t xa_td3_update_workspace_bytes(int batch, int obs_dim, int act_dim, int h1, int h2);
int xa_td3_update(const XaTd3UpdateArgs* args, void* stream);

/* The exploration step's actions of DDPG / TD3 in ONE launch (DDPG.get_step_actions,
 * ddpg/agent.py:60-71, with the actor of actor_model.cfg: in -> h1 relu -> h2 relu -> act
 * tanh): out[i][a] = clip(tanh(actor(states[i]))[a] + noise, lo, hi), noise = clip(sigma
 * N(0, 1), +-noise_clip) drawn by Philox4x32-10 at (i, a, *rng_counter, seed) exactly as
 * xa_noisy_actions draws it (noise_out optional); *rng_counter += 1 at the end when bump.
 * theta: the actor's flat Keras-order parameters. Workspace (xa_td3_act_workspace_bytes)
 * zeroed once by the caller and reused by every launch; n <= 256, h1, h2 <= 416 and
 * multiples of 4, act_dim <= 4. */
typedef struct XaTd3ActArgs {
  int n, obs_dim, act_dim, h1, h2;
  const float* states;
  const float* theta;
  float sigma, noise_clip, lo, hi;
  uint64_t* rng_counter;
  uint64_t seed;
  int bump;
  float* out;
  int ld_out;
  float* noise_out;
  void* workspace;
  size_t workspace_bytes;
  int n_blocks;
  int* status;
} XaTd3ActArgs;

size_t xa_td3_act_workspace_bytes(int n, int obs_dim, int act_dim, int h1, int h2);
int xa_td3_act(const XaTd3ActArgs* args, void* stream);

/* TFP Categorical(logits) over n logit rows (A2C.get_model_outputs, a2c/agent.py:65-94):
 * log-prob and entropy of the given actions (actions_in) or of an inverse-CDF sample
 * with uniforms[i] or Philox(i, step, *rng_counter, seed). Same arithmetic as the fused
 * MLP rollout. Outputs (optional) are written at i * ld_out. n_actions <= 64. */
int xa_categorical(const float* logits, int64_t ld_logits, int n, int n_actions,
                   const float* uniforms, const uint64_t* rng_counter, uint64_t seed, int step,
                   const int* actions_in, int* actions_out, float* logp, float* entropy,
                   int64_t ld_out, void* stream);

/* PPO / A2C loss of one minibatch (mean over its n samples) and its gradient w.r.t. the
 * logits and the value head, for models run through xa_gemm (the CNN actor-critic):
 * PPO.update_gradients (ppo/agent.py:96-137) with per-minibatch advantage normalisation
 * (run_ppo_epochs 180-183), A2C.train_step (a2c/agent.py:190-218). loss (optional):
 * [pg, value, entropy] means. */
typedef struct XaHeadGradArgs {
  int n, n_actions, loss_kind;
  const float* logits;
  int64_t ld_logits;
  const float* values;
  int64_t ld_values;
  const int* actions;
  const float* old_logp;
  const float* old_values;
  const float* returns;
  float clip_norm, entropy_coef, value_coef, adv_eps;
  float* dlogits;
  float* dvalues;
  float* loss;
  /* advantage statistics: 0 = this minibatch's own; 1 = only write [sum, sum^2, n] of
   * adv = returns - old_values to adv_stats (then all-reduce them over the ranks);
   * 2 = use the all-reduced adv_stats (the union minibatch's mean / population std) */
  int stats_mode;
  double* adv_stats;
  /* XA_DIST_CATEGORICAL (logits rows, `actions` int) or XA_DIST_DIAG_GAUSSIAN (`logits`
   * rows are the mean of MultivariateNormalDiag(loc) with unit scale, a2c/agent.py:59-60;
   * actions_f [n, ld_actions] f32; dlogits is then d loss / d mean) */
  int dist_kind;
  const float* actions_f;
  int64_t ld_actions;
} XaHeadGradArgs;

int xa_ac_head_grad(const XaHeadGradArgs* args, void* stream);

/* Advantage statistics of every minibatch of a PPO train step in one launch (the
 * per-minibatch normalisation of run_ppo_epochs, ppo/agent.py:157-191, with the
 * minibatches of get_mini_batches 139-155): idx [epochs * batch] holds each epoch's
 * shuffled flat sample indices (epoch e at e * batch, minibatch m at m * mb_size, the last
 * one ragged); out[(e * n_mb + m) * 3 + {0, 1, 2}] = f64 [sum, sum^2, count] of
 * adv = returns[i] - values[i], n_mb = ceil(batch / mb_size). The sums are linear:
 * all-reduce out across data-parallel ranks once per train step, then xa_ac_head_grad
 * stats_mode 2 reads each minibatch's triple. */
int xa_minibatch_adv_sums(const float* returns, const float* values, const int64_t* idx,
                          int batch, int mb_size, int epochs, double* out, void* stream);

/* MultivariateNormalDiag(loc = mu) with unit scale, the reference's distribution for Box
 * action spaces (A2C.get_distribution, a2c/agent.py:54-63): per row i of mu [n, d],
 * actions_out[i] = mu[i] + N(0, I) (noise [n, d] if given, else Philox4x32-10 Box-Muller
 * at (i, step, *rng_counter), key seed; TF's stream is not reproduced), or the log-prob of
 * actions_in; logp[i] = -0.5 |a - mu|^2 - 0.5 d log(2 pi), entropy[i] = 0.5 d (1 +
 * log(2 pi)). Outputs at i * ld_out (optional). */
int xa_diag_gaussian(const float* mu, int64_t ld_mu, int n, int d, const float* noise,
                     const uint64_t* rng_counter, uint64_t seed, int step,
                     const float* actions_in, int64_t ld_act, float* actions_out, float* logp,
                     float* entropy, int64_t ld_out, void* stream);

/* ACER loss gradient of a batch of n_envs trajectories (ACER.update_gradients,
 * xagents/acer/agent.py:295-347; calculate_returns 171-208; calculate_losses 210-260;
 * calculate_grads 262-293). Rows are env-major [n_envs, n_steps + 1] (acer/agent.py:164-169):
 * logits / q / avg_logits are the model's actor (pre-softmax) and critic outputs and the
 * average model's actor output on every row; mu_logits [n_envs, n_steps, A] the behaviour
 * policy's actor logits; actions / rewards / dones [n_envs, n_steps]. Writes dlogits
 * (gradient w.r.t. the pre-softmax logits) and dq for every row (zero on the bootstrap row
 * t = n_steps), the Retrace returns (optional) and per-env loss partials env_loss[n_envs][4]
 * = [sum gain, sum entropy, sum 0.5 (R - Q_a)^2, trust-region adjustments] (optional).
 * n_total = the mean's denominator (this rank's n_envs x n_steps). n_steps <= 4000. */
typedef struct XaAcerArgs {
  int n_envs, n_steps, n_actions, n_total;
  const float* logits;
  int64_t ld_logits;
  const float* q;
  int64_t ld_q;
  const float* avg_logits;
  int64_t ld_avg;
  const float* mu_logits;
  const int* actions;
  const float* rewards;
  const float* dones;
  float gamma, epsilon, importance_c, delta, entropy_coef, value_coef;
  int trust_region;
  float* dlogits;
  int64_t ld_dlogits;
  float* dq;
  int64_t ld_dq;
  float* returns;
  float* env_loss;
} XaAcerArgs;

int xa_acer_grad(const XaAcerArgs* args, void* stream);

/* shadow -= (shadow - var) (1 - decay): tf.train.ExponentialMovingAverage.apply without
 * zero-debias (ACER average model, acer/agent.py:46,114-125,346). */
int xa_ema(float* shadow, const float* var, int64_t n, float decay, void* stream);

/* Keras OptimizerV2 `iterations += 1` on device (before xa_clip_adam reads t). */
int xa_adam_step_bump(int* adam_step, void* stream);

/* dz = dy * act'(y) given the activation OUTPUT y (relu: [y > 0]; tanh: 1 - y^2). */
int xa_activation_grad(const float* y, const float* dy, int64_t n, int act, float* dz,
                       void* stream);

/*
 * One-shot peer all-reduce (SUM) of a small buffer over IPC-shared HBM blocks, for the
 * per-minibatch gradient / advantage-sum exchange of the data-parallel update
 * (the exchange a multi-worker run of ppo/agent.py:136-137 and the
 * global advantage statistics of ppo/agent.py:180-183 need). Each rank owns one block
 * per channel from xa_peer_block_alloc (uncached HBM), exports it with
 * xa_peer_ipc_handle and opens the peers' with xa_peer_ipc_open; blocks[p] = rank p's
 * block as mapped in this process. Every rank pushes (word, epoch) 8-byte pairs into
 * every peer's block and polls its own, then sums in rank order (identical bits on
 * every rank). `state` = xa_peer_state_words(slot_bytes) u32 of ordinary device
 * memory, zeroed, private to the rank: state[0] is a sticky error (0 healthy, 1 + p =
 * timed out waiting for rank p; afterwards calls return the local values without
 * waiting), the rest are per-chunk epochs. Waits are bounded by timeout_ticks of the
 * 100 MHz realtime clock. With has_tail the summed gradient goes straight into the
 * optimizer (XaAdamTail). These are the only entry points that allocate: IPC blocks
 * need the uncached flag.
 */
#define XA_PEER_MAX 16
#define XA_DTYPE_F32 0
#define XA_DTYPE_F64 1

typedef struct XaPeerAllReduceArgs {
  void* blocks[XA_PEER_MAX];
  int rank, world;
  int dtype;
  int64_t count;
  size_t slot_bytes; /* payload capacity per rank the blocks were sized with (multiple of 4096) */
  const void* src;
  void* dst;         /* may equal src (in place) */
  uint32_t* state;
  uint64_t timeout_ticks;
  int has_tail;      /* 1: the last workgroup applies `tail` to dst (f32 gradients) */
  XaAdamTail tail;
} XaPeerAllReduceArgs;

size_t xa_peer_block_bytes(size_t slot_bytes, int world);
int xa_peer_state_words(size_t slot_bytes);
int xa_peer_block_alloc(size_t bytes, void** block);
int xa_peer_block_free(void* block);
int xa_peer_ipc_handle(void* block, void* handle_out /* 64 bytes */);
int xa_peer_ipc_open(const void* handle /* 64 bytes */, void** block);
int xa_peer_ipc_close(void* block);
int xa_peer_allreduce(const XaPeerAllReduceArgs* args, void* stream);

#ifdef __cplusplus
}
#endif
#endif
