// Persistent PPO update: the C-ABI entry points (xa_ppo_update, its block count and
// workspace sizes) and the (obs, actions) = (4, 2) instantiations of the kernel
// (CartPole-v1, the headline shape). The kernel is ppo_update_impl.hpp; the other shapes'
// instantiations are ppo_update_oXY.hip (translation units that build in parallel).
#include "ppo_update_impl.hpp"

XA_PPO_SHAPE_DECL(6, 3)
XA_PPO_SHAPE_DECL(8, 4)
XA_PPO_SHAPE_DECL(2, 3)

namespace {
int capacity_for(int obs_dim, int n_actions) {
  if (obs_dim == 4 && n_actions == 2) return capacity<4, 2>();
  if (obs_dim == 6 && n_actions == 3) return xa_ppo_capacity_6_3();
  if (obs_dim == 8 && n_actions == 4) return xa_ppo_capacity_8_4();
  if (obs_dim == 2 && n_actions == 3) return xa_ppo_capacity_2_3();
  return -1;
}
}  // namespace

extern "C" int xa_ppo_update_blocks(int obs_dim, int n_actions, int mb_size) {
  const int cap = min(capacity_for(obs_dim, n_actions), 256);  // one block per thread in phase C
  if (cap <= 0 || mb_size <= 0) return 0;
  const int tiles = (mb_size + S - 1) / S;
  // small minibatches (<= 16 tiles of 32): 16-sample tiles on twice the blocks -- the step
  // is latency-bound, and the element-wise tile phases halve
  const int tiles16 = (mb_size + 15) / 16;
  if (tiles <= 16 && tiles16 <= cap) return tiles16;
  return tiles < cap ? tiles : cap;
}

extern "C" size_t xa_ppo_update_workspace_bytes(int obs_dim, int n_actions, int batch,
                                                int mb_size, int epochs, int n_blocks) {
  if (batch <= 0 || mb_size <= 0 || epochs <= 0 || n_blocks <= 0) return 0;
  const int n_mb = (batch + mb_size - 1) / mb_size;
  return ws_bytes(n_blocks, offs(obs_dim, n_actions).P, epochs * n_mb);
}

extern "C" size_t xa_ppo_update_dp_block_bytes(int obs_dim, int n_actions, int batch,
                                               int mb_size, int epochs, int n_blocks,
                                               int world) {
  if (batch <= 0 || mb_size <= 0 || epochs <= 0 || n_blocks <= 0 || world <= 1) return 0;
  const int n_mb = (batch + mb_size - 1) / mb_size;
  const int NP2 = padded(offs(obs_dim, n_actions).P) / 2;
  return dp_layout(n_blocks, world, epochs * n_mb, (NP2 + n_blocks - 1) / n_blocks).total;
}

extern "C" int xa_ppo_update(const XaPpoUpdateArgs* a, void* stream) {
  XA_CHECK_ARG(a && a->obs && a->actions && a->old_logp && a->old_values && a->returns &&
                   a->theta && a->adam_m && a->adam_v && a->adam_step && a->workspace,
               "xa_ppo_update: null pointer");
  XA_CHECK_ARG(a->batch > 0 && a->mb_size > 0 && a->epochs > 0, "xa_ppo_update: bad sizes");
  const int n_mb = (a->batch + a->mb_size - 1) / a->mb_size;
  const int K = a->epochs * n_mb;
  XA_CHECK_ARG(K <= kMaxSteps, "xa_ppo_update: %d optimizer steps per launch > %d", K, kMaxSteps);
  XA_CHECK_ARG(((uintptr_t)a->theta & 15) == 0 && ((uintptr_t)a->adam_m & 15) == 0 &&
                   ((uintptr_t)a->adam_v & 15) == 0 && ((uintptr_t)a->workspace & 255) == 0,
               "xa_ppo_update: theta/m/v need 16-byte and the workspace 256-byte alignment");
  const int cap = capacity_for(a->obs_dim, a->n_actions);
  XA_CHECK_ARG(cap != -1, "xa_ppo_update: unsupported (obs_dim, n_actions) = (%d, %d)",
               a->obs_dim, a->n_actions);
  XA_CHECK_ARG(cap > 0, "xa_ppo_update: could not query the resident capacity");
  const int G = a->n_blocks;
  XA_CHECK_ARG(G > 0 && G <= cap && G <= 256 && G <= (a->mb_size + 15) / 16,
               "xa_ppo_update: n_blocks %d must be in [1, min(resident capacity %d, 16-sample "
               "tiles per minibatch)] (xa_ppo_update_blocks)", G, cap);
  XA_CHECK_ARG(a->dp_world <= 1 ||
                   (a->dp_world <= XA_PPO_DP_MAX && a->dp_rank >= 0 && a->dp_rank < a->dp_world),
               "xa_ppo_update: bad data-parallel rank %d / world %d", a->dp_rank, a->dp_world);
  for (int r = 0; a->dp_world > 1 && r < a->dp_world; ++r)
    XA_CHECK_ARG(a->dp_blocks[r] != nullptr && ((uintptr_t)a->dp_blocks[r] & 255) == 0,
                 "xa_ppo_update: data-parallel exchange block %d is null or not 256-B aligned", r);
  const size_t need = ws_bytes(G, offs(a->obs_dim, a->n_actions).P, K);
  XA_CHECK_ARG(a->workspace_bytes >= need, "xa_ppo_update: workspace %zu bytes < %zu needed",
               a->workspace_bytes, need);
  if (a->stats_words > 0) {
    uintptr_t bits = (uintptr_t)a->stats_src;
    bool all = a->stats_src != nullptr;
    for (int i = 0; i < XA_PPO_STATS_SLOTS; ++i) {
      all = all && a->stats_dst[i] != nullptr;
      bits |= (uintptr_t)a->stats_dst[i];
    }
    XA_CHECK_ARG(all && (bits & 3) == 0,
                 "xa_ppo_update: stats_words > 0 needs stats_src and every (4-B aligned) "
                 "stats_dst slot");
  }
  hipStream_t s = (hipStream_t)stream;
  if (a->obs_dim == 4 && a->n_actions == 2) return launch<4, 2>(a, G, K, n_mb, s);
  if (a->obs_dim == 6 && a->n_actions == 3) return xa_ppo_launch_6_3(a, G, K, n_mb, s);
  if (a->obs_dim == 8 && a->n_actions == 4) return xa_ppo_launch_8_4(a, G, K, n_mb, s);
  return xa_ppo_launch_2_3(a, G, K, n_mb, s);
}
XA_DIAG_READER(xa_diag_read_stamps_ppo)
#ifdef XA_TRACE
extern "C" int xa_diag_read_trace_ppo(unsigned* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(xa_ppo_trace), sizeof(xa_ppo_trace)) == hipSuccess
             ? 0 : -1;
}
#endif
