// The persistent PPO update's (obs, actions) = (6, 3) instantiations (Acrobot-v1-shaped
// envs) in their own translation unit: ppo_update.hip holds the entry points and the
// CartPole-v1 (4, 2) kernels, and the shapes build in parallel.
#include "ppo_update_impl.hpp"

XA_PPO_SHAPE_TU(6, 3)
