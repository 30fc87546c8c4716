"""GPU tests of play() (xagents/base.py:595-653): one game of env 0 with the agent's play
policy on the device envs. The replay envs' reward / done streams do not depend on the
actions, so the expected total reward is env 0's recorded first episode; the dynamics env
is checked against its own rollout rows. Training counters stay untouched."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _first_episode(env, max_steps=None):
    rew = env.rep_rew[0].cpu().numpy().astype(np.float64)
    done = env.rep_done[0].cpu().numpy()
    k = int(np.nonzero(done)[0][0])
    if max_steps is not None and max_steps <= k:
        return float(rew[:max_steps].sum())
    return float(rew[:k + 1].sum())


def _counters(agent):
    return agent.steps, agent.games, list(agent.total_rewards)


@pytest.mark.parametrize('max_steps', [None, 3])
def test_ppo_play_replay_env(device, max_steps):
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 8, t_rec=512, seed=5, device=device)
    model = create_model(envs, 'ppo', 'model', seed=5, device=device)
    agent = PPO(envs, model, n_steps=16, seed=5, quiet=True)
    before = _counters(agent)
    total = agent.play(max_steps=max_steps)
    assert total == _first_episode(envs, max_steps)
    assert _counters(agent) == before


def test_ppo_play_dynamics_env_matches_its_rollout(device):
    from xagents_amd import PPO
    from xagents_amd.envs import CartPoleVecEnv
    from xagents_amd.utils.common import create_model
    envs = CartPoleVecEnv(4, seed=9, device=device)
    model = create_model(envs, 'ppo', 'model', seed=9, device=device)
    agent = PPO(envs, model, n_steps=512, seed=9, quiet=True)
    total = agent.play()
    # one 512-step chunk covers a CartPole-v1 episode (<= 500 steps): reward 1 per step
    # up to and including env 0's first done
    done = agent.b_done[0, 1:].cpu().numpy()
    k = int(np.nonzero(done)[0][0])
    assert total == float(k + 1)
    assert 1 <= total <= 500


def test_a2c_play_counts_to_max_steps(device):
    from xagents_amd import A2C
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 4, t_rec=256, seed=6, device=device)
    model = create_model(envs, 'a2c', 'model', seed=6, device=device)
    agent = A2C(envs, model, n_steps=5, seed=6, quiet=True)
    assert agent.play(max_steps=7) == _first_episode(envs, 7)
    with pytest.raises(NotImplementedError):
        agent.play(render=True)


def test_dqn_play_greedy(device):
    from xagents_amd import DQN
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('PongNoFrameskip-v4', 2, device=device, seed=7, t_rec=64)
    bufs = create_buffers('dqn', 40, 4, 2, initial_size=8)
    model = create_model(envs, 'dqn', 'model', seed=3, device=device)
    agent = DQN(envs, model, bufs, seed=11, quiet=True)
    sizes = [b.current_size for b in bufs]
    total = agent.play()
    assert total == _first_episode(envs)
    assert [b.current_size for b in bufs] == sizes  # play stores nothing
    # the greedy actions are argmax Q of the current states
    q = agent.ex_act.forward(envs.state)[0].cpu().numpy()
    acts = agent._play_actions().cpu().numpy()
    assert np.array_equal(acts, q.argmax(1))


@pytest.mark.parametrize('kind', ['td3', 'ddpg'])
def test_td3_ddpg_play_noise_free_actor(device, kind):
    from xagents_amd import DDPG, TD3
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    envs = create_envs('BipedalWalker-v3', 4, device=device, seed=4, t_rec=128)
    kw = dict(seed=7, device=device)
    actor = create_model(envs, kind, 'actor_model', **kw)
    critic = create_model(envs, kind, 'critic_model', **kw)
    bufs = create_buffers(kind, 32, 8, 4, initial_size=16)
    agent = (TD3 if kind == 'td3' else DDPG)(envs, actor, critic, bufs, seed=3, quiet=True)
    before = _counters(agent)
    assert agent.play(max_steps=50) == _first_episode(envs, 50)
    assert _counters(agent) == before
    a1 = agent._play_actions().clone()
    a2 = agent._play_actions()
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)  # deterministic: no exploration noise
