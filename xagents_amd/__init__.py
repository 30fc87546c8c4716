"""xagents_amd -- MI355X-native hot path for the xagents RL API.

Agent registry and command table mirror xagents/__init__.py:18-40. Only the
agents whose hot path is built are registered (see DESIGN.md for scope).
"""
from xagents_amd import a2c, acer, ddpg, dqn, ppo, td3, trpo
from xagents_amd.a2c.agent import A2C
from xagents_amd.acer.agent import ACER
from xagents_amd.base import BaseAgent, OffPolicy, OnPolicy
from xagents_amd.ddpg.agent import DDPG
from xagents_amd.dqn.agent import DQN
from xagents_amd.ppo.agent import PPO
from xagents_amd.td3.agent import TD3
from xagents_amd.trpo.agent import TRPO
from xagents_amd.utils.common import register_models

__version__ = '0.1.0'

agents = {
    'a2c': {'module': a2c, 'agent': A2C},
    'acer': {'module': acer, 'agent': ACER},
    'ppo': {'module': ppo, 'agent': PPO},
    'dqn': {'module': dqn, 'agent': DQN},
    'ddpg': {'module': ddpg, 'agent': DDPG},
    'td3': {'module': td3, 'agent': TD3},
    'trpo': {'module': trpo, 'agent': TRPO},
}
register_models(agents)

__all__ = ['A2C', 'ACER', 'DDPG', 'DQN', 'PPO', 'TD3', 'TRPO', 'BaseAgent', 'OnPolicy', 'OffPolicy', 'agents']
