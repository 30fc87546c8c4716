"""Checkpoint / resume (xagents/base.py:213-230, 370-386, 428-455,
utils/common.py:416-427, 616-623): the flat weight + Adam-state checkpoint round-trips
into a fresh agent so that the next train step is bit-identical, best-reward
checkpointing writes it, and the parquet training history restores the counters."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ppo(seed=11, **kw):
    from xagents_amd import PPO
    from xagents_amd.envs import ReplayVecEnv
    from xagents_amd.utils.common import create_model
    envs = ReplayVecEnv('CartPole-v1', 16, t_rec=256, seed=seed, device='cuda')
    model = create_model(envs, 'ppo', 'model', seed=seed, device='cuda')
    return PPO(envs, model, n_steps=32, seed=seed, quiet=True, **kw)


def _copy_env_state(dst, src):
    for name in ('state', 'done', 'cursor', 'ep_return'):
        getattr(dst.envs, name).copy_(getattr(src.envs, name))
    dst.rng_counter.copy_(src.rng_counter)


def test_weights_and_adam_state_round_trip(device, tmp_path):
    a = _ppo()
    for _ in range(2):
        a.train_step()
    torch.cuda.synchronize()
    ckpt = tmp_path / 'model.tf'
    a.model.save_weights(ckpt)
    b = _ppo()
    assert not np.array_equal(b.model.theta.cpu().numpy(), a.model.theta.cpu().numpy())
    b.model.load_weights(ckpt).expect_partial()
    opt_a, opt_b = a.model.optimizer, b.model.optimizer
    for x, y in ((a.model.theta, b.model.theta), (opt_a.m, opt_b.m), (opt_a.v, opt_b.v),
                 (opt_a.iterations, opt_b.iterations)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    # the same env position and RNG counter: the next train step is bit-identical
    _copy_env_state(b, a)
    a.train_step()
    b.train_step()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.b_act.cpu().numpy(), b.b_act.cpu().numpy())
    np.testing.assert_array_equal(a.model.theta.cpu().numpy(), b.model.theta.cpu().numpy())
    np.testing.assert_array_equal(opt_a.m.cpu().numpy(), opt_b.m.cpu().numpy())
    # a checkpoint of another architecture is refused
    bad = tmp_path / 'bad.npz'
    np.savez(bad, theta=np.zeros(10, np.float32))
    with pytest.raises(AssertionError, match='Checkpoint holds 10 parameters'):
        b.model.load_weights(bad)


def test_best_reward_checkpoint_and_history_resume(device, tmp_path):
    ckpt = str(tmp_path / 'best.tf')
    hist = str(tmp_path / 'history.parquet')
    a = _ppo(checkpoints=[ckpt], history_checkpoint=hist, log_frequency=16)
    a.fit(max_steps=16 * 32 * 6)
    assert a.games > 0 and a.best_reward > -float('inf')
    import pandas as pd
    rows = pd.read_parquet(hist)
    assert set(rows.columns) == {'mean_reward', 'best_reward', 'episode_reward', 'step', 'time'}
    assert len(rows) == a.games
    # the best-reward checkpoint exists and loads
    b = _ppo()
    b.model.load_weights(ckpt)
    assert np.isfinite(b.model.theta.cpu().numpy()).all()
    # a new agent on the same history resumes steps / games / best reward
    c = _ppo(history_checkpoint=hist)
    c.init_training(None, 10 ** 9, None)
    last = rows.loc[rows['time'].idxmax()]
    assert c.steps == int(last['step'])
    assert c.games == len(rows)
    assert c.best_reward == rows['best_reward'].max()
    assert list(c.total_rewards) == [last['episode_reward']]
