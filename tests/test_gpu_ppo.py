"""On-GPU PPO rollout (b747_rl_ctrl_amd/ppo.py, BASELINE config 5).

The env is deterministic given its actions, so a rollout is checked by replaying the stored
(clipped) actions through a fresh env with the same seed: rewards and dones must be identical
(bit-exact), and the stored observations must be the ones the policy saw."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(n=256, seed=3):
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST, tk=0.3, seed=seed)


@pytest.mark.parametrize("use_graph", [False, True])
def test_rollout_replays_exactly_through_a_fresh_env(use_graph):
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = _env()
    ppo = PPO(env, PPOConfig(n_steps=48, batch_size=4096), seed=1)
    ppo.last_obs.copy_(env.obs)
    ppo.collect_rollouts(48, use_graph=use_graph)
    torch.cuda.synchronize()
    ref = _env()
    obs = ref.obs.clone()
    for t in range(48):
        assert torch.equal(ppo.obs_buf[t], obs), f"obs step {t}"
        o, r, d, _ = ref.step(ppo.act_buf[t].clamp(-1, 1).view(-1))
        assert torch.equal(r, ppo.rew_buf[t]) and torch.equal(d, ppo.done_buf[t]), f"step {t}"
        obs = o.clone()
    assert int(ppo.done_buf.sum()) == 256                # tk = 0.3 s: every episode ends at step 30
    # log-probs are those of the Gaussian policy at the stored actions
    mean, value = ppo.policy(ppo.obs_buf[5])
    lp = ppo.policy.log_prob(mean, ppo.act_buf[5])
    torch.testing.assert_close(lp, ppo.logp_buf[5], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(value, ppo.val_buf[5], rtol=1e-5, atol=1e-5)


def test_learn_iteration_runs_and_losses_are_finite():
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    ppo = PPO(_env(512), PPOConfig(n_steps=32, batch_size=4096, n_epochs=2), seed=0)
    hist = ppo.learn(2)
    assert len(hist) == 2 and all(math.isfinite(h["policy_loss"]) and math.isfinite(h["value_loss"]) for h in hist)
    assert torch.isfinite(ppo.adv_buf).all()


def test_sb3_default_policy_shapes():
    from b747_rl_ctrl_amd.ppo import ActorCritic
    p = ActorCritic(3)
    n_params = sum(x.numel() for x in p.parameters())
    assert n_params == 2 * (3 * 64 + 64 + 64 * 64 + 64) + (64 + 1) + (64 + 1) + 1
