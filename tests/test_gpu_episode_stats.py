"""Device-side episode accumulators (b747_env_batch.ep_stats, BatchControllerEnv.track_episodes) and their
reduction (episode_stats.EpisodeStats): SURVEY 8(e)'s optional gather of scalar episode statistics.
Reference: what SB3's VecMonitor logs around the reference's SubprocVecEnv (neural/agent.py:63-82) --
per finished episode its return (float64 sum of the float32 rewards) and length.  Every accumulator
is checked bit-exactly against the same float64 sums taken from the per-step info buffers."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(n, tk, **kw):
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType, \
        ResetRefMode, RewardType
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=tk, seed=11, **kw)


@pytest.mark.parametrize("limiter", [False, True])   # False: the specialised single-step kernel; True: generic
def test_step_kernel_accumulates_every_finished_episode(limiter):
    from b747_rl_ctrl_amd.episode_stats import EpisodeStats
    n, steps = 4096, 130
    env = _env(n, 0.3, use_limiter=limiter)
    stats = EpisodeStats(env)
    g = torch.Generator(device="cuda").manual_seed(3)
    cnt = torch.zeros(n, dtype=torch.float64, device="cuda")
    ret, length = torch.zeros_like(cnt), torch.zeros_like(cnt)
    for t in range(steps):
        a = torch.rand(n, generator=g, device="cuda") * 2 - 1
        _, _, done, info = env.step(a * (3.0 if limiter else 1.0))
        d = done.to(torch.float64)
        cnt += d
        ret += torch.where(done, info["episode_return"], torch.zeros_like(ret))
        length += torch.where(done, info["episode_length"].to(torch.float64), torch.zeros_like(ret))
    acc = env.ep_stats.clone()
    assert torch.equal(acc[0], cnt) and torch.equal(acc[1], ret) and torch.equal(acc[2], length)
    assert int(cnt.sum()) >= n * (steps // 30)
    if limiter:
        assert not torch.all(length[cnt > 0] / cnt[cnt > 0] == 30)   # some episodes end early
    s = stats.collect()
    assert s["episodes"] == int(cnt.sum())
    assert abs(s["mean_return"] - float(ret.sum() / cnt.sum())) <= 1e-12 * abs(s["mean_return"])
    assert abs(s["mean_length"] - float(length.sum() / cnt.sum())) <= 1e-12 * s["mean_length"]
    assert torch.all(env.ep_stats == 0)                                # collect() restarts the window


def test_fused_ppo_rollout_accumulates_episodes():
    from b747_rl_ctrl_amd.episode_stats import EpisodeStats
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    n, T = 1024, 64
    env = _env(n, 0.2)
    stats = EpisodeStats(env)
    ppo = PPO(env, PPOConfig(n_steps=T), seed=0)
    assert ppo.rollout_kernel
    ppo.collect_rollouts(T)
    torch.cuda.synchronize()
    done, rew = ppo.done_buf.cpu(), ppo.rew_buf.cpu().to(torch.float64)
    run = torch.zeros(n, dtype=torch.float64)
    ret = torch.zeros(n, dtype=torch.float64)
    peak = torch.zeros(n, dtype=torch.float64)
    for t in range(T):                        # VecMonitor's float32 running return, reset at each done
        run = (run + rew[t]).to(torch.float32).to(torch.float64)
        peak = torch.maximum(peak, run.abs())
        ret += torch.where(done[t], run, torch.zeros_like(run))
        run = torch.where(done[t], torch.zeros_like(run), run)
    acc = env.ep_stats.cpu()
    assert torch.equal(acc[0], done.sum(0).to(torch.float64))
    assert torch.all(acc[0] == 3) and torch.all(acc[2] == 60)           # tk = 0.2 s: done at steps 20, 40, 60
    # the kernel adds its float64 reward, this replay the float32 one: a step's float32 rounding of the running
    # return may differ by one ulp where the two straddle a rounding boundary (3 episodes x 20 steps)
    assert bool(((acc[1] - ret).abs() <= 3 * 20 * 2.0 ** -23 * torch.clamp(peak, min=1.0)).all())
    assert stats.collect()["episodes"] == 3 * n
