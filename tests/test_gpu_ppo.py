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
@pytest.mark.parametrize("fused", [False, True])
def test_rollout_replays_exactly_through_a_fresh_env(use_graph, fused):
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = _env()
    ppo = PPO(env, PPOConfig(n_steps=48, batch_size=4096), seed=1, fused=fused)
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
    torch.testing.assert_close(value, ppo.val_buf[5], rtol=1e-5, atol=1e-5)   # fused: tanh within ~1e-6


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


def test_fused_policy_kernel_matches_the_torch_policy():
    """b747_policy_act vs ActorCritic on the same obs and noise (fp32; tolerance 2e-5 absolute:
    the kernel's tanh is exp/rcp based, torch's is libm)."""
    from b747_rl_ctrl_amd import _lib
    from b747_rl_ctrl_amd.ppo import ActorCritic
    L = _lib.lib()
    torch.manual_seed(0)
    for od in (3, 5, 7, 8, 10):
        pol = ActorCritic(od).cuda()
        with torch.no_grad():
            for prm in pol.parameters():                       # break the ortho-init symmetry/scale
                prm.add_(0.05 * torch.randn_like(prm))
        fp = pol.flat_params()
        flat = torch.zeros(L.b747_policy_num_params(od), device="cuda")
        derived_end = fp.numel() + 2 * 64 * 64 + 2 * 64 * (od + 1) + 4 * 64 + 3
        assert flat.numel() == ((derived_end + 3) & ~3) + 1024       # + the layer-1 MFMA fragments (16 B aligned)
        flat[:fp.numel()].copy_(fp)
        _lib.check(L.b747_policy_pack(flat.data_ptr(), od, None), "pack")
        n = 3000                                               # not a multiple of 64: tail wave
        obs = torch.randn(n, od, device="cuda")
        noise = torch.randn(n, device="cuda")
        out = {k: torch.empty(n, device="cuda") for k in ("act", "logp", "val", "env")}
        obs_copy = torch.empty(n, od, device="cuda")
        _lib.check(L.b747_policy_act(flat.data_ptr(), od, n, obs.data_ptr(), noise.data_ptr(), 0, None, 0, 0,
                                     obs_copy.data_ptr(), out["act"].data_ptr(), out["logp"].data_ptr(),
                                     out["val"].data_ptr(), out["env"].data_ptr(), -1.0, 1.0, None), "policy")
        torch.cuda.synchronize()
        with torch.no_grad():
            mean, value = pol(obs)
            act = mean.squeeze(-1) + pol.log_std.exp() * noise
            lp = pol.log_prob(mean, act[:, None])
        assert torch.equal(obs_copy, obs)
        torch.testing.assert_close(out["act"], act, rtol=0, atol=2e-5)
        torch.testing.assert_close(out["val"], value, rtol=0, atol=2e-5)
        torch.testing.assert_close(out["logp"], lp, rtol=0, atol=2e-5)
        torch.testing.assert_close(out["env"], out["act"].clamp(-1, 1), rtol=0, atol=0)


@pytest.mark.parametrize("od", [3, 5])   # 3: the matrix-core layer 1 (f16 hi/lo split of the obs); 5: the VALU layer 1
def test_fused_policy_kernel_large_observations_saturate_like_the_torch_policy(od):
    """an observation beyond the f16 range (a diverged env's integral term, |obs| > 65504) must not turn
    the matrix-core layer 1's hi/lo split into inf - inf = NaN; the f32 torch policy saturates through tanh.  One
    large component per row (signs and magnitudes 7e4 .. 3e38), the others ordinary; NaN rows stay NaN."""
    from b747_rl_ctrl_amd import _lib
    from b747_rl_ctrl_amd.ppo import ActorCritic
    L = _lib.lib()
    torch.manual_seed(1)
    pol = ActorCritic(od).cuda()
    flat = torch.zeros(L.b747_policy_num_params(od), device="cuda")
    fp = pol.flat_params()
    flat[:fp.numel()].copy_(fp)
    _lib.check(L.b747_policy_pack(flat.data_ptr(), od, None), "pack")
    n = 640
    obs = torch.randn(n, od, device="cuda")
    big = torch.tensor([7e4, -7e4, 1e6, -3e7, 3e38, -3e38, 65504.0, 65520.0], device="cuda")
    rows = torch.arange(n - 64, device="cuda")
    obs[rows, rows % od] = big[rows % big.numel()]
    obs[n - 64:n - 60, 0] = float("nan")
    noise = torch.randn(n, device="cuda")
    out = {k: torch.empty(n, device="cuda") for k in ("act", "logp", "val", "env")}
    obs_copy = torch.empty(n, od, device="cuda")
    _lib.check(L.b747_policy_act(flat.data_ptr(), od, n, obs.data_ptr(), noise.data_ptr(), 0, None, 0, 0,
                                 obs_copy.data_ptr(), out["act"].data_ptr(), out["logp"].data_ptr(),
                                 out["val"].data_ptr(), out["env"].data_ptr(), -1.0, 1.0, None), "policy")
    torch.cuda.synchronize()
    with torch.no_grad():
        mean, value = pol(obs)
        act = mean.squeeze(-1) + pol.log_std.exp() * noise
    fin = torch.isfinite(obs).all(dim=1)
    assert bool(torch.isfinite(out["act"][fin]).all()) and bool(torch.isfinite(out["val"][fin]).all())
    torch.testing.assert_close(out["act"][fin], act[fin], rtol=0, atol=2e-5)
    torch.testing.assert_close(out["val"][fin], value[fin], rtol=0, atol=2e-5)
    assert bool(torch.isnan(out["act"][~fin]).all()) and bool(torch.isnan(value[~fin]).all())


def test_fused_policy_noise_is_standard_normal_and_fresh_per_rollout():
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    ppo = PPO(_env(4096), PPOConfig(n_steps=8, batch_size=4096), seed=7, fused=True)
    ppo.last_obs.copy_(ppo.env.obs)
    ppo.collect_rollouts(8)
    a1 = ppo.act_buf.clone()
    ppo.collect_rollouts(8)
    assert not torch.equal(a1, ppo.act_buf)                  # step_base advanced inside the graph
    with torch.no_grad():
        mean, _ = ppo.policy(ppo.obs_buf[3])
        z = (ppo.act_buf[3] - mean) / ppo.policy.log_std.exp()
    assert abs(float(z.mean())) < 0.05 and abs(float(z.std()) - 1) < 0.05
    # the whole rollout (8 x 4096 draws; Box-Muller on the hardware log/sqrt/cos): Kolmogorov-Smirnov
    # against N(0, 1) and the two-sided 3-sigma tail mass (0.27 %)
    import scipy.stats
    with torch.no_grad():
        mean, _ = ppo.policy(ppo.obs_buf.reshape(-1, ppo.obs_buf.shape[-1]))
        z = ((ppo.act_buf.reshape(-1) - mean.reshape(-1)) / ppo.policy.log_std.exp()).double().cpu().numpy()
    assert scipy.stats.kstest(z, "norm").pvalue > 1e-3
    tail = float((abs(z) > 3).mean())
    assert 0.0015 < tail < 0.0045, tail


def _aero_env(n=256, seed=3, sample_time=None):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=0.3, seed=seed,
                              sample_time=sample_time)


def _same_episode_books(e1, e2):
    """ep_final_len / ep_final_return / ep_stats (track_episodes) of the fused kernel and the reference path"""
    assert torch.equal(e1.ep_final_len, e2.ep_final_len), "ep_final_len"
    assert torch.equal(e1.ep_stats[0], e2.ep_stats[0]) and torch.equal(e1.ep_stats[2], e2.ep_stats[2]), \
        "ep_stats: episode count / length sum"
    torch.testing.assert_close(e1.ep_final_return, e2.ep_final_return, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1.ep_stats[1], e2.ep_stats[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1.ep_return, e2.ep_return, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,T,st", [(256, 48, None), (320, 48, None), (192, 37, None),   # 320, 192: partial
                                    (256, 48, 0.05), (320, 24, 0.05), (192, 19, "0.05-misaligned")])  # workgroups
def test_fused_rollout_kernel_matches_two_launch_rollout(n, T, st):   # (waves past N idle); 37 x 192 rows: a partial value-pass block
    """b747_ppo_rollout (policy + env step in one launch for all T steps, the training configuration)
    against the two-launch path (b747_policy_act + b747_env_step per step): same policy, same Philox
    noise, same env.  Both are the FAST variant; the fused kernel's code may fuse mul+add pairs
    differently (FMA contraction), so floats agree to rounding and dones / episode resets / episode lengths
    (ep_final_len, ep_stats) exactly.
    st = 0.05: main.py's sample_time (5 DLL steps per env step, core/controller.py:258-264),
    with the reference path's env step on the one-wave kernel (b747_set_specialization(2)), which sub-steps
    through env_step_lane; "0.05-misaligned": every env starts at k = 0..4, so its first env step is shorter."""
    from b747_rl_ctrl_amd import _lib
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    L = _lib.lib()
    sample_time = None if st is None else 0.05
    e1, e2 = _aero_env(n, sample_time=sample_time), _aero_env(n, sample_time=sample_time)
    for e in (e1, e2):
        e.track_episodes()
        if st == "0.05-misaligned":
            e.k.copy_(torch.arange(n, device="cuda", dtype=e.k.dtype) % 5)
    p1 = PPO(e1, PPOConfig(n_steps=T, batch_size=4096), seed=1, rollout_kernel=True)
    p2 = PPO(e2, PPOConfig(n_steps=T, batch_size=4096), seed=1, rollout_kernel=False)
    assert p1.rollout_kernel and not p2.rollout_kernel
    prev = L.b747_set_specialization(1)
    try:
        for _ in range(2):                               # two rollouts: fresh noise (step_base) each
            p1.collect_rollouts(T)
            L.b747_set_specialization(1 if st is None else 2)
            p2.collect_rollouts(T, use_graph=True)
            L.b747_set_specialization(1)
            torch.cuda.synchronize()
            assert torch.equal(p1.done_buf, p2.done_buf)
            assert int(p1.done_buf.sum()) >= n           # tk = 0.3 s: every env ends an episode per rollout
            for a, b in ((p1.obs_buf, p2.obs_buf), (p1.act_buf, p2.act_buf), (p1.logp_buf, p2.logp_buf),
                         (p1.val_buf, p2.val_buf), (p1.rew_buf, p2.rew_buf), (e1.obs, e2.obs),
                         (e1.terminal_obs, e2.terminal_obs)):
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
            scale = e2.X.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
            assert float(((e1.X - e2.X).abs() / scale).max()) <= 1e-9
            assert torch.equal(e1.k, e2.k) and torch.equal(e1.episode, e2.episode)
            _same_episode_books(e1, e2)
    finally:
        L.b747_set_specialization(prev)
    if sample_time:
        assert bool((e1.k % 5 == 0).all())


def test_fused_rollout_kernel_workgroup_geometry_does_not_change_results():
    """The fused PPO rollout kernel runs 64 envs per workgroup up to 32,768 envs and 256 above (b747_fast.hip).  Env
    i's policy noise (Philox counter (env id, step_base + step)) and reset draws depend only on its global id, and the
    policy weights only on the seed, so the first 8,192 envs of a 40,960-env batch (256 per workgroup) and an
    8,192-env batch (64 per workgroup) roll out the same trajectories: dones and episode books exactly, floats to the
    rounding two compilations of one source differ by (as between the fused and the two-launch path above)."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    m, T = 8192, 48
    e1, e2 = _aero_env(40960), _aero_env(m)
    for e in (e1, e2):
        e.track_episodes()
    p1 = PPO(e1, PPOConfig(n_steps=T, batch_size=4096), seed=4, rollout_kernel=True)
    p2 = PPO(e2, PPOConfig(n_steps=T, batch_size=4096), seed=4, rollout_kernel=True)
    assert p1.rollout_kernel and p2.rollout_kernel
    for _ in range(2):                                   # two rollouts: fresh noise (step_base) each
        p1.collect_rollouts(T)
        p2.collect_rollouts(T)
        torch.cuda.synchronize()
        assert torch.equal(p1.done_buf[:, :m], p2.done_buf)
        assert int(p2.done_buf.sum()) >= m
        for a, b in ((p1.obs_buf[:, :m], p2.obs_buf), (p1.act_buf[:, :m], p2.act_buf),
                     (p1.logp_buf[:, :m], p2.logp_buf), (p1.val_buf[:, :m], p2.val_buf),
                     (p1.rew_buf[:, :m], p2.rew_buf), (e1.obs[:m], e2.obs), (e1.terminal_obs[:m], e2.terminal_obs)):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
        scale = e2.X.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
        assert float(((e1.X[:, :m] - e2.X).abs() / scale).max()) <= 1e-9
        assert torch.equal(e1.k[:m], e2.k) and torch.equal(e1.episode[:m], e2.episode)
        assert torch.equal(e1.ep_final_len[:m], e2.ep_final_len)
        torch.testing.assert_close(e1.ep_final_return[:m], e2.ep_final_return, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(e1.ep_return[:m], e2.ep_return, rtol=1e-5, atol=1e-5)


def test_fused_rollout_kernel_lock_step_workgroups_match_two_launch_rollout():
    """The two-wave rollout kernel (csrc/b747_ppo_split.h) runs a workgroup in lock step when one of its envs has
    a delta that depends on the stage (SS PID in the loop: flags |= F_PID_SS) or on the current action (no rate
    limiter: flags = 0); the other workgroups keep the policy beside the stages.  Workgroup 0 holds SS-PID envs,
    workgroup 1 envs without the rate limiter, workgroup 2 is untouched: all three against the two-launch path."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    n = 768
    e1, e2 = _aero_env(n), _aero_env(n)
    for e in (e1, e2):
        e.track_episodes()
        e.flags[0:256:37] |= 1                           # F_PID_SS
        e.flags[256 + 5:512:41] = 0                      # neither the rate limiter nor a PID
    p1 = PPO(e1, PPOConfig(n_steps=40, batch_size=4096), seed=2, rollout_kernel=True)
    p2 = PPO(e2, PPOConfig(n_steps=40, batch_size=4096), seed=2, rollout_kernel=False)
    for _ in range(2):
        p1.collect_rollouts(40)
        p2.collect_rollouts(40, use_graph=True)
        torch.cuda.synchronize()
        assert torch.equal(p1.done_buf, p2.done_buf)
        assert int(p1.done_buf.sum()) >= n
        for a, b in ((p1.obs_buf, p2.obs_buf), (p1.act_buf, p2.act_buf), (p1.logp_buf, p2.logp_buf),
                     (p1.val_buf, p2.val_buf), (p1.rew_buf, p2.rew_buf), (e1.obs, e2.obs)):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
        scale = e2.X.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
        assert float(((e1.X - e2.X).abs() / scale).max()) <= 1e-9
        for f in ("k", "episode", "mem", "flags"):
            assert torch.equal(getattr(e1, f), getattr(e2, f)), f
        torch.testing.assert_close(e1.disc, e2.disc, rtol=1e-9, atol=1e-12)
        _same_episode_books(e1, e2)


def test_fused_rollout_kernel_rejects_other_configurations():
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = _env()                                         # no AERO disturbance: not the covered configuration
    assert PPO(env, PPOConfig(n_steps=8, batch_size=4096), seed=1).rollout_kernel is False
    with pytest.raises(ValueError):
        PPO(env, PPOConfig(n_steps=8, batch_size=4096), seed=1, rollout_kernel=True)
