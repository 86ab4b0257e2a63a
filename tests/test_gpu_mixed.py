"""The MIXED variant (include/b747.h B747_VARIANT_MIXED) against the C env oracle, at the north star's
parity gate: "outputs match the reference DLL step-for-step within 1e-5 relative fp32 on identical (state, action)
sequences" (BASELINE.json north_star).  MIXED computes the two-wave kernels' flight aerodynamics (ISA, speed, alpha,
the table lookups, forces, pitching moment) in fp32 and everything else -- state, attitude, RK4 integration, the
control side with its Derivative blocks, read-out -- in fp64 as FAST does.

Per step means: the oracle's compact state (X, disc, k, Memory bits) is loaded into the GPU batch before every step
(per-step kernel) or every launch (multi-step kernels: at most 10 env steps of free run), both advance with the same
actions, and every env's observation and reward are compared: |gpu - oracle| <= 1e-5 max(|oracle|, 1) -- relative
1e-5 of the value, or of the signal's full scale where the value is smaller (the observations are normalised by
obs_max, env/ctrl_env.py:200-214, so 1 is their full scale; the reward's terms are <= 1).  A value-relative bound
alone is not meaningful for the Derivative-block observation dtheta/dt near zero: an fp32 rounding of the pitching
moment moves it by ~1e-8 of its scale, which on a value of 6.5e-7 is 3e-5 of the value (measured worst case,
tools/exp_mixed_parity.py: absolute errors obs 7.5e-9 / 1.5e-8 / 5.8e-11, reward 2.8e-7).  done is exact."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_lib as O  # noqa: E402
from test_gpu_episode_replay import _load_oracle_state  # noqa: E402
from test_gpu_fullsize import _device_draws  # noqa: E402

pytestmark = pytest.mark.gpu

N = 65536
REL, FULL_SCALE = 1e-5, 1.0


def _env(n, tk, sample_time=None, seed=2024):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=tk, sample_time=sample_time,
                              seed=seed, variant="mixed")


def _gate(got, ref, what):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    tol = REL * np.maximum(np.abs(ref), FULL_SCALE)
    err = np.abs(got - ref)
    bad = np.flatnonzero(err > tol)
    assert bad.size == 0, (f"{what}: {bad.size} envs beyond 1e-5, e.g. env {bad[0]} gpu {got[bad[0]]!r} oracle "
                           f"{ref[bad[0]]!r} (tolerance {tol[bad[0]]:.3g})")
    return float(np.max(err / tol))


def _compare(full, actions, obs, rew, done, term, env, step):
    o_ref, r_ref, d_ref = full.step(actions)
    d = np.asarray(done, bool)
    assert np.array_equal(d, d_ref.astype(bool)), f"step {step}: done differs in {np.flatnonzero(d != d_ref)[:10]}"
    o = np.where(d[:, None], term, obs)
    worst = max(_gate(o[:, c], o_ref[:, c], f"obs[{c}] step {step}") for c in range(o.shape[1]))
    worst = max(worst, _gate(rew, r_ref.astype(np.float32), f"reward step {step}"))
    if d.any():
        full.reset(*_device_draws(env), mask=d)
    return worst


def test_mixed_per_step_kernel_within_the_north_star_gate():
    """b747_env_step (k_env_step_split<double, MIX>) on 65,536 envs, 250 steps across an auto-reset (tk = 1 s)."""
    from b747_rl_ctrl_amd import _lib
    assert _lib.lib().b747_set_specialization(1) == 1
    env = _env(N, 1.0)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=1.0)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(5)
    worst = 0.0
    for t in range(250):
        _load_oracle_state(env, full)
        a = torch.rand(N, device="cuda", generator=g) * 2 - 1
        obs, rew, done, info = env.step(a)
        worst = max(worst, _compare(full, a.cpu().numpy(), obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(),
                                    info["terminal_observation"].cpu().numpy(), env, t))
    assert int(env.episode.min()) >= 3
    print(f"\nMIXED per-step kernel: worst error / tolerance {worst:.3f}")


@pytest.mark.parametrize("sample_time", [None, 0.05])
def test_mixed_rollout_kernel_within_the_north_star_gate(sample_time):
    """b747_env_rollout (k_rollout_split<false, double, SUB, MIX>): launches of 10 env steps (4 at sample_time 0.05),
    the oracle's state loaded before each."""
    K = 10 if sample_time is None else 4
    env = _env(N, 1.0, sample_time)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=sample_time or 0.01, tk=1.0)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(6)
    obs_seq = torch.empty(K, N, 3, device="cuda")
    rew_seq = torch.empty(K, N, device="cuda")
    done_seq = torch.empty(K, N, dtype=torch.uint8, device="cuda")
    worst = 0.0
    for launch in range(25):
        _load_oracle_state(env, full)
        acts = torch.rand(K, N, device="cuda", generator=g) * 2 - 1
        env.rollout(acts, obs_seq, rew_seq, done_seq)
        a_h, o_h, r_h, d_h = acts.cpu().numpy(), obs_seq.cpu().numpy(), rew_seq.cpu().numpy(), done_seq.cpu().numpy()
        term = env.terminal_obs.cpu().numpy()
        for t in range(K):
            worst = max(worst, _compare(full, a_h[t], o_h[t], r_h[t], d_h[t], term, env, launch * K + t))
    assert int(env.episode.min()) >= 2
    print(f"\nMIXED rollout kernel (sample_time {sample_time}): worst error / tolerance {worst:.3f}")


@pytest.mark.parametrize("sample_time", [None, 0.05])
def test_mixed_ppo_rollout_kernel_within_the_north_star_gate(sample_time):
    """b747_ppo_rollout (k_rollout_split<true, double, SUB, MIX>): the policy's own clipped actions drive the oracle;
    launches of 10 env steps (4 at sample_time 0.05), the oracle's state loaded before each."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    T = 10 if sample_time is None else 4
    env = _env(N, 1.0, sample_time, seed=9)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=sample_time or 0.01, tk=1.0)
    full.reset(*_device_draws(env))
    ppo = PPO(env, PPOConfig(n_steps=T, batch_size=N), seed=1, rollout_kernel=True)
    assert ppo.rollout_kernel
    gen = torch.Generator(device="cuda").manual_seed(4)
    with torch.no_grad():
        for prm in ppo.policy.parameters():
            prm.add_(0.05 * torch.randn(prm.shape, generator=gen, device="cuda"))
    ppo.sync_params()
    prev = np.zeros((N, 3), np.float32)
    worst = 0.0
    for launch in range(25):
        _load_oracle_state(env, full)
        ppo.collect_rollouts(T)
        obs_b, rew_b = ppo.obs_buf.cpu().numpy(), ppo.rew_buf.cpu().numpy()
        done_b = ppo.done_buf.cpu().numpy()
        act_b = ppo.act_buf[..., 0].clamp(-1, 1).cpu().numpy()
        term = env.terminal_obs.cpu().numpy()
        for t in range(T):
            for c in range(3):
                worst = max(worst, _gate(obs_b[t, :, c], prev[:, c], f"obs the policy saw [{c}] step {launch * T + t}"))
            o_ref, r_ref, d_ref = full.step(act_b[t])
            assert np.array_equal(done_b[t], d_ref), f"done step {launch * T + t}"
            worst = max(worst, _gate(rew_b[t], r_ref.astype(np.float32), f"reward step {launch * T + t}"))
            if d_ref.any():
                for c in range(3):
                    worst = max(worst, _gate(term[d_ref, c], o_ref[d_ref, c], f"terminal obs [{c}]"))
                full.reset(*_device_draws(env), mask=d_ref)
            prev = np.where(d_ref[:, None], 0.0, o_ref).astype(np.float32)
    assert int(env.episode.min()) >= 2
    print(f"\nMIXED PPO rollout kernel (sample_time {sample_time}): worst error / tolerance {worst:.3f}")
