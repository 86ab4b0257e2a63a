"""The MIXED variant (include/b747.h B747_VARIANT_MIXED) against the C env oracle.  MIXED computes the
two-wave kernels' flight aerodynamics (ISA, speed, alpha, the table lookups, forces, pitching moment) in fp32 and
everything else -- state, attitude, RK4 integration, the control side with its Derivative blocks, read-out -- in fp64
as FAST does.

Per step (round 5): the oracle's compact state (X, disc, k, Memory bits) is loaded into the GPU
batch before every step (per-step kernel) or every launch (multi-step kernels: at most 10 env steps of free run),
both advance with the same actions, and every env's observation and reward are held to FAST's own replay bar
(tests/test_gpu_episode_replay.py): |gpu - oracle| <= 2e-6 |oracle| + 1e-7 + 1e-7 x the component's largest |value|
in the batch at that step.  That is tighter than the north star's "1e-5 relative" wherever |oracle| exceeds ~0.02 of
its batch scale; below it (the Derivative-block observation dtheta/dt near zero: an fp32 rounding of the pitching
moment moves it by ~1e-8 of its scale) the bar is the absolute floor, which the measured worst errors (obs 7.5e-9 /
1.5e-8 / 5.8e-11, reward 2.8e-7; tools/exp_mixed_parity.py) meet with a factor ~7-13 to spare -- the printed worst
error / tolerance says how much.  done is exact.  The free-running whole episode is compared with FAST and the oracle
below (test_mixed_free_running_episode_against_fast_and_the_oracle), and tests/test_gpu_episode_replay.py replays
MIXED's bench kernels over the tk = 20 s episode in 50- / 100-step free windows like FAST's."""
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
RTOL, ATOL, SCALE_TOL = 2e-6, 1e-7, 1e-7   # FAST's episode-replay bar (tests/test_gpu_episode_replay.py)


def _env(n, tk, sample_time=None, seed=2024):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=tk, sample_time=sample_time,
                              seed=seed, variant="mixed")


def _gate(got, ref, what):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    tol = RTOL * np.abs(ref) + ATOL + SCALE_TOL * float(np.max(np.abs(ref))) if ref.size else 1.0
    err = np.abs(got - ref)
    bad = np.flatnonzero(err > tol)
    assert bad.size == 0, (f"{what}: {bad.size} envs beyond the bar, e.g. env {bad[0]} gpu {got[bad[0]]!r} oracle "
                           f"{ref[bad[0]]!r} (tolerance {np.broadcast_to(tol, err.shape)[bad[0]]:.3g})")
    return float(np.max(err / tol)) if err.size else 0.0


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


def test_mixed_per_step_kernel_per_step_parity():
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
def test_mixed_rollout_kernel_per_step_parity(sample_time):
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
def test_mixed_ppo_rollout_kernel_per_step_parity(sample_time):
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


def test_mixed_free_running_episode_against_fast_and_the_oracle():
    """ADVICE r4 / VERDICT r4 #1c: the bench's whole tk = 20 s episode (2,000 env steps of the per-step kernel,
    65,536 envs, the bench's randomized trim / reference / aero-error sweep) run FREE -- no state reload -- by MIXED
    and by FAST with the same actions, against the C env oracle.  What training sees of the difference: per env, the
    largest deviation of the observation over the episode (relative to the component's batch scale at that step)
    and the episode return (VecMonitor's).  Saturated PID envs are chaotic (ulp differences double
    every ~50 steps), so the bounds are on quantiles over the envs; FAST, whose per-step error is ~1e-16, shows the
    chaos floor, MIXED (per step ~1e-8 of scale) must stay within a small factor of it in the bulk."""
    from b747_rl_ctrl_amd import _lib
    from test_gpu_fullsize import _bench_env
    assert _lib.lib().b747_set_specialization(1) == 1
    TK = 20.0
    envs = {v: _bench_env(N, 2024, TK, variant=v) for v in ("fast", "mixed")}
    for v in ("mixed",):                       # the same reset draws (Philox per global env id): same episodes
        for name in ("X", "disc", "k", "mem", "ref", "aero_err", "state0"):
            assert torch.equal(getattr(envs[v], name), getattr(envs["fast"], name)), name
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=TK)
    full.reset(*_device_draws(envs["fast"]))
    g = torch.Generator(device="cuda").manual_seed(7)
    dev = {v: np.zeros(N) for v in envs}       # per env: max over steps of |obs - oracle| / batch scale
    for t in range(2000):
        a = torch.rand(N, device="cuda", generator=g) * 2 - 1
        out = {v: envs[v].step(a) for v in envs}
        o_ref, r_ref, d_ref = full.step(a.cpu().numpy())
        scale = np.maximum(np.abs(o_ref).max(axis=0), 1e-30)
        for v, (obs, rew, done, info) in out.items():
            d = done.cpu().numpy().astype(bool)
            assert np.array_equal(d, d_ref.astype(bool)), f"{v} step {t}: done"
            o = np.where(d[:, None], info["terminal_observation"].cpu().numpy(), obs.cpu().numpy())
            e = np.abs(o.astype(np.float64) - o_ref) / scale
            dev[v] = np.maximum(dev[v], np.nan_to_num(e, nan=np.inf).max(axis=1))
    assert all(int(e.episode.min()) == 2 for e in envs.values())
    q = (50, 90, 99, 99.9, 100)
    lines = []
    for v in envs:
        p = np.percentile(dev[v], q)
        lines.append(f"{v}: max |obs - oracle| / batch scale over the episode, percentiles {q}: "
                     + " ".join(f"{x:.1e}" for x in p))
    rf, rm = envs["fast"].ep_final_return.cpu().numpy(), envs["mixed"].ep_final_return.cpu().numpy()
    rr = np.abs(rm - rf) / np.maximum(np.abs(rf), 1.0)
    lines.append("MIXED vs FAST episode return, relative: percentiles " + " ".join(f"{x:.1e}" for x in np.percentile(rr, q)))
    print("\n" + "\n".join(lines))
    # measured (profiles/r05/pytest_gpu.log): FAST p99 2.2e-11, max 2.7e-8; MIXED p50 6.0e-8, p99 1.8e-5, max 2.3e-2
    # (chaotic envs); MIXED vs FAST return p50 6.5e-8, p99 2.3e-6
    assert np.percentile(dev["fast"], 99) <= 1e-9 and dev["fast"].max() <= 1e-6, lines
    assert np.percentile(dev["mixed"], 50) <= 1e-6 and np.percentile(dev["mixed"], 99) <= 1e-3, lines
    assert np.percentile(rr, 50) <= 1e-6 and np.percentile(rr, 99) <= 1e-4, lines
