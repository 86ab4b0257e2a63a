"""The bench kernels over the bench's OWN episode, every env replayed through the oracle.

bench.py steps 65,536 envs of the reference's training configuration with tk = 20 s (main.py:95-96):
2,000 env steps per episode, the auto-reset at t = 20 s (core/controller.py:317-319), and a CLASSIC
reward whose r3 = 0.2 exp(-kt t) and r4 (ITSE) terms grow with t (env/ctrl_env.py:135-139).  Here:

  * k_env_step_split (b747_env_step, the headline kernel: one launch per env step) for 2,100 steps;
  * the K-step rollout kernel (b747_env_rollout with K = 100, the `rollout` bench line; round 3: k_rollout_split<false>) for 21 launches,

both on all 65,536 envs, and EVERY env's obs / reward / done of EVERY step against the C restatement of
the reference's env loop (oracle/b747_oracle_env.c; bit-identical to oracle/ref_env.py,
tests/test_oracle_env.py), across the auto-reset (terminal observation included), with the device's reset
draws.  Shadow scheme (as tests/test_gpu_model.py): every 50 env steps (per-step kernel) or before every
100-step launch (rollout), the oracle's own compact model state (X, disc, k, mem) is loaded into the GPU
batch, so each window is a free GPU run from the oracle's state and every t in [0, 20] s is covered; the
state the GPU reached at the end of a window is compared with the oracle's before it is overwritten.
Tolerances: done exact; obs / reward as tests/test_gpu_fullsize.py (2e-6 relative + 1e-7 absolute) plus
1e-7 of the component's scale over the batch at that step (its largest |value|, the "of each signal's
range" of DESIGN.md 2).  Measured (tools/exp_replay_drift.py, 100-step windows): the only elements that
need the scale term are dvartheta_dt = (e - e_prev)/h of tumbling envs late in the episode, |e| ~ pi, where
the FAST arithmetic's 1e-9-relative drift in e after ~80 free steps is amplified 100x by the Derivative
block (1.05e-7 absolute on a normalised obs of -6.6e-4, batch scale 16; the same for both kernels)."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_lib as O  # noqa: E402
from test_gpu_fullsize import ATOL, RTOL, _bench_env, _device_draws  # noqa: E402

pytestmark = pytest.mark.gpu

N = 65536
TK = 20.0            # main.py:95-96
SCALE_TOL = 1e-7     # x the component's largest |value| in the batch at that step
STATE_TOL = 1e-7     # GPU state after a <= 100-step window vs the oracle's, per field, relative to max(range, 1)
# MIXED (the flight aerodynamics in fp32) over the same free windows: done exact, obs / reward within a
# per-quantity multiple of FAST's bar set near its measured worst, its state within STATE_TOL_MIXED (fp32 forces: ~1e-8
# of scale per step, grown over up to 100 free steps).  Measured (profiles/r05/pytest_gpu.log, worst error / FAST's
# bar): per-step kernel obs 0.03 / 0.96 / 26.6, reward 316, state 3.4e-6; K = 100 kernel obs 0.03 / 1.8 / 34.4, reward
# 234, state 6.4e-6 -- the worst elements are the chaotic saturated-PID envs late in a window (tests/test_gpu_mixed.py's
# free-running quantiles).  So that a regression of the bulk cannot hide under a bar sized for those few envs, at most
# MIXED_BULK of the envs of any step may exceed FAST's own bar.
MIXED_BAR = {"obs[0]": 1.0, "obs[1]": 5.0, "obs[2]": 100.0, "reward": 1000.0}
MIXED_BULK = 1e-3      # measured worst (round 6): 3.05e-4 (reward, K = 100 kernel)
STATE_TOL_MIXED = 1e-5
_MIXED = [False]   # the running test is MIXED's
_OVER = {}         # largest fraction of a step's envs above FAST's bar, per quantity (MIXED)


def _load_oracle_state(env, full):
    X, disc, k, mem = full.compact_full()
    env.X.copy_(torch.from_numpy(X))
    env.disc.copy_(torch.from_numpy(disc))
    env.k.copy_(torch.from_numpy(k.astype(np.int32)))
    env.mem.copy_(torch.from_numpy(mem))


def _state_drift(env, full):
    """Largest per-field deviation of the GPU state from the oracle's, relative to that field's range
    (q1 = q2 = 0 rows and constant rows fall back to an absolute 1); k and mem must be equal."""
    X, disc, k, mem = full.compact_full()
    assert np.array_equal(env.k.cpu().numpy().astype(np.uint32), k), "step counters differ"
    assert np.array_equal(env.mem.cpu().numpy(), mem), "anti-windup Memory bits differ"
    worst = 0.0
    for got, ref in ((env.X.cpu().numpy(), X), (env.disc.cpu().numpy(), disc)):
        span = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1.0)
        worst = max(worst, float(np.max(np.abs(got - ref) / span)))
    return worst


_WORST = {}   # largest error / tolerance per compared quantity of the running test (printed at its end)


def _close(got, ref, what):
    ref = ref.astype(np.float64)
    err = np.abs(got.astype(np.float64) - ref)
    tol = RTOL * np.abs(ref) + ATOL + SCALE_TOL * float(np.nanmax(np.abs(ref)))
    key = what.split(" step")[0]
    ok = ~(np.isnan(got) & np.isnan(ref))
    if ok.any():
        _WORST[key] = max(_WORST.get(key, 0.0), float(np.max(err[ok] / tol[ok])))
    mult = MIXED_BAR[key] if _MIXED[0] else 1.0
    bad = np.flatnonzero(~((err <= mult * tol) | (np.isnan(got) & np.isnan(ref))))
    assert bad.size == 0, (f"{what}: {bad.size} envs, e.g. env {bad[0]} gpu {got[bad[0]]!r} oracle {ref[bad[0]]!r} "
                           f"(tolerance {mult * tol[bad[0]]:.3g})")
    if _MIXED[0]:
        over = float(np.count_nonzero(ok & (err > tol))) / err.size
        _OVER[key] = max(_OVER.get(key, 0.0), over)
        assert over <= MIXED_BULK, f"{what}: {over:.2%} of the envs above FAST's bar"


def _compare_step(t, full, actions, obs, rew, done, term, env):
    """One env step of the oracle with the same actions; the env's obs is the reset observation (zeros)
    where an episode ended, so the terminal observation is compared there."""
    o_ref, r_ref, d_ref = full.step(actions)
    d = done.cpu().numpy().astype(bool)
    assert np.array_equal(d, d_ref.astype(bool)), f"step {t}: done differs in {np.flatnonzero(d != d_ref)[:10]}"
    o = obs.cpu().numpy()
    if d.any():
        assert np.all(o[d] == 0.0), f"step {t}: the auto-reset observation is all zeros"
        o = np.where(d[:, None], term.cpu().numpy(), o)
    for c in range(o.shape[1]):
        _close(o[:, c], o_ref[:, c], f"obs[{c}] step {t}")
    _close(rew.cpu().numpy(), r_ref.astype(np.float32), f"reward step {t}")
    if d.any():
        full.reset(*_device_draws(env), mask=d)
    return int(d.sum())


@pytest.mark.parametrize("variant", ["fast", "mixed"])
def test_bench_kernel_tk20_episode_every_env_every_step(variant):
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    assert L.b747_set_specialization(1) == 1          # the headline two-wave kernel (k_env_step_split)
    seed = 2024                                       # bench.py's seed
    _WORST.clear()
    _OVER.clear()
    _MIXED[0] = variant == "mixed"
    env = _bench_env(N, seed, TK, variant=variant)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=TK)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(5)
    n_done, drift = 0, 0.0
    for t in range(2100):
        if t % 50 == 0:
            if t:
                drift = max(drift, _state_drift(env, full))
            _load_oracle_state(env, full)
        a = torch.rand(N, device="cuda", generator=g) * 2 - 1
        obs, rew, done, info = env.step(a)
        n_done += _compare_step(t, full, a.cpu().numpy(), obs, rew, done, info["terminal_observation"], env)
        if t == 1999:
            assert n_done == N, "every env ends its episode at t = 20 s"
    assert n_done == N and int(env.episode.min()) == 2 and int(env.episode.max()) == 2
    print(f"\nper-step kernel ({variant}): max state drift over a 50-step window {drift:.2e}; worst error / tolerance "
          + ", ".join(f"{k} {v:.3f}" for k, v in sorted(_WORST.items()))
          + "".join(f"; largest fraction above FAST's bar {k} {v:.2e}" for k, v in sorted(_OVER.items())))
    assert drift <= (STATE_TOL if variant == "fast" else STATE_TOL_MIXED)


@pytest.mark.parametrize("variant", ["fast", "mixed"])
def test_rollout_kernel_k100_tk20_episode_every_env_every_step(variant):
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    assert L.b747_set_specialization(1) == 1          # K-step two-wave kernel (k_rollout_split<false>)
    seed, K = 77, 100
    _WORST.clear()
    _OVER.clear()
    _MIXED[0] = variant == "mixed"
    env = _bench_env(N, seed, TK, variant=variant)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=TK)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(6)
    obs_seq = torch.empty(K, N, 3, device="cuda")
    rew_seq = torch.empty(K, N, device="cuda")
    done_seq = torch.empty(K, N, dtype=torch.uint8, device="cuda")
    n_done, drift = 0, 0.0
    for launch in range(21):                          # 2,100 env steps: the 2,000-step episode + 100
        if launch:
            drift = max(drift, _state_drift(env, full))
        _load_oracle_state(env, full)
        acts = torch.rand(K, N, device="cuda", generator=g) * 2 - 1
        env.rollout(acts, obs_seq, rew_seq, done_seq)
        a_h = acts.cpu().numpy()
        for t in range(K):
            # a done row of obs_seq is the reset observation; the terminal one is env.terminal_obs, which
            # holds the last done of the launch: the tk = 20 s episode ends on a launch's last step
            step = launch * K + t
            if done_seq[t].any():
                assert t == K - 1, f"step {step}: the episode ends on the launch's last step"
            n_done += _compare_step(step, full, a_h[t], obs_seq[t], rew_seq[t], done_seq[t], env.terminal_obs, env)
    assert n_done == N and int(env.episode.min()) == 2 and int(env.episode.max()) == 2
    print(f"\nK = 100 rollout kernel ({variant}): max state drift over a 100-step launch {drift:.2e}; worst error / "
          "tolerance " + ", ".join(f"{k} {v:.3f}" for k, v in sorted(_WORST.items()))
          + "".join(f"; largest fraction above FAST's bar {k} {v:.2e}" for k, v in sorted(_OVER.items())))
    assert drift <= (STATE_TOL if variant == "fast" else STATE_TOL_MIXED)


@pytest.mark.parametrize("sample_time", [0.01, 0.05])
def test_ppo_rollout_kernel_tk20_episode_every_env_every_step(sample_time):
    """The config-5 kernel (b747_ppo_rollout: k_rollout_split<true, double, SUB> + k_policy_value) over the
    tk = 20 s episode of 65,536 envs, every env and every env step against the C env oracle driven by the
    rollout's own clipped actions: sample_time = dt (2,000 env steps, the
    POLICY instantiation's late-episode r3 / r4 terms) and main.py's sample_time = 0.05 (main.py:18: 5 DLL
    steps per env step, 400 env steps per episode; core/controller.py:258-264).  Launches of 50 DLL steps, the
    oracle's compact state loaded before each (the shadow scheme above), 2,100 DLL steps: across the auto-reset
    at t = 20 s, where done, the terminal observation, ep_final_len (2,000 or 400: exact) and ep_final_return
    (VecMonitor's float32 accumulation of the episode's float64 rewards) are checked."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    _MIXED[0] = False                                 # FAST: the bar itself
    n_sub = int(round(sample_time / 0.01))
    per_launch = 50 // n_sub                          # env steps per launch (50 DLL steps)
    ep_steps = int(round(TK / sample_time))
    env = _bench_env(N, 11, TK, sample_time=sample_time)
    env.track_episodes()
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=sample_time, tk=TK)
    full.reset(*_device_draws(env))
    ppo = PPO(env, PPOConfig(n_steps=per_launch, batch_size=N), seed=1, rollout_kernel=True)
    assert ppo.rollout_kernel
    g = torch.Generator(device="cuda").manual_seed(4)
    with torch.no_grad():
        for prm in ppo.policy.parameters():           # break the ortho-init symmetry / scale
            prm.add_(0.05 * torch.randn(prm.shape, generator=g, device="cuda"))
    ppo.sync_params()
    prev_obs = np.zeros((N, 3), np.float32)           # the reset observation
    ref_rewards, n_done, drift = [], 0, 0.0
    for launch in range(2100 // 50):
        if launch:
            drift = max(drift, _state_drift(env, full))
        _load_oracle_state(env, full)
        ppo.collect_rollouts(per_launch)
        obs_b, rew_b = ppo.obs_buf.cpu().numpy(), ppo.rew_buf.cpu().numpy()
        done_b = ppo.done_buf.cpu().numpy().astype(bool)
        act_b = ppo.act_buf[..., 0].clamp(-1, 1).cpu().numpy()
        for t in range(per_launch):
            step = launch * per_launch + t
            for c in range(3):
                _close(obs_b[t, :, c], prev_obs[:, c], f"obs the policy saw [{c}] step {step}")
            o_ref, r_ref, d_ref = full.step(act_b[t])
            ref_rewards.append(np.array(r_ref, np.float64))    # (a copy: the oracle reuses its buffer)
            d = done_b[t]
            assert np.array_equal(d, d_ref), f"step {step}: done differs in {np.flatnonzero(d != d_ref)[:10]}"
            _close(rew_b[t], r_ref.astype(np.float32), f"reward step {step}")
            if d.any():
                assert step == ep_steps - 1 and d.all() and t == per_launch - 1, f"step {step}: the episode end"
                term = env.terminal_obs.cpu().numpy()
                for c in range(3):
                    _close(term[:, c], o_ref[:, c], f"terminal obs [{c}] step {step}")
                full.reset(*_device_draws(env), mask=d)
                n_done += int(d.sum())
            prev_obs = np.where(d[:, None], 0.0, o_ref).astype(np.float32)
    assert n_done == N and int(env.episode.min()) == 2 and int(env.episode.max()) == 2
    assert bool((env.ep_final_len == ep_steps).all()), "ep_final_len: the episode's env steps, exactly"
    assert bool((env.ep_stats[0] == 1).all()) and bool((env.ep_stats[2] == ep_steps).all())
    ret = np.zeros(N, np.float32)                     # SB3 VecMonitor: float32 returns += float64 rewards
    peak = np.zeros(N)                                # largest |partial return| of the episode
    for t in range(ep_steps):
        ret = (ret.astype(np.float64) + ref_rewards[t]).astype(np.float32)
        peak = np.maximum(peak, np.abs(ret))
    got = env.ep_final_return.cpu().numpy()
    assert np.array_equal(got.astype(np.float32).astype(np.float64), got), "the return is float32-valued"
    # the kernel accumulates its own float64 reward (FAST: the f32 hardware exp, <= 2e-7 from the oracle's), so a
    # step's float32 rounding of the return can differ by one ulp of the partial return where the two rewards
    # straddle a rounding boundary (measured: 85 of 65,536 envs, one ulp): 4 float32 ulps of the largest partial sum
    err = np.abs(got - ret)
    tol = 4 * np.float32(2.0 ** -23) * np.maximum(peak, 1.0)
    assert bool((err <= tol).all()), (f"{int((err > tol).sum())} returns beyond 4 ulps, worst "
                                      f"{float((err / tol).max()):.2f} x the bound")
    print(f"\nPPO rollout kernel, sample_time {sample_time}: max state drift over a 50-DLL-step launch {drift:.2e}")
    assert drift <= STATE_TOL
