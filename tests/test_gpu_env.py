"""GPU parity of the fused env step (b747_env_step through the C ABI) against the CPU restatement
of the reference's Python loop (oracle/ref_env.py: Model/Controller/ControllerEnv mirrors over
oracle/build/model_simple.so, the DLL-ABI build of the fp64 oracle).

Random resets: the GPU draws ICs / references / aero errors with Philox; the test reads those
draws back from device memory and hands them to the CPU env, so both run identical episodes.
Tolerance: obs and reward are float32 outputs of fp64 arithmetic on both sides; they must agree
to 2e-6 relative (+1e-7 absolute) -- the fp64 results differ only at the 1e-13 level (libm ulps
amplified by the Derivative blocks), so this only absorbs float32 rounding-boundary flips.
done flags, episode lengths and step counters must match exactly.
"""
import math
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_env as R  # noqa: E402

pytestmark = pytest.mark.gpu

RTOL, ATOL = 2e-6, 1e-7


def _draws(env, i):
    """What Controller.reset drew for env i on the GPU (read back from device)."""
    s0 = env.state0[:, i].cpu().numpy().astype(np.float64)
    kind = "osc" if int(env.ref_kind[i]) == 1 else "const"
    ref = env.ref[:, i].cpu().numpy().astype(np.float64)
    d = {"state0": s0, "kind": kind, "ref": float(ref[0]), "osc": tuple(float(x) for x in ref[1:7]),
         "h": float(ref[7]), "aero_err": env.aero_err[:, i].cpu().numpy().astype(np.float64)}
    if env.reset_ref_mode is not None and env.reset_ref_mode.value == 2:
        d["hybrid_ctrl"] = bool(int(env.flags[i]) & 2)
    return d


def _run(obs_type, rew_type, ctrl_type, ctrl_mode, reset_mode, n=8, steps=90, tk=1.5, sample_time=0.05,
         use_limiter=False, disturbance=None, seed=7, norm=True, rew_config=None, actions_scale=1.0):
    from b747_rl_ctrl_amd import BatchControllerEnv
    env = BatchControllerEnv(n, obs_type, rew_type, norm, norm, ctrl_type, ctrl_mode, reset_ref_mode=reset_mode,
                             disturbance_mode=disturbance, tk=tk, sample_time=sample_time, use_limiter=use_limiter,
                             seed=seed, reward_config=rew_config)
    if reset_mode is None:   # deterministic per-env ICs and references
        rng = np.random.default_rng(seed)
        s0 = np.stack([np.zeros(n), rng.uniform(1000, 11000, n), rng.uniform(100, 265, n), rng.uniform(-20, 20, n),
                       np.zeros(n), rng.uniform(-1e-3, 1e-3, n)], 1)
        env.set_state0(torch.from_numpy(s0))
        env.set_reference(vartheta=torch.from_numpy(rng.uniform(-0.17, 0.17, n)),
                          h=torch.from_numpy(s0[:, 1] + rng.uniform(-500, 500, n)))
        env.reset()
    ctrl_args = dict(tk=tk, sample_time=sample_time, use_limiter=use_limiter, action_max=env.action_max)
    refs = []
    for i in range(n):
        c = R.RefController(ctrl_type.value, None if ctrl_mode is None else ctrl_mode.value,
                            None if reset_mode is None else reset_mode.value, **ctrl_args)
        e = R.RefControllerEnv(obs_type.value, rew_type.value, norm, norm, c, rew_config)
        e.reset(_draws(env, i))
        refs.append(e)
    rng = np.random.default_rng(seed + 1)
    n_done = 0
    for t in range(steps):
        a = (rng.uniform(-1, 1, n) * actions_scale).astype(np.float32)
        obs, rew, done, info = env.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        term = info["terminal_observation"].cpu().numpy()
        for i, e in enumerate(refs):
            o_ref, r_ref, d_ref = e.step(a[i])
            assert bool(done[i]) == d_ref, f"step {t} env {i}: done {done[i]} vs {d_ref}"
            got_o = term[i] if d_ref else obs[i]
            np.testing.assert_allclose(got_o, o_ref.astype(np.float32), rtol=RTOL, atol=ATOL,
                                       err_msg=f"obs step {t} env {i}")
            np.testing.assert_allclose(rew[i], np.float32(r_ref), rtol=RTOL, atol=ATOL,
                                       err_msg=f"reward step {t} env {i}")
            if d_ref:
                n_done += 1
                assert np.all(obs[i] == 0.0), "auto-reset obs must be all zeros (A.6)"
                e.reset(_draws(env, i))
    return env, n_done


MANUAL_MODES = ["DIRECT_CONTROL", "ADD_PROC_CONTROL", "ANG_VEL_CONTROL", "ADD_DIRECT_CONTROL"]


@pytest.mark.parametrize("mode", MANUAL_MODES)
def test_manual_modes_const_reset_classic(mode):
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    scale = {"ADD_PROC_CONTROL": 1.0, "ANG_VEL_CONTROL": 1.0}.get(mode, 1.0)
    env, n_done = _run(ObservationType.PID_LIKE, RewardType.CLASSIC, CtrlType.MANUAL, CtrlMode[mode],
                       ResetRefMode.CONST, actions_scale=scale)
    assert n_done >= 8      # tk = 1.5 s = 30 env steps: every env finished 3 episodes


@pytest.mark.parametrize("obs", ["PID_LIKE", "SPEED_MODE", "PID_AERO", "PID_SPEED_AERO", "MODEL_STATE"])
def test_observation_types(obs):
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    _run(ObservationType[obs], RewardType.CLASSIC, CtrlType.MANUAL, CtrlMode.DIRECT_CONTROL, ResetRefMode.OSCILLATING,
         steps=40)


@pytest.mark.parametrize("rew", ["CLASSIC", "PID_LIKE", "QUALITY", "MINIMAL", "TF_REFERENCE"])
def test_reward_types(rew):
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    _run(ObservationType.PID_LIKE, RewardType[rew], CtrlType.MANUAL, CtrlMode.ADD_DIRECT_CONTROL, ResetRefMode.CONST,
         steps=40)


def test_hybrid_reset_and_aero_disturbance():
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, DisturbanceMode, ObservationType, ResetRefMode, RewardType
    env, _ = _run(ObservationType.SPEED_MODE, RewardType.CLASSIC, CtrlType.MANUAL, CtrlMode.DIRECT_CONTROL,
                  ResetRefMode.HYBRID, disturbance=DisturbanceMode.AERO_DISTURBANCE, n=12, steps=70)
    fl = env.flags.cpu().numpy()
    assert (fl & 2).any() and not (fl & 2).all(), "HYBRID should mix SEMI_MANUAL and MANUAL envs"
    assert float(env.aero_err.abs().max()) > 0


@pytest.mark.parametrize("ctrl", ["AUTO", "FULL_AUTO", "SEMI_MANUAL"])
def test_pid_control_types_explicit_state0(ctrl):
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, ObservationType, RewardType
    mode = None if ctrl in ("AUTO", "FULL_AUTO") else CtrlMode.DIRECT_CONTROL
    _run(ObservationType.MODEL_STATE, RewardType.PID_LIKE, CtrlType[ctrl], mode, None, steps=40, tk=3.0)


def test_limiter_and_dt_sampling():
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    _run(ObservationType.PID_LIKE, RewardType.CLASSIC, CtrlType.MANUAL, CtrlMode.DIRECT_CONTROL, ResetRefMode.CONST,
         use_limiter=True, sample_time=None, tk=0.5, steps=120)


def test_rollout_equals_step_loop():
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    mk = lambda: BatchControllerEnv(1000, ObservationType.SPEED_MODE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                                    CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST, tk=1.0,
                                    sample_time=0.05, seed=3)
    e1, e2 = mk(), mk()
    T = 50
    acts = torch.rand(T, 1000, device="cuda") * 2 - 1
    obs_seq = torch.zeros(T, 1000, e1.obs_dim, device="cuda")
    rew_seq = torch.zeros(T, 1000, device="cuda")
    done_seq = torch.zeros(T, 1000, dtype=torch.uint8, device="cuda")
    e1.rollout(acts, obs_seq, rew_seq, done_seq)
    for t in range(T):
        o, r, d, _ = e2.step(acts[t])
        assert torch.equal(o, obs_seq[t]) and torch.equal(r, rew_seq[t]) and torch.equal(d, done_seq[t].bool())
    assert torch.equal(e1.X, e2.X) and torch.equal(e1.ep_return, e2.ep_return)


def test_reset_draw_distributions_and_sharding_independence():
    """Philox streams are keyed by global env id: a shard at env_offset reproduces the same envs."""
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, ResetRefMode, RewardType
    mk = lambda n, off: BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True,
                                           CtrlType.MANUAL, CtrlMode.DIRECT_CONTROL,
                                           reset_ref_mode=ResetRefMode.CONST, seed=11, env_offset=off)
    full, shard = mk(65536, 0), mk(16384, 32768)
    assert torch.equal(full.state0[:, 32768:49152], shard.state0)
    s0 = full.state0.cpu().numpy()
    assert 1000 <= s0[1].min() and s0[1].max() <= 11000 and abs(s0[1].mean() - 6000) < 60
    assert 100 <= s0[2].min() and s0[2].max() <= 265
    ref = full.ref[0].cpu().numpy()
    assert np.all(np.abs(ref) >= math.pi / 180 - 1e-6) and np.all(np.abs(ref) <= 10 * math.pi / 180 + 1e-6)
    assert abs((ref > 0).mean() - 0.5) < 0.02


def _spec(on):
    from b747_rl_ctrl_amd import _lib
    return _lib.lib().b747_set_specialization(int(on))


@pytest.mark.parametrize("sample_time", [None, 0.05])
def test_training_config_parity_specialised_kernel(sample_time):
    """The reference's training configuration (PID_LIKE, CLASSIC, MANUAL/DIRECT, CONST resets, drawn AERO
    errors) runs the config-specialised kernel (b747_set_specialization): parity with the CPU env."""
    from b747_rl_ctrl_amd import CtrlMode, CtrlType, DisturbanceMode, ObservationType, ResetRefMode, RewardType
    assert _spec(True) == 1
    env, n_done = _run(ObservationType.PID_LIKE, RewardType.CLASSIC, CtrlType.MANUAL, CtrlMode.DIRECT_CONTROL,
                       ResetRefMode.CONST, disturbance=DisturbanceMode.AERO_DISTURBANCE, sample_time=sample_time,
                       tk=0.5 if sample_time is None else 1.5, steps=120 if sample_time is None else 90)
    assert n_done >= 8


def test_specialised_kernel_equals_generic_kernel():
    """Same inputs through the config-specialised and the generic env kernel over 200 steps with
    auto-resets (tk = 1 s), plus a 100-step rollout launch.  Both are the FAST variant, whose translation
    unit contracts mul+add pairs into FMAs wherever the compiler finds them: the two instantiations may
    fuse differently (a product with fewer uses once the specialised read-out drops signals), so the
    state agrees to the ulp level (<= 1e-13 of each component's range; the CPU-oracle parity tests bound
    both kernels), float32 obs / reward to float32 rounding, done flags and episode counters exactly."""
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    mk = lambda: BatchControllerEnv(4096, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                                    CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                                    disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=1.0, sample_time=None,
                                    seed=11)
    g = torch.Generator(device="cuda").manual_seed(4)
    acts = torch.rand(300, 4096, device="cuda", generator=g) * 2 - 1
    out = []
    for on in (True, False):
        _spec(on)
        try:
            e = mk()
            o_seq = torch.zeros(100, 4096, e.obs_dim, device="cuda")
            r_seq = torch.zeros(100, 4096, device="cuda")
            d_seq = torch.zeros(100, 4096, dtype=torch.uint8, device="cuda")
            obs, rew, done, xs = [], [], [], []
            for t in range(200):
                o, r, d, _ = e.step(acts[t])
                obs.append(o.clone()); rew.append(r.clone()); done.append(d.clone()); xs.append(e.X.clone())
            e.rollout(acts[200:], o_seq, r_seq, d_seq)
            torch.cuda.synchronize()
            out.append(dict(obs=torch.stack(obs), rew=torch.stack(rew), done=torch.stack(done), X=torch.stack(xs),
                            o_seq=o_seq, r_seq=r_seq, d_seq=d_seq, ep=e.episode.clone(), k=e.k.clone()))
        finally:
            _spec(True)
    s, g_ = out
    assert int(s["done"].sum()) > 4096   # every env reset at least once (tk = 100 steps)
    for key in ("done", "d_seq", "ep", "k"):
        assert torch.equal(s[key], g_[key]), key
    scale = g_["X"].abs().amax(dim=(0, 2), keepdim=True).clamp_min(1e-300)
    assert float(((s["X"] - g_["X"]).abs() / scale).max()) <= 1e-13
    for key in ("obs", "rew", "o_seq", "r_seq"):
        torch.testing.assert_close(s[key], g_[key], rtol=2e-6, atol=1e-7, msg=key)
