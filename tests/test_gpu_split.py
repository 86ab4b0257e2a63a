"""The two-wave single-step env kernel (csrc/b747_split.h: every env over a flight and a control wave) against
the one-wave single-step kernel it replaces (k_env_steps<double, FAST, 3, K1>), same configuration and
actions, on a batch whose last workgroup is partial, across auto-resets.  Both are the FAST variant, whose
translation unit contracts mul+add pairs into FMAs wherever the compiler finds them: the two kernels may
pick a different product of a sum to fuse (the DSS update A x + B u, the force sums), so the state agrees
to the ulp level (<= 1e-13 of each component's range over 100-step episodes, as
test_gpu_env.py::test_specialised_kernel_equals_generic_kernel), float32 obs / reward to float32 rounding,
and done flags, step counters, episode counters and reset draws exactly.  The oracle anchoring of the
bench kernel is tests/test_gpu_fullsize.py, which runs whichever kernel b747_env_step selects -- this one
by default."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(n, tk, x_f64=True, sample_time=None):
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType, \
        ResetRefMode, RewardType
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=tk, seed=31, x_f64=x_f64,
                              sample_time=sample_time)


# fp64 X: ulp-level; fp32 X: both kernels round the same fp64 stage result to fp32 once per step, so a
# value within ~1e-13 of an fp32 rounding boundary can land one fp32 ulp apart and carry forward
_TOL = {True: dict(x=1e-13, rtol=2e-6, atol=1e-7, ret_atol=1e-5, disc=1e-12),
        False: dict(x=1e-5, rtol=1e-4, atol=1e-5, ret_atol=1e-3, disc=1e-5)}


@pytest.mark.parametrize("x_f64", [True, False])
def test_two_wave_kernel_equals_one_wave_kernel(x_f64):
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    tol = _TOL[x_f64]
    n, tk, steps = 65536 - 37, 1.0, 260
    split, one = _env(n, tk, x_f64), _env(n, tk, x_f64)
    g = torch.Generator(device="cuda").manual_seed(9)
    prev = L.b747_set_specialization(1)
    worst = 0.0
    try:
        for t in range(steps):
            a = torch.rand(n, generator=g, device="cuda") * 2 - 1
            L.b747_set_specialization(1)
            split.step(a)
            L.b747_set_specialization(2)
            one.step(a)
            for f in ("done", "k", "mem", "episode", "state0", "ref", "aero_err", "flags"):
                assert torch.equal(getattr(split, f), getattr(one, f)), f"step {t + 1}: {f}"
            xs, xo = split.X.double(), one.X.double()
            scale = xo.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
            err = float(((xs - xo).abs() / scale).max())
            worst = max(worst, err)
            assert err <= tol["x"], f"step {t + 1}: X {err:.3e}"
            torch.testing.assert_close(split.obs, one.obs, rtol=tol["rtol"], atol=tol["atol"], msg=f"step {t + 1}: obs")
            torch.testing.assert_close(split.reward, one.reward, rtol=tol["rtol"], atol=tol["atol"],
                                       msg=f"step {t + 1}: reward")
            torch.testing.assert_close(split.ep_return, one.ep_return, rtol=tol["rtol"], atol=tol["ret_atol"])
        assert int(split.episode.min()) >= 3          # every env went through two auto-resets
        dsc = one.disc.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
        assert float(((split.disc - one.disc).abs() / dsc).max()) <= tol["disc"]
    finally:
        L.b747_set_specialization(prev)
    print(f"max state difference {worst:.2e} of range")


def test_two_wave_kernel_writes_rollout_rows():
    """b747_env_rollout with K = 1 (the two-launch PPO path) goes through the same kernel: obs / reward /
    done rows equal the env's own buffers."""
    n = 4096
    env = _env(n, 0.3)
    a = torch.rand(1, n, device="cuda") * 2 - 1
    obs_seq = torch.zeros(1, n, 3, device="cuda")
    rew_seq = torch.zeros(1, n, device="cuda")
    done_seq = torch.zeros(1, n, dtype=torch.uint8, device="cuda")
    for t in range(35):
        env.rollout(a, obs_seq, rew_seq, done_seq)
        torch.cuda.synchronize()
        assert torch.equal(obs_seq[0], env.obs) and torch.equal(rew_seq[0], env.reward)
        assert torch.equal(done_seq[0].bool(), env.done)
    assert int(env.episode.min()) == 2                 # done at step 30, auto-reset


@pytest.mark.parametrize("extra_flag", [1, 8])   # F_PID_SS, F_RL: delta depends on the pitch error
def test_lock_step_fallback_equals_one_wave_kernel(extra_flag):
    """Workgroups holding an env whose flags put the SS PID (1) or its dead zone (8) into the loop run the two
    waves in lock step (delta of a stage needs that stage's pitch error): same results as the one-wave kernel,
    for those envs and for the plain MANUAL envs sharing their workgroups."""
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    n, tk, steps = 3000, 0.6, 130
    split, one = _env(n, tk), _env(n, tk)
    for e in (split, one):
        e.flags[::97] |= extra_flag | 1               # (the dead zone acts on the SS PID's output)
    g = torch.Generator(device="cuda").manual_seed(5)
    prev = L.b747_set_specialization(1)
    try:
        for t in range(steps):
            a = torch.rand(n, generator=g, device="cuda") * 2 - 1
            L.b747_set_specialization(1)
            split.step(a)
            L.b747_set_specialization(2)
            one.step(a)
            for f in ("done", "k", "mem", "episode", "flags"):
                assert torch.equal(getattr(split, f), getattr(one, f)), f"step {t + 1}: {f}"
            scale = one.X.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
            err = float(((split.X - one.X).abs() / scale).max())
            assert err <= 1e-13, f"step {t + 1}: X {err:.3e}"
            torch.testing.assert_close(split.obs, one.obs, rtol=2e-6, atol=1e-7, msg=f"step {t + 1}: obs")
            torch.testing.assert_close(split.reward, one.reward, rtol=2e-6, atol=1e-7, msg=f"step {t + 1}: reward")
        assert int(split.episode.min()) >= 3
    finally:
        L.b747_set_specialization(prev)


@pytest.mark.parametrize("n", [1, 63, 257])   # one env; a partial first wave; one env past a full workgroup
def test_tiny_and_ragged_batches_equal_one_wave_kernel(n):
    """The workgroup's idle lanes (past N, stepping a copy of env N-1, storing nothing) in batches far below one
    workgroup, across an auto-reset (tk = 0.3 s: done at step 30)."""
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    split, one = _env(n, 0.3), _env(n, 0.3)
    g = torch.Generator(device="cuda").manual_seed(3)
    prev = L.b747_set_specialization(1)
    try:
        for t in range(40):
            a = torch.rand(n, generator=g, device="cuda") * 2 - 1
            L.b747_set_specialization(1)
            split.step(a)
            L.b747_set_specialization(2)
            one.step(a)
            for f in ("done", "k", "mem", "episode", "state0", "ref", "aero_err", "flags"):
                assert torch.equal(getattr(split, f), getattr(one, f)), f"step {t + 1}: {f}"
            scale = one.X.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
            assert float(((split.X - one.X).abs() / scale).max()) <= 1e-13, f"step {t + 1}: X"
            torch.testing.assert_close(split.obs, one.obs, rtol=2e-6, atol=1e-7)
            torch.testing.assert_close(split.reward, one.reward, rtol=2e-6, atol=1e-7)
        assert int(split.episode.min()) == 2
    finally:
        L.b747_set_specialization(prev)


_ROLLOUT_FLOAT = ("obs", "reward", "terminal_obs", "ep_return", "ep_final_return", "deltaz", "vartheta", "h_zh",
                  "state0", "upid")
_ROLLOUT_EXACT = ("done", "k", "mem", "episode", "ep_len", "ep_final_len", "ref", "aero_err", "flags", "ref_kind",
                  "tp")


@pytest.mark.parametrize("case", ["f64", "f32", "lockstep", "sub5", "sub5_f32", "sub5_lockstep", "sub5_misaligned",
                                  "sub5_k1"])
def test_k_step_two_wave_rollout_equals_one_wave_rollout(case):
    """b747_env_rollout with K = 64 (k_rollout_split<false>, the two-wave step in a loop on per-pair hand-offs, state in registers,
    stored once) against the one-wave K-step kernel (b747_set_specialization(2)) over three launches with
    auto-resets (tk = 0.3 s), on a batch whose last workgroup is partial: every obs / reward / done row and
    every env slot the launches leave behind (env_store with a reset in the launch), the episode
    accumulators included.
    sub5*: main.py's sample_time = 0.05 (5 DLL steps per env step, core/controller.py:258-264; the SUB
    instantiation, which also serves the per-step API at n_sub > 1: sub5_k1 = K 1); sub5_misaligned: every env's
    step counter starts at k = 0..4 (a batch stepped before with another sample_time), so its first env step of the
    first launch takes 5 - k % 5 DLL steps (Controller.step stops at the next multiple of n_sub)."""
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    sub = case.startswith("sub5")
    n, K = 4096 + 320, (1 if case == "sub5_k1" else (16 if sub else 64))
    launches = 40 if case == "sub5_k1" else 3
    x_f64 = not case.endswith("f32")
    envs = [_env(n, 0.3, x_f64, 0.05 if sub else None) for _ in range(2)]
    for e in envs:
        e.track_episodes()
        if case.endswith("lockstep"):
            e.flags[::97] |= 1                         # SS PID in the loop: those workgroups run in lock step
        if case == "sub5_misaligned":
            e.k.copy_(torch.arange(n, device="cuda", dtype=e.k.dtype) % 5)
    g = torch.Generator(device="cuda").manual_seed(7)
    tol = _TOL[x_f64]
    prev = L.b747_set_specialization(1)
    try:
        for it in range(launches):
            acts = torch.rand(K, n, generator=g, device="cuda") * 2 - 1
            seqs = []
            for e, spec in zip(envs, (1, 2)):
                L.b747_set_specialization(spec)
                o = torch.zeros(K, n, 3, device="cuda")
                r = torch.zeros(K, n, device="cuda")
                d = torch.zeros(K, n, dtype=torch.uint8, device="cuda")
                e.rollout(acts, o, r, d)
                seqs.append((o, r, d))
            torch.cuda.synchronize()
            (o1, r1, d1), (o2, r2, d2) = seqs
            s, w = envs
            assert torch.equal(d1, d2), f"launch {it}: done rows"
            torch.testing.assert_close(o1, o2, rtol=tol["rtol"], atol=tol["atol"])
            torch.testing.assert_close(r1, r2, rtol=tol["rtol"], atol=tol["atol"])
            for f in _ROLLOUT_EXACT:
                assert torch.equal(getattr(s, f), getattr(w, f)), f"launch {it}: {f}"
            for f in _ROLLOUT_FLOAT + ("ep_stats",):
                torch.testing.assert_close(getattr(s, f), getattr(w, f), rtol=tol["rtol"], atol=tol["ret_atol"],
                                           msg=lambda m: f"launch {it}: {f}: {m}")
            for name in ("X", "disc"):
                xs, xo = getattr(s, name).double(), getattr(w, name).double()
                scale = xo.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
                err = float(((xs - xo).abs() / scale).max())
                assert err <= max(tol["x"], tol["disc"]), f"launch {it}: {name} {err:.2e}"
    finally:
        L.b747_set_specialization(prev)
    if sub:
        assert int(envs[0].k.max()) % 5 == 0 and bool((envs[0].k % 5 == 0).all())   # aligned after any env step
        assert int(envs[0].episode.min()) >= 3
    else:
        assert int(envs[0].episode.min()) >= 6         # every env reset several times across the launches


def test_workgroup_geometry_does_not_change_results():
    """The per-step kernel runs 64 envs per workgroup up to 32,768 envs and 256 above; the K-step rollout 64 up to
    16,384 (b747_fast.hip).  Env i's reset draws depend only on its global id, so the first 16,384 envs of a 40,000-env
    batch (256 per workgroup) and a 16,384-env batch (64 per workgroup) step the same envs.  The two instantiations
    are the same source but compile separately (register allocation differs; the FAST unit's FMA contraction may fuse
    differently), so, as between any two kernels here: X within 1e-13 and the discrete state within 1e-12 of each
    component's range, float32
    obs / reward to float32 rounding, the integer state exactly -- 60 per-step launches across auto-resets, then three
    16-step rollout launches (24,576 envs: 256 per workgroup; 8,192: 64)."""
    m = 16384
    big, small = _env(40000, 0.3), _env(m, 0.3)
    g = torch.Generator(device="cuda").manual_seed(12)

    def check(what, m):
        for f in ("k", "mem", "episode", "done", "flags", "aero_err", "ref"):
            assert torch.equal(getattr(big, f)[..., :m], getattr(small, f)), f"{what}: {f}"
        for f, tol in (("X", 1e-13), ("disc", 1e-12)):   # (disc: the Derivative inputs magnify ulps by 1/h, _TOL)
            b, s_ = getattr(big, f)[..., :m].double(), getattr(small, f).double()
            scale = s_.abs().amax(dim=1, keepdim=True).clamp_min(1e-300)
            err = float(((b - s_).abs() / scale).max())
            assert err <= tol, f"{what}: {f} {err:.3e}"
        torch.testing.assert_close(big.obs[:m], small.obs, rtol=2e-6, atol=1e-7, msg=what)
        torch.testing.assert_close(big.reward[:m], small.reward, rtol=2e-6, atol=1e-7, msg=what)
        torch.testing.assert_close(big.ep_return[:m], small.ep_return, rtol=2e-6, atol=1e-5, msg=what)

    for t in range(60):
        a = torch.rand(40000, generator=g, device="cuda") * 2 - 1
        big.step(a)
        small.step(a[:m])
        check(f"step {t + 1}", m)
    assert int(small.episode.min()) >= 2              # (across an auto-reset)
    m2 = 8192
    big, small = _env(24576, 0.3), _env(m2, 0.3)
    for launch in range(3):
        a = torch.rand(16, 24576, generator=g, device="cuda") * 2 - 1
        big.rollout(a)
        small.rollout(a[:, :m2].contiguous())
        check(f"rollout {launch + 1}", m2)
