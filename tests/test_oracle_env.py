"""The C restatement of the env loop (oracle/b747_oracle_env.c, b747oe_*) against the Python one
(oracle/ref_env.py): both drive the same DLL-faithful oracle model, so obs (float32), reward
(float64) and done must agree bit for bit in every observation / reward / control / reset mode."""
import math
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

sys.path.insert(0, os.path.join(O.ROOT, "oracle"))
import ref_env as R  # noqa: E402

N = 6


def _draws(rng, n, osc=False, hybrid=False, h0=None):
    s0 = np.stack([np.zeros(n), rng.uniform(1000, 11000, n), rng.uniform(100, 265, n), rng.uniform(-20, 20, n),
                   np.zeros(n), rng.uniform(-1e-3, 1e-3, n)])
    ref = np.zeros((8, n), np.float64)
    ref[0] = rng.uniform(1, 10, n) * np.pi / 180 * rng.choice([-1, 1], n)
    ref[1:4] = rng.uniform(0, 0.05, (3, n))
    ref[4:7] = rng.uniform(0.01, 0.5, (3, n))
    ref[7] = s0[1] + rng.uniform(-1000, 1000, n)
    kind = np.full(n, 1 if osc else 0, np.uint8)
    aero = rng.normal([[-0.1], [0.1], [-0.1], [-0.1], [0.1]], 0.5, (5, n))   # float64, as the reference draws
    hyb = rng.integers(0, 2, n).astype(bool) if hybrid else None
    return s0, ref, kind, aero, hyb


def _as_ref_draw(d, i):
    s0, ref, kind, aero, hyb = d
    out = {"state0": s0[:, i], "kind": "osc" if kind[i] else "const", "ref": float(ref[0, i]),
           "osc": tuple(float(x) for x in ref[1:7, i]), "h": float(ref[7, i]), "aero_err": aero[:, i].astype(np.float64)}
    if hyb is not None:
        out["hybrid_ctrl"] = bool(hyb[i])
    return out


CASES = [  # obs, reward, ctrl_type, ctrl_mode, osc, hybrid, limiter, sample_time
    (0, 0, 3, 0, False, False, False, None),
    (1, 0, 3, 1, True, False, False, 0.05),
    (2, 1, 3, 3, False, False, False, 0.05),
    (3, 2, 3, 2, False, False, True, None),   # QUALITY divides by vref^2: the reference raises at an OSC zero
    (4, 3, 2, 0, False, True, False, 0.05),
    (0, 4, 3, 0, True, False, False, 0.05),
    (4, 1, 1, None, False, False, False, None),
    (1, 0, 0, None, False, False, False, 0.05),
]


@pytest.mark.parametrize("case", CASES, ids=[f"obs{c[0]}-rew{c[1]}-ct{c[2]}-cm{c[3]}" for c in CASES])
def test_c_env_restatement_equals_python_restatement(case):
    obs_t, rew_t, ctrl_t, mode, osc, hybrid, limiter, st = case
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    use_ctrl, manual = ctrl_t in (0, 2), ctrl_t in (2, 3)
    flags = O.F_RP | (O.F_PID_CS if use_ctrl else 0) | (0 if manual else O.F_PID_SS)
    tk = 0.6
    E = O.EnvOracle(N, obs_t, rew_t, mode, flags=flags, use_limiter=limiter, sample_time=st, tk=tk)
    refs = []
    for i in range(N):
        c = R.RefController(ctrl_t, mode, 2 if hybrid else 0, tk=tk, sample_time=st, use_limiter=limiter)
        refs.append(R.RefControllerEnv(obs_t, rew_t, True, True, c))
    d = _draws(rng, N, osc, hybrid)
    fresh = None if d[4] is None else np.where(d[4], O.F_RP | O.F_PID_CS, O.F_RP).astype(np.uint8)
    E.reset(d[0], d[1], d[2], d[3], fresh_flags=fresh)
    for i, e in enumerate(refs):
        e.reset(_as_ref_draw(d, i))
    n_done = 0
    for t in range(150):
        a = rng.uniform(-1, 1, N).astype(np.float32)
        obs, rew, done = E.step(a)
        for i, e in enumerate(refs):
            o_ref, r_ref, d_ref = e.step(a[i])
            assert np.array_equal(obs[i], o_ref.astype(np.float32)), f"step {t} env {i} obs"
            assert rew[i] == r_ref or (math.isnan(rew[i]) and math.isnan(r_ref)), f"step {t} env {i} reward"
            assert bool(done[i]) == d_ref, f"step {t} env {i} done"
        if done.any():
            n_done += int(done.sum())
            d = _draws(rng, N, osc, hybrid)
            fresh = None if d[4] is None else np.where(d[4], O.F_RP | O.F_PID_CS, O.F_RP).astype(np.uint8)
            E.reset(d[0], d[1], d[2], d[3], mask=done, fresh_flags=fresh)
            for i in np.flatnonzero(done):
                refs[i].reset(_as_ref_draw(d, i))
    assert n_done >= N


def test_compact_full_export_is_the_batch_oracles_state():
    """b747oe_export_full (the GPU shadow tests load it into a device batch) returns the same compact
    state as the batched model oracle reaches from the same initial state and elevator sequence."""
    rng = np.random.default_rng(4)
    n = 5
    d = _draws(rng, n)
    env = O.EnvOracle(n, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=20.0)
    env.reset(d[0], d[1], d[2], d[3])
    b = O.Batch(n)
    b.flags[:] = O.F_RP
    b.state0 = d[0].copy()
    b.aero_err = d[3].astype(np.float64)
    O.oracle_initialize(b)
    for t in range(37):
        a = rng.uniform(-1, 1, n).astype(np.float32)
        env.step(a)
        b.deltaz = (a.astype(np.float64) * (17 * math.pi / 180)).astype(np.float32).astype(np.float64)
        b.vartheta = d[1][0].astype(np.float64)
        O.oracle_step(b, 1)
    X, disc, k, mem = env.compact_full()
    X2, k2 = env.compact()
    assert np.array_equal(X, X2) and np.array_equal(k, k2)
    assert np.array_equal(X, b.X) and np.array_equal(disc, b.disc) and np.array_equal(k, b.k)
    assert np.array_equal(mem, b.mem)


def test_nan_and_inf_actions_c_restatement_equals_python_restatement():
    """Non-finite actions (a diverged policy): ControllerEnv.step scales and hands them to the DLL as they are
    (env/ctrl_env.py:262-264, core/controller.py:242), and NaN spreads through the delay line, the DSS and
    the rate limiter's comparisons until the auto-reset at tk.  Both restatements must agree bit for bit
    (NaN where the other has NaN); the GPU is checked against the C one (tests/test_gpu_nonfinite.py)."""
    rng = np.random.default_rng(12)
    tk, n = 0.6, N
    E = O.EnvOracle(n, 0, 0, 0, flags=O.F_RP, sample_time=None, tk=tk)
    refs = [R.RefControllerEnv(0, 0, True, True, R.RefController(3, 0, 0, tk=tk, sample_time=None)) for _ in range(n)]
    d = _draws(rng, n)
    E.reset(d[0], d[1], d[2], d[3])
    for i, e in enumerate(refs):
        e.reset(_as_ref_draw(d, i))
    # the 0.05 s DSS samples the 0.03 s-delayed command only on its ticks: a single non-finite step can fall
    # between them, so env 0 and env 3 get five NaN steps; -inf / +inf are clamped by the rate limiter
    # (fall > du holds against -inf), NaN passes it (every comparison is false)
    bad = {t: (0, np.nan) for t in range(5, 10)}
    bad.update({12: (1, np.inf), 13: (2, -np.inf), 14: (2, -np.inf)})
    bad.update({t: (3, np.nan) for t in range(40, 45)})
    n_nan = 0
    for t in range(130):
        a = rng.uniform(-1, 1, n).astype(np.float32)
        if t in bad:
            a[bad[t][0]] = bad[t][1]
        obs, rew, done = E.step(a)
        for i, e in enumerate(refs):
            o_ref, r_ref, d_ref = e.step(a[i])
            assert np.array_equal(obs[i], o_ref.astype(np.float32), equal_nan=True), f"step {t} env {i} obs"
            assert rew[i] == r_ref or (math.isnan(rew[i]) and math.isnan(r_ref)), f"step {t} env {i} reward"
            assert bool(done[i]) == d_ref, f"step {t} env {i} done"
        n_nan += int(np.isnan(obs).any(axis=1).sum())
        if done.any():
            d = _draws(rng, n)
            E.reset(d[0], d[1], d[2], d[3], mask=done)
            for i in np.flatnonzero(done):
                refs[i].reset(_as_ref_draw(d, i))
    assert n_nan > 0, "the non-finite actions should reach the observations"
