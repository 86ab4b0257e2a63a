"""Non-finite actions through the bench kernels, every env against the C env restatement (GPU).

A diverged policy hands the env NaN or +-inf.  ControllerEnv.step passes them on unchanged
(env/ctrl_env.py:262-264, core/controller.py:242): the DLL's 0.03 s delay line and 0.05 s DSS pick a
command up only around a DSS tick, its rate limiter clamps +-inf (one of its comparisons holds) and passes
NaN (none does), and a NaN state stays NaN until the auto-reset at tk.  tests/test_oracle_env.py checks
the C restatement against the Python one for exactly this; here the per-step split kernel
(b747_env_step, kind 3), the generic one-wave kernel and the K-step split kernel (b747_env_rollout) must
give the same obs / reward / done as the C restatement in every env, NaN where it has NaN."""
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

N, STEPS, TK = 4096, 130, 0.6


def _actions(seed):
    g = np.random.default_rng(seed)
    a = g.uniform(-1, 1, (STEPS, N)).astype(np.float32)
    a[5:10, ::37] = np.nan          # five steps: the DSS tick samples at least one
    a[12, 1::41] = np.inf
    a[13:15, 2::43] = -np.inf
    a[40:45, 3::29] = np.nan
    return a


def _close(got, ref, what):
    ref = ref.astype(np.float64)
    got = got.astype(np.float64)
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), f"{what}: NaN pattern differs in {np.flatnonzero(nan_g != nan_r)[:8]}"
    ok = ~nan_r
    g, r = got[ok], ref[ok]
    inf = np.isinf(r) | np.isinf(g)                      # +-inf must match exactly (the rf reward term)
    assert np.array_equal(g[inf], r[inf]), f"{what}: infinities differ"
    g, r = g[~inf], r[~inf]
    err = np.abs(g - r)
    tol = RTOL * np.abs(r) + ATOL
    bad = np.flatnonzero(err > tol)
    assert bad.size == 0, f"{what}: {bad.size} envs off, e.g. {g[bad[0]]!r} vs {r[bad[0]]!r}"


@pytest.mark.parametrize("kernel", ["split", "generic", "rollout"])
def test_nonfinite_actions_match_the_env_oracle(kernel):
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    prev = L.b747_set_specialization(0 if kernel == "generic" else 1)
    try:
        env = _bench_env(N, 31, TK)
        full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=TK)
        full.reset(*_device_draws(env))
        acts = _actions(3)
        K = 10
        n_nan = 0
        for t0 in range(0, STEPS, K):
            if kernel == "rollout":
                obs_seq = torch.empty(K, N, 3, device="cuda")
                rew_seq = torch.empty(K, N, device="cuda")
                done_seq = torch.empty(K, N, dtype=torch.uint8, device="cuda")
                env.rollout(torch.from_numpy(acts[t0:t0 + K]).cuda(), obs_seq, rew_seq, done_seq)
                rows = [(obs_seq[t], rew_seq[t], done_seq[t]) for t in range(K)]
                term = env.terminal_obs
            else:
                rows = []
                for t in range(K):
                    o, r, d, info = env.step(torch.from_numpy(acts[t0 + t]).cuda())
                    rows.append((o.clone(), r.clone(), d.clone(), info["terminal_observation"].clone()))
            for t in range(K):
                o, r, d = rows[t][:3]
                o_ref, r_ref, d_ref = full.step(acts[t0 + t])
                dn = d.cpu().numpy().astype(bool)
                assert np.array_equal(dn, d_ref.astype(bool)), f"{kernel} step {t0 + t}: done"
                oh = o.cpu().numpy()
                if dn.any():   # the finished episode's obs is the terminal observation
                    tm = (rows[t][3] if kernel != "rollout" else term).cpu().numpy()
                    oh = np.where(dn[:, None], tm, oh)
                for c in range(3):
                    _close(oh[:, c], o_ref[:, c], f"{kernel} step {t0 + t} obs[{c}]")
                _close(r.cpu().numpy(), r_ref.astype(np.float32), f"{kernel} step {t0 + t} reward")
                n_nan += int(np.isnan(o_ref).any(axis=1).sum())
                if dn.any():
                    full.reset(*_device_draws(env), mask=dn)
        assert n_nan > 0
    finally:
        L.b747_set_specialization(prev)
