"""The float32 storage of the reset draws, measured (aero_err and the pitch reference).

The reference passes the drawn aero errors (numpy float64, core/controller.py:181-193) and pitch
reference (Python float, :150-152) to the DLL in float64.  The GPU path stores both as float32
(b747_env_batch.aero_err / .ref, include/b747.h), so the dynamics run on the float32-rounded values.
This test runs the CPU restatement of the reference (oracle/ref_env.py over the DLL-ABI oracle) on
the same draws twice -- float64 as the reference, float32-rounded as the GPU -- for a 2000-step
episode under a fixed linear control law, and bounds the gap it makes in the observations and
rewards: far below the north-star per-step gate of 1e-5 (the rounding is ~3e-8 relative in the
inputs, and the closed loop does not amplify it)."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_env as R  # noqa: E402


def _episode(draws, steps=2000):
    c = R.RefController(3, 0, 0, disturbance_mode=0, tk=20, sample_time=None)
    e = R.RefControllerEnv(0, 0, True, True, c)
    obs = e.reset(draws)
    o_all, r_all = [], []
    for _ in range(steps):
        a = np.float32(np.clip(-3.0 * obs[1] - 0.5 * obs[2], -1, 1))
        obs, r, _ = e.step(a)
        o_all.append(obs)
        r_all.append(r)
    return np.array(o_all), np.array(r_all)


def test_float32_draws_change_the_episode_far_below_the_gate():
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(3):
        s0 = np.array([0, rng.uniform(1000, 11000), rng.uniform(100, 265), rng.uniform(-20, 20), 0,
                       rng.uniform(-1e-3, 1e-3)])
        ref = rng.uniform(math.pi / 180, 10 * math.pi / 180) * rng.choice([-1.0, 1.0])
        aero = rng.normal([-0.1, 0.1, -0.1, -0.1, 0.1], 0.5)
        d64 = {"state0": s0, "kind": "const", "ref": float(ref), "aero_err": aero}
        d32 = {"state0": s0, "kind": "const", "ref": float(np.float32(ref)),
               "aero_err": aero.astype(np.float32).astype(np.float64)}
        o64, r64 = _episode(d64)
        o32, r32 = _episode(d32)
        scale = np.maximum(np.abs(o64).max(0), 1e-12)
        gap = max(float(np.max(np.abs(o32 - o64) / scale)), float(np.max(np.abs(r32 - r64)) / np.abs(r64).max()))
        worst = max(worst, gap)
    print(f"float32 draw rounding: worst relative gap over 3 x 2000 steps {worst:.2e}")
    assert worst < 1e-6                       # measured 1.6e-7 (seed 7); the gate is 1e-5
