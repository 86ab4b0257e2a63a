"""Batched ControlTestCallback metrics (b747_rl_ctrl_amd/evaluate.py run_step_tests) against the
reference's single-env loop restated on the CPU (oracle/ref_env.py with the Storage hook recording
after every DLL step, core/controller.py:209-228, and calc_stepinfo, oracle/stepinfo_ref.py).

The policy is a fixed linear law a = float32(-3 * obs[1]) (exact IEEE float32 on both sides; the
float32 observations agree to 2e-6 relative, see test_gpu_env.py), so the trajectories agree to
~1e-6 and the metrics within: overshoot 1e-3 relative, rise/settling time within one sample
(0.01 s), static error 1e-5 deg, quality 1e-6 relative."""
import math
import os
import sys

import numpy as np
import pytest
import torch

from stepinfo_ref import calc_stepinfo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_env as R  # noqa: E402

pytestmark = pytest.mark.gpu

REFS = [5 * math.pi / 180, -5 * math.pi / 180, 10 * math.pi / 180, -10 * math.pi / 180]   # neural/agent.py:117
STATE0 = [0, 11000, 250, 0, 0, 0]
TK, ST = 10.0, 0.05


def _cpu_episode(vref):
    c = R.RefController(3, 0, None, None, tk=TK, sample_time=ST)
    e = R.RefControllerEnv(0, 0, True, True, c)
    obs = e.reset({"state0": np.array(STATE0, float), "kind": "const", "ref": vref, "aero_err": None})
    t, th = [], []

    def rec(m):
        t.append(m.time)
        th.append(float(np.nan_to_num(m.state[4])) * 180 / math.pi)
    done = False
    while not done:
        a = np.float32(-3.0) * np.float32(obs[1])
        obs, _, done = e.step(a, rec)
    info = calc_stepinfo(th, vref * 180 / math.pi, ts=t)
    return info, c.quality()


def test_batched_step_tests_match_the_single_env_callback():
    from b747_rl_ctrl_amd.evaluate import run_step_tests
    out = run_step_tests(lambda o: -3.0 * o[:, 1], REFS, state0=STATE0, tk=TK, sample_time=ST)
    assert bool(out["done"].all())
    for j, vref in enumerate(REFS):
        info, q = _cpu_episode(vref)
        assert float(out["overshoot"][j]) == pytest.approx(abs(info["overshoot"]), rel=1e-3)
        for k in ("rise_time", "settling_time"):
            if info[k] is None:
                assert math.isnan(float(out[k][j]))
            else:
                assert abs(float(out[k][j]) - info[k]) <= 0.0100001, (k, float(out[k][j]), info[k])
        assert float(out["static_error"][j]) == pytest.approx(info["static_error"], abs=1e-5)
        assert float(out["quality"][j]) == pytest.approx(q, rel=1e-6)
    assert float(out["mean_quality"]) == pytest.approx(float(out["quality"].mean()))


def test_record_signals_gives_every_dll_step():
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, RewardType
    env = BatchControllerEnv(64, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                             CtrlMode.DIRECT_CONTROL, sample_time=0.05, tk=5)
    env.record_signals(True)
    env.reset()
    env.step(torch.zeros(64, device="cuda"))
    t = env.signal("sim_time")
    assert t.shape == (5, 64)
    torch.testing.assert_close(t[:, 0], torch.tensor([0.01, 0.02, 0.03, 0.04, 0.05], dtype=torch.float64,
                                                     device="cuda"), rtol=0, atol=1e-15)
