"""The HIP path (through the C ABI) against the committed golden fixtures (tests/golden/).

Tolerances (written here):
  * model trajectories (c1, c2), per signal, |gpu - gold| / max_t|gold| over the kept rows:
      FAITHFUL variant <= 1e-9, FAST variant <= 1e-6    (north-star gate: 1e-5)
    step counter / sim_time exact.
  * env surface (c3): reset draws state0 <= 1e-12 relative, ref exact, aero_err <= 1e-14 relative (float64
    normal draws: the device's log / cos against the host build's libm);
    obs and reward float32 within 2e-6 relative + 1e-7 absolute; done exact; the finished
    episode's obs is info["terminal_observation"], and the auto-reset obs is all zeros.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = {"faithful": 1e-9, "fast": 1e-6}


def _gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def _colrel(got, ref):
    scale = np.max(np.abs(ref), axis=0, keepdims=True)
    scale = np.where(scale > 0, scale, 1.0)
    return np.max(np.abs(got - ref) / scale, axis=0)


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_c1_pitch_command(variant):
    from b747_rl_ctrl_amd import BatchModel
    g = _gold("c1_pitch_command")
    m = BatchModel(1, use_PID_CS=False, initial_state=g["state0"], variant=variant)
    m.hzh = 2000
    m.P = 300000
    m.vartheta_zh = -0.1
    rows, prev = [], 0
    for s in g["steps"]:
        m.step(int(s) + 1 - prev)
        prev = int(s) + 1
        rows.append(m.sig[:, 0].cpu().numpy())
    got = np.array(rows)
    np.testing.assert_array_equal(got[:, 0], g["sig"][:, 0])        # sim_time = k * h exactly
    rel = _colrel(got, g["sig"])
    assert rel.max() <= TOL[variant], f"worst signal {np.argmax(rel)}: {rel.max():.3e}"


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_c2_step_elevator(variant):
    from b747_rl_ctrl_amd import BatchModel
    g = _gold("c2_step_elevator")
    dz = g["deltaz"]
    m = BatchModel(len(dz), use_PID_CS=False, use_PID_SS=False, variant=variant)
    m.deltaz = torch.from_numpy(dz)
    rows, prev = [], 0
    for s in g["steps"]:
        m.step(int(s) + 1 - prev)
        prev = int(s) + 1
        rows.append(m.sig.T.cpu().numpy())
    got = np.array(rows)                                            # [rows, n, 31]
    for i in range(len(dz)):
        rel = _colrel(got[:, i], g["sig"][:, i])
        assert rel.max() <= TOL[variant], f"env {i} worst signal {np.argmax(rel)}: {rel.max():.3e}"


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_c3_env_episodes(variant):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    g = _gold("c3_env_episodes")
    n = g["state0"].shape[0]
    env = BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                             CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                             disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=float(g["tk"]),
                             seed=int(g["seed"]), variant=variant)
    np.testing.assert_allclose(env.state0.T.cpu().numpy(), g["state0"], rtol=1e-12, atol=0)
    np.testing.assert_array_equal(env.ref.T.cpu().numpy(), g["ref"])
    np.testing.assert_allclose(env.aero_err.T.cpu().numpy(), g["aero_err"], rtol=1e-14, atol=0)
    acts = torch.from_numpy(g["actions"]).cuda()
    for t in range(acts.shape[0]):
        obs, rew, done, info = env.step(acts[t])
        d = done.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(d, g["done"][t].astype(bool), err_msg=f"done step {t}")
        o = np.where(d[:, None], info["terminal_observation"].cpu().numpy(), obs.cpu().numpy())
        np.testing.assert_allclose(o, g["obs"][t], rtol=2e-6, atol=1e-7, err_msg=f"obs step {t}")
        np.testing.assert_allclose(rew.cpu().numpy(), g["reward"][t], rtol=2e-6, atol=1e-7,
                                   err_msg=f"reward step {t}")
        if d.any():
            assert np.all(obs.cpu().numpy()[d] == 0.0)
