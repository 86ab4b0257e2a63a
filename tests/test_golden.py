"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py) against the CPU side.

CPU tier: the faithful oracle, its DLL-ABI build (oracle/build/model_simple.so driven the way
core/model.py drives the DLL), the host build of the compact HIP formulation and the host build of
the Philox reset draws must reproduce the committed vectors -- bit-exact, because they run the same
operations on the same libm.  The GPU tier (test_gpu_golden.py) checks the HIP path against the
same files with the tolerances written there.
"""
import ctypes
import math
import os
import sys

import numpy as np

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))


def _gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def test_c1_oracle_trajectory_matches_fixture():
    g = _gold("c1_pitch_command")
    sig = O.trajectory(2000, consts=g["consts"], vartheta=float(g["vartheta"]), h_zh=float(g["h_zh"]),
                       flags=int(g["flags"]), state0=g["state0"])
    np.testing.assert_array_equal(sig[g["steps"]], g["sig"])


def test_c1_dll_abi_library_matches_fixture():
    """core/model.py:270-279 through the exported-globals ABI (model_simple.so)."""
    g = _gold("c1_pitch_command")
    import ref_env as R
    m = R.RefModel(use_PID_CS=False, initial_state=g["state0"])
    m.hzh = 2000
    m.P = 300000
    m.vartheta_zh = -0.1
    keep = set(int(s) for s in g["steps"])
    rows = []
    for s in range(2000):
        m.step()
        if s in keep:
            st = m.state
            rows.append([m.time, m.dvartheta, *st, m.ITSE, m.deltaz_real])
    ref = g["sig"][:, [0, 1, 5, 6, 7, 8, 9, 10, 19, 28]]
    np.testing.assert_array_equal(np.array(rows), ref)


def test_c2_oracle_and_compact_formulation_match_fixture():
    g = _gold("c2_step_elevator")
    dz = g["deltaz"]
    n = len(dz)
    b = O.Batch(n)
    b.deltaz = dz.copy()
    O.oracle_initialize(b)
    b.deltaz = dz.copy()
    h = O.Batch(n)
    h.deltaz = dz.copy()
    O.oracle_initialize(h)
    h.deltaz = dz.copy()
    prev = 0
    for row, s in enumerate(g["steps"]):
        O.oracle_step(b, int(s) + 1 - prev)
        O.hostcheck_step(h, int(s) + 1 - prev)
        prev = int(s) + 1
        np.testing.assert_array_equal(b.sig.T, g["sig"][row], err_msg=f"oracle step {s}")
        np.testing.assert_array_equal(h.sig.T, g["sig"][row], err_msg=f"compact step {s}")


def test_c3_reset_draws_match_fixture():
    g = _gold("c3_env_episodes")
    s0, ref, ae, _ = O.draw_resets(int(g["seed"]), 0, g["state0"].shape[0], episode=0, mode=0, dist_mode=0)
    np.testing.assert_array_equal(s0, g["state0"])
    np.testing.assert_array_equal(ref, g["ref"])
    np.testing.assert_array_equal(ae, g["aero_err"])
    # Controller.reset distributions (core/controller.py:148-193)
    assert np.all((s0[:, 1] >= 1000) & (s0[:, 1] <= 11000)) and np.all((s0[:, 2] >= 100) & (s0[:, 2] <= 265))
    assert np.all((np.abs(ref[:, 0]) >= math.pi / 180 * 0.999) & (np.abs(ref[:, 0]) <= 10 * math.pi / 180 * 1.001))


def test_c3_env_restatement_matches_fixture():
    g = _gold("c3_env_episodes")
    import ref_env as R
    n = g["state0"].shape[0]
    draws = [O.draw_resets(int(g["seed"]), 0, n, episode=e) for e in (0, 1)]
    for i in range(n):
        c = R.RefController(3, 0, 0, 0, tk=float(g["tk"]))
        e = R.RefControllerEnv(0, 0, True, True, c)
        ep = 0

        def d(ep):
            s0, ref, ae, _ = draws[ep]
            return {"state0": s0[i], "kind": "const", "ref": float(ref[i, 0]), "h": float(ref[i, 7]),
                    "aero_err": ae[i].astype(np.float64)}
        e.reset(d(0))
        for t in range(g["actions"].shape[0]):
            o, r, dn = e.step(g["actions"][t, i])
            assert dn == bool(g["done"][t, i])
            np.testing.assert_array_equal(np.float32(o), g["obs"][t, i])
            assert np.float32(r) == g["reward"][t, i]
            if dn:
                ep += 1
                e.reset(d(ep))


def test_fixtures_load_without_pickle():
    for f in sorted(os.listdir(GOLD)):
        if f.endswith(".npz"):
            z = np.load(os.path.join(GOLD, f), allow_pickle=False)
            assert all(z[k].dtype != object for k in z.files)
