"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle (TEST INFRASTRUCTURE).

The reference ships no tests, fixtures or golden vectors and its DLL may not be executed here
(SURVEY.md 8(c)), so these vectors come from the fp64 oracle (oracle/b747_oracle.c, the DLL
restatement) and its Python env mirror (oracle/ref_env.py).  They freeze the restatement: any
change to the oracle that moves a number shows up as a fixture diff, and the GPU tests check the
HIP path against the same files without needing the oracle libraries.

  python tests/golden/make_golden.py        (after __graft_entry__.build())

Fixtures (numpy .npz, allow_pickle=False):
  c1_pitch_command.npz  BASELINE configs[0]: core/model.py:270-279 scenario, 2000 DLL steps, 1 env
  c2_step_elevator.npz  BASELINE configs[1]: 10 envs, MANUAL, held elevator step -(1+i) deg, 2000 steps
  c3_env_episodes.npz   BASELINE configs[2] env surface: 8 envs (Philox draws, seed 0, ids 0..7),
                        PID_LIKE/CLASSIC/DIRECT/AERO, tk 2 s, 260 env steps (auto-reset at 200)
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_lib as O  # noqa: E402

C1_STEPS = np.r_[np.arange(0, 20), np.arange(24, 2000, 25)]      # rows kept (step index, 0-based)
C2_STEPS = np.arange(0, 2000, 50)
C2_N = 10
C3_N, C3_STEPS, C3_TK, C3_SEED = 8, 260, 2.0, 0


def c1():
    c = O.DEFAULT_CONSTS.copy()
    c[1] = 300000.0                                   # P
    s0 = (100.0, 1000.0, 300.0, 0.0, 0.0, 0.0)
    sig = O.trajectory(2000, consts=c, vartheta=-0.1, h_zh=2000.0, flags=O.F_PID_SS | O.F_RP, state0=s0)
    return dict(consts=c, state0=np.array(s0), vartheta=np.float64(-0.1), h_zh=np.float64(2000.0),
                flags=np.uint8(O.F_PID_SS | O.F_RP), steps=C1_STEPS, sig=sig[C1_STEPS])


def c2():
    dz = -(1 + np.arange(C2_N) % 10) * math.pi / 180
    sig = np.stack([O.trajectory(2000, deltaz=d, flags=O.F_RP) for d in dz], 1)   # [2000, n, 31]
    return dict(deltaz=dz, steps=C2_STEPS, sig=sig[C2_STEPS])


def c3():
    import ref_env as R
    n = C3_N
    draws = [O.draw_resets(C3_SEED, 0, n, episode=e, mode=0, dist_mode=0) for e in (0, 1)]
    rng = np.random.default_rng(11)
    actions = rng.uniform(-1, 1, (C3_STEPS, n)).astype(np.float32)
    obs = np.zeros((C3_STEPS, n, 3), np.float32)
    rew = np.zeros((C3_STEPS, n), np.float32)
    done = np.zeros((C3_STEPS, n), np.uint8)
    for i in range(n):
        ep = 0
        c = R.RefController(3, 0, 0, 0, tk=C3_TK, sample_time=None)
        e = R.RefControllerEnv(0, 0, True, True, c)

        def d(ep):
            s0, ref, ae, _ = draws[ep]
            return {"state0": s0[i], "kind": "const", "ref": float(ref[i, 0]), "h": float(ref[i, 7]),
                    "aero_err": ae[i].astype(np.float64)}
        e.reset(d(0))
        for t in range(C3_STEPS):
            o, r, dn = e.step(actions[t, i])
            obs[t, i], rew[t, i], done[t, i] = o, r, dn
            if dn:
                ep += 1
                e.reset(d(ep))
    s0, ref, ae, _ = draws[0]
    return dict(seed=np.uint64(C3_SEED), tk=np.float64(C3_TK), actions=actions, obs=obs, reward=rew, done=done,
                state0=s0, ref=ref, aero_err=ae)


def main():
    for name, fn in (("c1_pitch_command", c1), ("c2_step_elevator", c2), ("c3_env_episodes", c3)):
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **fn())
        print(f"{path}: {os.path.getsize(path)} B")


if __name__ == "__main__":
    main()
