"""The reset draws reach the dynamics in float64, as in the reference (ABI v7).

The reference hands the DLL float64 values: numpy normal draws for aero_err (core/controller.py:181-193,
the DLL's double aero_err[5], core/model.py:164) and Python-float references (:153-177).  Through ABI v6
the env batch stored both as float32 (a ~3e-8 relative rounding of every coefficient); since v7
b747_env_batch.aero_err / .ref are double.  On the CPU: the host build of the product's draw_reset
(b747_env.h, the code every reset kernel runs; tests/native/hostcheck.cpp) returns draws that float32
cannot hold, and the C env restatement the GPU replays are checked against sees the difference -- so a
path that rounded them again would fail the replays (tests/test_gpu_fullsize.py,
tests/test_gpu_episode_replay.py), not just move them."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_lib as O  # noqa: E402


def test_host_draws_are_float64_and_not_float32_representable():
    n = 4096
    for mode in (0, 1, 2):                                   # CONST, OSCILLATING, HYBRID
        s0, ref, ae, fl = O.draw_resets(3, 0, n, episode=1, mode=mode, dist_mode=0)
        assert ref.dtype == np.float64 and ae.dtype == np.float64
        lossy = lambda a: np.mean(a.astype(np.float32).astype(np.float64) != a)
        assert lossy(ae) > 0.99, "aero_err draws rounded to float32"
        cols = {0: [0], 1: [1, 2, 3, 4, 5, 6], 2: [0, 7]}[mode]
        live = ref[:, cols][ref[:, cols] != 0]
        assert live.size and lossy(live) > 0.99, f"reset mode {mode}: references rounded to float32"


def test_the_env_oracle_sees_float32_rounding_of_the_draws():
    n, steps = 64, 300
    s0, ref, ae, _ = O.draw_resets(5, 0, n, episode=0, mode=0, dist_mode=0)
    kind = np.zeros(n, np.uint8)
    rounded = lambda a: a.astype(np.float32).astype(np.float64)
    out = []
    for r, a in ((ref, ae), (rounded(ref), rounded(ae))):
        e = O.EnvOracle(n, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=20.0)
        e.reset(s0.T.copy(), r.T.copy(), kind, a.T.copy())
        acts = np.random.default_rng(1).uniform(-1, 1, (steps, n)).astype(np.float32)
        o = [e.step(acts[t])[0].copy() for t in range(steps)]
        out.append(np.array(o))
    gap = np.abs(out[0] - out[1]).max()
    assert gap > 0.0, "float32-rounded draws should change the observations"
    print(f"\nfloat32 rounding of the draws moves the 300-step observations by up to {gap:.2e}")
