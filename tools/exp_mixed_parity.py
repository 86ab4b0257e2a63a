"""Per-step divergence of a library build from the C env oracle on the bench workload (GPU): every step the
oracle's compact state is loaded into the GPU batch, one env step is taken on both, and the obs / reward of
every env are compared -- the north star's "<= 1e-5 rel per-step divergence" measured directly.  Used to
qualify the MIXED variant (variant="mixed") against the fp64 FAST build (round 4 ran it on the
B747_FLIGHT_F32 experiment builds that became MIXED; --lib selects any build).
Run: python tools/exp_mixed_parity.py [--lib tools/ab/e_f32.so] [--steps 300]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--variant", default="fast")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--tk", type=float, default=1.0)
    a = ap.parse_args()
    import b747_rl_ctrl_amd._lib as L
    if a.lib:
        L.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import oracle_lib as O
    from test_gpu_episode_replay import _load_oracle_state
    from test_gpu_fullsize import _device_draws
    import bench
    env = bench.make_env(a.n, 0, True, torch.device("cuda"), variant=a.variant)
    env.cfg.tk = a.tk
    full = O.EnvOracle(a.n, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=a.tk)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(5)
    worst = {"obs0": 0.0, "obs1": 0.0, "obs2": 0.0, "reward": 0.0}
    worst_abs = dict(worst)
    for t in range(a.steps):
        _load_oracle_state(env, full)
        act = torch.rand(a.n, device="cuda", generator=g) * 2 - 1
        obs, rew, done, info = env.step(act)
        o_ref, r_ref, d_ref = full.step(act.cpu().numpy())
        d = done.cpu().numpy().astype(bool)
        assert np.array_equal(d, d_ref), f"step {t}: done differs"
        o = np.where(d[:, None], info["terminal_observation"].cpu().numpy(), obs.cpu().numpy()).astype(np.float64)
        for c in range(3):
            ref = o_ref[:, c].astype(np.float64)
            err = np.abs(o[:, c] - ref)
            scale = max(float(np.abs(ref).max()), 1e-30)
            worst[f"obs{c}"] = max(worst[f"obs{c}"], float(np.max(err / np.maximum(np.abs(ref), 1e-3 * scale))))
            worst_abs[f"obs{c}"] = max(worst_abs[f"obs{c}"], float(err.max()))
        ref = r_ref.astype(np.float64)
        err = np.abs(rew.cpu().numpy().astype(np.float64) - ref)
        worst["reward"] = max(worst["reward"], float(np.max(err / np.maximum(np.abs(ref), 1e-3))))
        worst_abs["reward"] = max(worst_abs["reward"], float(err.max()))
        if d.any():
            full.reset(*_device_draws(env), mask=d)
    print(f"lib {a.lib or 'libb747.so'} variant {a.variant}: {a.n} envs x {a.steps} steps, per-step max relative error (floor 1e-3 of the "
          f"component's batch max): " + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) +
          " | max abs: " + ", ".join(f"{k} {v:.2e}" for k, v in worst_abs.items()))


if __name__ == "__main__":
    main()
