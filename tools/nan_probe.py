"""Diagnostic (GPU): find envs of the bench workload whose state turns non-finite, and replay them
through the C restatement of the env loop (oracle/b747_oracle_env.c) with the same actions.
python tools/nan_probe.py [--shard 6] [--steps 800]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
from test_gpu_fullsize import N, _bench_env, _device_draws  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard", type=int, default=6)
    ap.add_argument("--steps", type=int, default=800)
    a = ap.parse_args()
    env = _bench_env(N, 2024, 20, env_offset=a.shard * N)
    draws = _device_draws(env)
    g = torch.Generator(device="cuda").manual_seed(9)
    acts, first_bad = [], torch.full((N,), -1, dtype=torch.int64, device="cuda")
    for t in range(a.steps):
        full_a = torch.rand(8 * N, device="cuda", generator=g) * 2 - 1
        act = full_a[a.shard * N:(a.shard + 1) * N]
        acts.append(act.cpu().numpy())
        env.step(act)
        bad = ~torch.isfinite(env.X).all(0)
        first_bad = torch.where(bad & (first_bad < 0), torch.full_like(first_bad, t), first_bad)
    idx = torch.nonzero(first_bad >= 0).flatten().cpu().numpy()
    print(f"shard {a.shard}: {idx.size} envs non-finite within {a.steps} steps: {idx[:10]} at {first_bad[idx[:10]].tolist()}")
    if idx.size == 0:
        return
    i = int(idx[0])
    s0, ref, rk, ae = draws
    print("env", i, "state0", s0[:, i], "ref", ref[0, i], "aero", ae[:, i])
    env2 = _bench_env(N, 2024, 20, env_offset=a.shard * N)      # second pass: the GPU trajectory of env i
    gx = []
    for t in range(int(first_bad[i]) + 3):
        env2.step(torch.from_numpy(acts[t]).cuda())
        gx.append(env2.X[:, i].cpu().numpy())
    orc = O.EnvOracle(1, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=20.0)
    orc.reset(s0[:, i:i + 1], ref[:, i:i + 1], rk[i:i + 1], ae[:, i:i + 1])
    for t in range(a.steps):
        o, r, d = orc.step(acts[t][i:i + 1])
        X, k = orc.compact()
        if t % 50 == 0 or not np.isfinite(X).all() or t >= int(first_bad[i]) - 3:
            print(f"oracle t={t} k={k[0]} obs={o[0]} r={r[0]:.4g} d={d[0]} h={X[1,0]:.6g} Vx={X[6,0]:.6g} "
                  f"Vy={X[7,0]:.6g} wz={X[8,0]:.6g} q0={X[2,0]:.6g} q3={X[5,0]:.6g}")
            if t < len(gx):
                G = gx[t]
                print(f"   gpu t={t} h={G[1]:.6g} Vx={G[6]:.6g} Vy={G[7]:.6g} wz={G[8]:.6g} q0={G[2]:.6g} q3={G[5]:.6g}")
        if not np.isfinite(X).all() or t > int(first_bad[i]) + 2:
            break


if __name__ == "__main__":
    main()
