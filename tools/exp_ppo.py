"""Probe: config-5 rollout (fused policy + env step) for rocprofv3 kernel timing."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from b747_rl_ctrl_amd.ppo import PPO, PPOConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
tag = sys.argv[2] if len(sys.argv) > 2 else ""
env = bench.make_env(n, 0, True, torch.device("cuda"))
ppo = PPO(env, PPOConfig(n_steps=64), seed=0, rollout_kernel=False if tag.endswith("split") else None)   # split: 2 launches/step
for use_graph in (False, True):
    ppo.collect_rollouts(64, use_graph=use_graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ppo.collect_rollouts(64, use_graph=use_graph)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (3 * 64)
    print(f"{tag} graph={use_graph}: {dt * 1e6:.2f} us/step -> {n / dt:.3e} env-steps/s", flush=True)
