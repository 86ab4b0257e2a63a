"""End-to-end PPO training throughput (bench.py ppo_training_rate) alone, for profiling the update.
Run: python tools/exp_ppo_train.py [--iterations 2]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iterations", type=int, default=2)
ap.add_argument("--profile", action="store_true", help="torch.profiler table of one PPO.train")
a = ap.parse_args()
if not a.profile:
    print(json.dumps(bench.ppo_training_rate(65536, 0, torch.device("cuda"), "fast", iterations=a.iterations)))
    sys.exit(0)
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from b747_rl_ctrl_amd.ppo import PPO, PPOConfig  # noqa: E402
env = bench.make_env(65536, 0, True, torch.device("cuda"), seed=98, sample_time=0.05)
ppo = PPO(env, PPOConfig(n_steps=64, batch_size=65536), seed=0)
ppo.last_obs.copy_(env.obs)
ppo.collect_rollouts(64)
ppo.compute_gae(64)
ppo.train(64)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    ppo.train(64)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30))
