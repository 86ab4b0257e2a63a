"""Kernel timing probe (GPU): per-launch HIP-event time of b747_env_step, HIP-graph launch period,
and per-step time of K-step rollout launches, on the bench workload (65,536 envs, config 3)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="current")
    ap.add_argument("--variant", default="fast")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--tk", type=float, default=None, help="episode length override (s)")
    a = ap.parse_args()
    n = a.n
    env = bench.make_env(n, 0, True, torch.device("cuda"), variant=a.variant)
    if a.tk is not None:
        env.cfg.tk = a.tk
    acts = torch.rand(400, n, device="cuda") * 2 - 1
    for t in range(10):
        env.step(acts[t])
    torch.cuda.synchronize()
    ms = env.time_steps(acts[:100])
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        for t in range(200):
            env.step(acts[t])
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    periods = []
    for _ in range(5):   # median of 5 replays of the 200-launch graph
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        periods.append((time.perf_counter() - t0) / 200 * 1e6)
    period = sorted(periods)[2]
    roll = {}
    for K in (1, 10, 100):
        reps = max(1, 200 // K)
        env.rollout(acts[:K])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            env.rollout(acts[:K])
        torch.cuda.synchronize()
        roll[K] = (time.perf_counter() - t0) / (reps * K) * 1e6
    print(f"{a.tag:>12s}  launch(events) mean {ms.mean() * 1e3:6.2f} min {ms.min() * 1e3:6.2f} us | graph period "
          f"{period:6.2f} us ({n / period * 1e6:.3e}/s) | rollout us/step K=1 {roll[1]:6.2f} K=10 {roll[10]:6.2f} "
          f"K=100 {roll[100]:6.2f} ({n / roll[100] * 1e6:.3e}/s)", flush=True)


if __name__ == "__main__":
    main()
