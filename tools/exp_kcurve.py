"""Per-launch env-step time against the step within the episode (GPU): b747_env_time_steps over one whole
20 s episode (2000 steps + the auto-reset) of the bench workload, HIP events around every launch;
prints the median per 100-step bucket.  Also a HIP-graph period per bucket (K = 100 launches)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    n = 65536
    env = bench.make_env(n, 0, True, torch.device("cuda"))
    acts = torch.rand(2100, n, device="cuda") * 2 - 1
    ms = env.time_steps(acts)
    print("isolated launch (events), median us per 100-step bucket:")
    print(" ".join(f"{int(np.median(ms[b:b + 100]) * 1e3 * 100) / 100:.2f}" for b in range(0, 2100, 100)), flush=True)
    env.reset()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        for t in range(100):
            env.step(acts[t])
    torch.cuda.synchronize()
    env.reset()
    torch.cuda.synchronize()
    per = []
    for b in range(21):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        per.append((time.perf_counter() - t0) / 100 * 1e6)
    print("graph period (K = 100 replay incl. ~25 us fixed), us per step per 100-step bucket:")
    print(" ".join(f"{p:.2f}" for p in per), flush=True)


if __name__ == "__main__":
    main()
