"""Env-step time against the step within the episode (GPU): a 100-launch graph replayed 21 times from a fresh
reset (one 20 s episode + the auto-reset), HIP events around each replay."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    n = 65536
    env = bench.make_env(n, 0, True, torch.device("cuda"))
    acts = torch.rand(2100, n, device="cuda") * 2 - 1
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for b in range(21):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) * 10)
    print("K = 100 graph replays from a fresh reset, event us per step per 100-step bucket:")
    print(" ".join(f"{p:.2f}" for p in per), flush=True)


if __name__ == "__main__":
    main()
