"""Does the env-step time drift under sustained load (GPU)?  A 100-launch graph is replayed back to back
for ~3 s; the per-step time of every 20th replay is printed with the elapsed time."""
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
    acts = torch.rand(100, n, device="cuda") * 2 - 1
    for t in range(5):
        env.step(acts[t])
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        for t in range(100):
            env.step(acts[t])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    out = []
    for r in range(2000):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        if r % 50 == 0:
            out.append(f"{time.perf_counter() - t_start:5.2f}s {e0.elapsed_time(e1) * 10:6.2f}")
        if time.perf_counter() - t_start > float(os.environ.get("SECS", "3")):
            break
    print(" | ".join(out), flush=True)


if __name__ == "__main__":
    main()
