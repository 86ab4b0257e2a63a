"""Which detail of bench.py's protocol changes the env-step time (GPU)?  Variants by flags:
--setdev (torch.cuda.set_device first), --gen (actions from a seeded device Generator), --rows R (actions
tensor rows), --distinct (graph steps use rows warmup + t instead of t).  Prints the per-step event time
of the second replay of a 100-launch graph."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--setdev", action="store_true")
    ap.add_argument("--gen", action="store_true")
    ap.add_argument("--rows", type=int, default=100)
    ap.add_argument("--distinct", action="store_true")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    if a.setdev:
        torch.cuda.set_device(dev)
    n, K, W = 65536, 100, 5
    env = bench.make_env(n, 0, True, dev)
    g = torch.Generator(device=dev).manual_seed(77) if a.gen else None
    acts = torch.rand(a.rows, n, generator=g, device=dev) * 2 - 1
    for t in range(W):
        env.step(acts[t])
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for t in range(K):
            env.step(acts[(W + t) % a.rows if a.distinct else t % a.rows])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for r in range(4):
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / K)
    print(f"{a.tag:>12s} per-step event us over 4 replays: " + " ".join(f"{x:.2f}" for x in res), flush=True)


if __name__ == "__main__":
    main()
