"""Experiment (GPU): the bench workload (65,536 envs, config 3) split into S env shards stepped on S
independent streams inside one HIP graph -- S chains of one-step launches with no dependency between
chains, so one shard's loads / kernel boundary overlap another shard's compute.  Reports the wall
time per env step of the whole batch.  Usage: python tools/exp_streams.py [S ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

N, STEPS = 65536, 200


def run(S):
    dev = torch.device("cuda")
    per = N // S
    envs = [bench.make_env(per, s, True, dev) for s in range(S)]   # shard s: global ids [s*per, (s+1)*per)
    g = torch.Generator(device=dev).manual_seed(77)
    acts = torch.rand(STEPS + 10, N, generator=g, device=dev) * 2 - 1
    for t in range(10):
        for s, e in enumerate(envs):
            e.step(acts[t, s * per:(s + 1) * per])
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        for st in streams:
            st.wait_stream(cap)
        for t in range(STEPS):
            for s, e in enumerate(envs):
                with torch.cuda.stream(streams[s]):
                    e.step(acts[10 + t, s * per:(s + 1) * per], stream=streams[s])
        for st in streams:
            cap.wait_stream(st)
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    walls = []
    for _ in range(5):
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) / STEPS * 1e6)
    w = sorted(walls)[2]
    print(f"S={S}: {w:7.2f} us per env step of all {N} envs ({N / w * 1e6:.3e} env-steps/s)", flush=True)


if __name__ == "__main__":
    for S in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]:
        run(S)
