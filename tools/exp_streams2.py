"""Experiment (GPU): does splitting the bench batch (65,536 envs, the two-wave per-step kernel) into S env
shards on S streams let one shard's launch ramp / tail / kernel boundary overlap another's compute?

Two ranks sharing one GPU measured 6.85e9 env-steps/s together against 6.3e9 for one rank alone
(profiles/r03/bench_2ranks_gloo_one_gpu.json): kernels from two queues overlap.  Round 1's
tools/exp_streams.py captured the S streams into ONE HIP graph and saw them serialise.  Here, per S:
  * seq:   each shard's K launches issued by one C call (b747_env_step_seq) on its own stream, the S
           calls back to back from the host (eager, no graph);
  * graph: each shard's K launches captured in its own graph, the S graphs replayed on S streams.
Wall time per env step of the whole batch (median of 5).  Usage: python tools/exp_streams2.py [S ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

N, K = 65536, 400


def run(S):
    dev = torch.device("cuda")
    per = N // S
    envs = [bench.make_env(per, s, True, dev) for s in range(S)]   # shard s: global ids [s*per, (s+1)*per)
    g = torch.Generator(device=dev).manual_seed(77)
    acts = torch.rand(K + 10, N, generator=g, device=dev) * 2 - 1
    shard_acts = [acts[:, s * per:(s + 1) * per].contiguous() for s in range(S)]
    for s, e in enumerate(envs):
        e.step_seq(shard_acts[s][:10])
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    out = {}
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, e in enumerate(envs):
            e.step_seq(shard_acts[s][10:], stream=streams[s])
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) / K * 1e6)
    out["seq"] = sorted(walls)[2]
    graphs = []
    for s, e in enumerate(envs):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=streams[s]):
            for t in range(K):
                e.step(shard_acts[s][10 + t], stream=streams[s])
        graphs.append(gr)
    torch.cuda.synchronize()
    for s, gr in enumerate(graphs):
        with torch.cuda.stream(streams[s]):
            gr.replay()
    torch.cuda.synchronize()
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, gr in enumerate(graphs):
            with torch.cuda.stream(streams[s]):
                gr.replay()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) / K * 1e6)
    out["graph"] = sorted(walls)[2]
    print(f"S={S}: " + ", ".join(f"{k} {v:6.2f} us/step ({N / v * 1e6:.3e} env-steps/s)" for k, v in out.items()),
          flush=True)


if __name__ == "__main__":
    for S in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
        run(S)
