"""Per-launch durations and gaps inside one K-launch graph replay of the bench workload (torch.profiler):
is the short timed region's extra cost in its first launch, in the gaps, or outside the kernels?
Run: python tools/exp_k20.py [K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
env = bench.make_env(65536, 0, True, dev)
acts = torch.rand(K + 5, 65536, device=dev) * 2 - 1
for t in range(5):
    env.step(acts[t])
g = bench.graph_of(lambda: [env.step(acts[5 + t]) for t in range(K)], dev)
g.replay()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU]) as prof:
    for _ in range(3):
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
evs = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA and "k_env_step" in e.name]
evs.sort(key=lambda e: e.time_range.start)
for r in range(3):
    chunk = evs[r * K:(r + 1) * K]
    d = [e.time_range.elapsed_us() for e in chunk]
    gaps = [chunk[i + 1].time_range.start - chunk[i].time_range.end for i in range(len(chunk) - 1)]
    span = chunk[-1].time_range.end - chunk[0].time_range.start
    print(f"replay {r}: span {span:.1f} us over {K} launches ({span / K:.2f}/launch); first {d[0]:.2f} "
          f"second {d[1]:.2f} median {sorted(d)[K // 2]:.2f} last {d[-1]:.2f}; gaps median "
          f"{sorted(gaps)[len(gaps) // 2]:.2f} max {max(gaps):.2f}")
cpu = [e for e in prof.events() if "Graph" in e.name or "graph" in e.name]
for e in cpu[:6]:
    print("host", e.name, round(e.time_range.elapsed_us(), 1))
