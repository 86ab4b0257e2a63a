"""Experiment: per-launch kernel time (events) vs rollout (K steps / launch) per-step time."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, bench
for variant in ("fast",):
    env = bench.make_env(65536, 0, True, torch.device("cuda"), variant=variant)
    acts = torch.rand(400, 65536, device="cuda") * 2 - 1
    for t in range(10):
        env.step(acts[t])
    ms = env.time_steps(acts[:100])
    print(variant, "per-launch kernel us: mean %.2f min %.2f max %.2f" % (ms.mean() * 1e3, ms.min() * 1e3, ms.max() * 1e3))
    for K in (1, 10, 100):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for r in range(max(1, 100 // K)):
            env.rollout(acts[:K])
        torch.cuda.synchronize(); dt = time.perf_counter() - t0
        n = max(1, 100 // K) * K
        print(variant, "rollout K=%d: %.2f us/step -> %.3e env-steps/s" % (K, dt / n * 1e6, 65536 * n / dt))
