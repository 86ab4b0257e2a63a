"""Fixed cost of bench.py's timed region (GPU): wall time of one replay of a K-launch env-step graph,
bracketed by torch.cuda.synchronize() as in bench.py, for K = 1, 5, 20, 100; the intercept of wall(K)
is the graph-launch + synchronisation latency that a K = 20 region spreads over its 20 launches.
--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the first HIP call (busy-wait synchronisation
instead of the runtime's default wait)."""
import argparse
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--yield", dest="yld", action="store_true")
    ap.add_argument("--ramp-ms", type=float, default=0.0, help="untimed back-to-back replays first (clock ramp)")
    a = ap.parse_args()
    import torch
    if a.spin or a.yld:
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1 if a.spin else 2))   # hipDeviceScheduleSpin / Yield
        print("hipSetDeviceFlags rc", rc)
    import bench
    n = 65536
    env = bench.make_env(n, 0, True, torch.device("cuda"))
    acts = torch.rand(120, n, device="cuda") * 2 - 1
    for t in range(10):
        env.step(acts[t])
    torch.cuda.synchronize()
    res = {}
    graphs = {}
    for K in (1, 5, 20, 100):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=s):
            for t in range(K):
                env.step(acts[t])
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        graphs[K] = g
    for K, g in graphs.items():
        if a.ramp_ms > 0:                    # keep the GPU busy for ramp_ms before this K's samples
            t0 = time.perf_counter()
            while (time.perf_counter() - t0) * 1e3 < a.ramp_ms:
                graphs[100].replay()
                torch.cuda.synchronize()
        walls = []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        res[K] = statistics.median(walls)
    slope = (res[100] - res[20]) / 80
    print(f"spin={a.spin} yield={a.yld} ramp={a.ramp_ms}ms  wall us: " + "  ".join(f"K={k} {v:.1f}" for k, v in res.items())
          + f"  | per launch {slope:.2f} us, fixed {res[20] - 20 * slope:.1f} us, K=20 rate {n * 20 / res[20] * 1e6:.3e}/s",
          flush=True)


if __name__ == "__main__":
    main()
