"""Where does the fixed cost of a short timed region go (GPU)?  bench.py's protocol at --steps 20 spends
~1.4 us/step more than at --steps 400.  Replays a K-launch graph of the bench env under variants of the
timing bracket and prints the median wall time per region (20 repeats):
  plain    sync; t0; replay; sync; t1
  events   sync; t0; ev0; replay; ev1; sync; t1                 (bench.py's bracket at N = 1 ...)
  events2  ... + a second synchronize before t1                 (... as it was: sync, [barrier], sync)
  empty    sync; t0; sync; t1
  evpre    sync; ev0; t0; replay; ev1; sync; t1                 (the start event queued before the clock)
  seq      sync; t0; env.step_seq (one C call: K per-step launches, no graph); sync; t1
  seqev    sync; ev0; t0; env.step_seq; ev1; sync; t1
  eager    sync; t0; K x env.step (one ctypes call and one kernel launch each, no graph); sync; t1
python tools/exp_fixed.py [K ...]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 65536
    Ks = [int(a) for a in sys.argv[1:]] or [1, 20, 100]
    env = bench.make_env(n, 0, True, dev)
    acts = torch.rand(max(Ks) + 5, n, device=dev) * 2 - 1
    for t in range(5):
        env.step(acts[t])
    torch.cuda.synchronize()
    for K in Ks:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for t in range(K):
                env.step(acts[5 + t])
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        res = {}
        for mode in ("plain", "events", "events2", "evpre", "empty", "eager", "seq", "seqev"):
            ws = []
            for _ in range(20):
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                if mode in ("evpre", "seqev"):
                    ev0.record()
                t0 = time.perf_counter()
                if mode in ("seq", "seqev"):
                    env.step_seq(acts[5:5 + K])
                    if mode == "seqev":
                        ev1.record()
                elif mode == "evpre":
                    g.replay()
                    ev1.record()
                elif mode == "eager":
                    for t in range(K):
                        env.step(acts[5 + t])
                elif mode != "empty":
                    if mode != "plain":
                        ev0.record()
                    g.replay()
                    if mode != "plain":
                        ev1.record()
                torch.cuda.synchronize()
                if mode == "events2":
                    torch.cuda.synchronize()
                ws.append((time.perf_counter() - t0) * 1e6)
            res[mode] = statistics.median(ws)
        print(f"K={K:4d} " + " ".join(f"{m} {v:8.1f} us ({v / K:6.2f}/step)" for m, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
