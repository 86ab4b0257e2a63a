"""Phase shares of the env-step kernel from a diagnostic build with in-kernel stamps (GPU).

The library under test must be built with -DB747_STAMPS (tools/build_ab_flags.sh "stamps|-DB747_STAMPS");
run as: python tools/exp_stamps.py --lib tools/build/ab/stamps.so.  Reports, over the 1024 waves of
one launch on the bench workload (65,536 envs, config 3): cycles from wave start to the barrier
(table staging), to the state landing, through the env step, through issuing the stores, to the
stores completing; and the spread of wave start / end times (s_memrealtime, 100 MHz).  Read the
SHARES: the stamps' drains forbid overlaps the real kernel has."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--k", type=int, default=1, help="env steps per launch (rollout launch when > 1)")
    ap.add_argument("--stages", action="store_true", help="library built with -DB747_STAMPS_STAGES (use --k 2)")
    ap.add_argument("--step", action="store_true", help="library built with -DB747_STAMPS_STEP")
    a = ap.parse_args()
    import b747_rl_ctrl_amd._lib as L
    L.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import bench
    env = bench.make_env(a.n, 0, True, torch.device("cuda"))
    acts = torch.rand(20, a.n, device="cuda") * 2 - 1
    for t in range(20):
        env.step(acts[t])
    if a.k > 1:
        env.rollout(torch.rand(a.k, a.n, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    nw = a.n // 64
    buf = (ctypes.c_ulonglong * (nw * 16))()
    rc = L.lib().b747_debug_stamps(buf, nw * 16)
    assert rc == 0, rc
    s16 = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
    s = s16[:, :8]
    names = ["table+barrier", "state landed", "env step", "stores issued", "stores done"]
    d = np.diff(s[:, 1:7], axis=1)
    tot = s[:, 6] - s[:, 1]
    print(f"waves {nw}; wave lifetime (s_memtime cycles) median {np.median(tot):.0f} p10 {np.percentile(tot, 10):.0f} "
          f"p90 {np.percentile(tot, 90):.0f}")
    for j, nm in enumerate(names):
        print(f"  {nm:>14s}: median {np.median(d[:, j]):7.0f}  p10 {np.percentile(d[:, j], 10):7.0f}  "
              f"p90 {np.percentile(d[:, j], 90):7.0f}  share {np.median(d[:, j]) / np.median(tot):.3f}")
    if a.stages:   # slots 8-15: RK4 stage ends of two consecutive major steps (by k parity)
        st = s16[:, 8:16].reshape(nw, 2, 4)
        first = np.where(st[:, 0, 0] < st[:, 1, 0], 0, 1)
        a0, a1 = st[np.arange(nw), first], st[np.arange(nw), 1 - first]
        seq = np.concatenate([s[:, 3:4], a0, a1], axis=1)
        print("  per RK4 stage of steps 0 and 1 (median cycles):", [int(np.median(x)) for x in np.diff(seq, axis=1).T])
    elif a.step:   # slots 8-15: {controller, dynamics, read-out, end} of env steps 0 and 1
        seq = np.concatenate([s[:, 3:4], s16[:, 8:8 + 4 * min(a.k, 2)]], axis=1)
        names = ["controller", "dynamics", "read-out", "end/reset"]
        d = [int(np.median(x)) for x in np.diff(seq, axis=1).T]
        print("  env-step phases (median cycles):", ", ".join(f"s{j // 4} {names[j % 4]} {v}" for j, v in enumerate(d)))
    elif a.k > 1:
        ends = np.concatenate([s[:, 3:4], s16[:, 8:8 + min(a.k, 8)]], axis=1)
        print("  per env step (median cycles):", [int(np.median(x)) for x in np.diff(ends, axis=1).T])
    r0, r1 = s[:, 0], s[:, 7]
    t0 = r0.min()
    print(f"realtime (us): wave starts spread {(r0.max() - t0) / 100:.2f} (p50 {(np.median(r0) - t0) / 100:.2f}), "
          f"ends {(r1.min() - t0) / 100:.2f} .. {(r1.max() - t0) / 100:.2f}")


if __name__ == "__main__":
    main()
