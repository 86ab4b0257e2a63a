"""Phase times of the two-wave env-step kernel (csrc/b747_split.h) from a -DB747_STAMPS build (GPU):
per role (flight waves 0-3, control waves 4-7 of each 512-thread workgroup), the median s_memtime cycles
between consecutive stamps: 1 table barrier, 2 the barrier after the flight's stage-0 pre / the control prologue, 3-5
iteration barriers j = 1..3, 6 after iteration 4, 8 before the reset barrier, 9 after it; realtime slots 0 / 10 give the launch span.
Run: python tools/exp_stamps_split.py --lib tools/st/stamps.so"""
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
    ap.add_argument("--flight", action="store_true",
                    help="a -DB747_STAMPS_FLIGHT build: phases inside the flight wave's stage 2")
    ap.add_argument("--chain", action="store_true",
                    help="a -DB747_STAMPS_CHAIN build: readiness probes along the flight stage-2 dependency chain")
    a = ap.parse_args()
    import b747_rl_ctrl_amd._lib as L
    L.LIB_PATH = os.path.abspath(a.lib)
    import torch
    import bench
    env = bench.make_env(a.n, 0, True, torch.device("cuda"))
    acts = torch.rand(30, a.n, device="cuda") * 2 - 1
    for t in range(30):
        env.step(acts[t])
    torch.cuda.synchronize()
    nw = 2 * a.n // 64
    buf = (ctypes.c_ulonglong * (nw * 16))()
    assert L.lib().b747_debug_stamps(buf, nw * 16) == 0
    s = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
    role = (np.arange(nw) % 8) >= 4                     # waves 4-7 of each workgroup: control
    if a.chain:
        x = s[role == False]  # noqa: E712
        names = ["start (post+combine done)", "|q|^-1 (rsqrt)", "cos theta", "V^2", "1/V (rsqrt)", "sin alpha",
                 "alpha (unit_atan2)", "M", "CYa record", "CYa", "CXa record", "forces (a_y)"]
        prev = 3
        for slot, nm in zip(range(4, 16), names):
            print(f"  {nm:>26s}: +{int(np.median(x[:, slot] - x[:, prev])):5d}  (at {int(np.median(x[:, slot] - x[:, 3])):5d})")
            prev = slot
        return
    # (from slot, to slot, name): stamps 1 table barrier, 2 barrier after the flight's stage-0 pre / the control
    # prologue, 3-5 iteration barriers j = 1..3, 6 end of iteration 4, 11 X stored, 12 after the stash barrier,
    # 8 before the reset barrier (flight: read-out done), 9 after it
    spans = {False: [(1, 2, "stage0 pre"), (2, 3, "iter1"), (3, 4, "iter2"), (4, 5, "iter3"), (5, 6, "iter4"),
                     (6, 11, "combine+X0..8"), (11, 12, "barrier T"), (12, 8, "read-out"), (8, 9, "barrier E")],
             True: [(1, 2, "prologue"), (2, 3, "iter1"), (3, 4, "iter2"), (4, 5, "iter3"), (5, 6, "iter4"),
                    (6, 11, "combine+X9..17"), (11, 12, "barrier T"), (12, 8, "-"), (8, 9, "barrier E")]}
    for r, nm in ((False, "flight"), (True, "control")):
        x = s[role == r]
        parts = [f"{lab} {int(np.median(x[:, b] - x[:, a]))}" for a, b, lab in spans[r]]
        print(f"{nm:>8s}: " + ", ".join(parts) + f" | table barrier -> barrier E {int(np.median(x[:, 9] - x[:, 1]))}")
        busy = [int(np.median(x[:, 12 + j] - x[:, 1 + j])) for j in (1, 2, 3)]
        print(f"{'':>8s}  busy in iterations 1-3 (to its barrier): {busy}")
    if a.flight:
        x = s[role == False]  # noqa: E712
        parts = [(3, 7, "post(1)+combine"), (7, 13, "attitude/air data/alpha"), (13, 14, "lookups fetched"),
                 (14, 15, "bilin, CXa, ISA, forces"), (15, 4, "to barrier 2")]
        print("flight stage 2: " + ", ".join(f"{lab} {int(np.median(x[:, b] - x[:, a]))}" for a, b, lab in parts))
        return
    r0, r1 = s[:, 0], s[:, 10]
    t0 = r0.min()
    print(f"realtime (us): starts spread {(r0.max() - t0) / 100:.2f}, ends {(r1.min() - t0) / 100:.2f} .. {(r1.max() - t0) / 100:.2f}")


if __name__ == "__main__":
    main()
