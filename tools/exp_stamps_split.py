"""Phase times of the two-wave env-step kernel (csrc/b747_split.h, round 5: the control wave leads) from a
-DB747_STAMPS build (GPU): per role (flight waves 0-3, control waves 4-7 of each 512-thread workgroup), the median
s_memtime cycle at which each stamp is reached, relative to the table barrier (slot 1).  Slots: 2-5 end of the wave's
stage 0-3, 6 control read-out done / flight stores issued; flight 8-10 ahead values of stage 1-3 arrived, 11-14 delta
of stage 0-3 arrived; control 8-10 the flight combine 1-3 arrived, 11-13 ahead values of stage 1-3 posted; realtime
slots 0 / 7 give the launch span.
Run: python tools/exp_stamps_split.py --lib tools/st/stamps.so"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {False: {2: "stage0 end", 8: "ahead1 in", 3: "stage1 end", 9: "ahead2 in", 4: "stage2 end", 10: "ahead3 in",
                 5: "stage3 end", 6: "stores issued", 11: "delta0 in", 12: "delta1 in", 13: "delta2 in", 14: "delta3 in"},
         True: {8: "ahead1 posted", 2: "ctl stage0 end", 9: "ahead2 posted", 3: "ctl stage1 end", 10: "ahead3 posted",
                4: "ctl stage2 end", 5: "ctl stage3 end", 11: "read-out math", 6: "read-out stores",
                },
         2: {8: "ahead1 posted", 9: "ahead2 posted", 10: "ahead3 posted"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--roles", type=int, default=2, help="3: the ahead-wave build (waves 4-7 ahead, 8-11 control)")
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
    nw = a.roles * a.n // 64
    buf = (ctypes.c_ulonglong * (nw * 16))()
    assert L.lib().b747_debug_stamps(buf, nw * 16) == 0
    s = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
    rw = (np.arange(nw) % (4 * a.roles)) // 4           # 0 flight, then (3 roles) 1 ahead, 2 control, or 1 control
    role = np.where(rw == 0, 0, np.where(rw == a.roles - 1, 1, 2))
    roles = [(0, "flight"), (1, "control")] + ([(2, "ahead")] if a.roles == 3 else [])
    for r, nm in roles:
        x = s[role == r]
        names = NAMES[r if r == 2 else bool(r)]
        if r == 1 and a.roles == 3:
            names = {k: v for k, v in names.items() if k not in (8, 9, 10)}
        at = sorted(((int(np.median(x[:, k] - x[:, 1])), lab) for k, lab in names.items()))
        print(f"{nm:>8s} (cycles after the table barrier): " + ", ".join(f"{lab} {c}" for c, lab in at))
    for r, nm in roles:
        x = s[role == r]
        print(f"{nm:>8s}: start -> table barrier (realtime) median {np.median(x[:, 15] - x[:, 0]) / 100:.2f} us, "
              f"last {(x[:, 15].max() - s[:, 0].min()) / 100:.2f} us after the first start")
    r0, r1 = s[:, 0], s[:, 7]
    t0 = r0.min()
    print(f"realtime (us): starts spread {(r0.max() - t0) / 100:.2f}, ends {(r1.min() - t0) / 100:.2f} .. "
          f"{(r1.max() - t0) / 100:.2f}; median wave life {np.median(r1 - r0) / 100:.2f}")


if __name__ == "__main__":
    main()
