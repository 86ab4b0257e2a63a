"""Phase times of the per-step kernel (csrc/b747_split.h k_env_step_split, round 5: flight, ahead and control waves)
from a -DB747_STAMPS build (GPU): per role (flight waves 0-3, ahead 4-7, control 8-11 of each 768-thread workgroup), the median
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
                13: "deltas posted", 14: "delta inputs in"},
         2: {8: "ahead1 posted", 9: "ahead2 posted", 10: "ahead3 posted"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--roles", type=int, default=3, help="2: a two-role build (waves 4-7 control; round 4)")
    ap.add_argument("--diag", action="store_true", help="the prologue-stamp build of DESIGN.md 4 (load phase)")
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
    # per workgroup: the first wave's start, the table barrier, the last wave's end (realtime, us after the launch's
    # first start), and how the end spread relates to them
    wpg = 4 * a.roles
    g = s[: (nw // wpg) * wpg].reshape(-1, wpg, 16)
    t00 = s[:, 0].min()
    gs, gb, ge = ((g[:, :, 0].min(axis=1) - t00) / 100, (g[:, :, 15].max(axis=1) - t00) / 100,
                  (g[:, :, 7].max(axis=1) - t00) / 100)
    q = (0, 10, 50, 90, 100)
    for lab, v in (("workgroup start", gs), ("table barrier", gb), ("workgroup end", ge), ("end - barrier", ge - gb)):
        print(f"{lab:>16s} (us) percentiles {q}: " + " ".join(f"{x:.2f}" for x in np.percentile(v, q)))
    print(f"corr(end, start) {np.corrcoef(ge, gs)[0, 1]:.2f}  corr(end, barrier) {np.corrcoef(ge, gb)[0, 1]:.2f}  "
          f"corr(end - barrier, barrier) {np.corrcoef(ge - gb, gb)[0, 1]:.2f}")
    if a.roles == 3:                                    # control slot 12: the argument segment arrived (realtime)
        x = g[:, (role[:wpg] == 1)]
        ka = (x[:, :, 12] - x[:, :, 0]) / 100
        print(f"control: start -> argument segment waited, at the table barrier (realtime) median {np.median(ka):.2f} us, p90 {np.percentile(ka, 90):.2f}")
    for r, nm in roles:                                 # which role ends the workgroup
        x = g[:, (rw[:wpg] == 0) if r == 0 else (role[:wpg] == r)]
        print(f"{nm:>8s}: end - table barrier (realtime) median {np.median((x[:, :, 7] - g[:, :, 15].max(axis=1)[:, None]) / 100):.2f} us; "
              f"last wave of the role ends the workgroup in {np.mean(x[:, :, 7].max(axis=1) >= g[:, :, 7].max(axis=1)) * 100:.0f} % of them")
    xcd = np.arange(len(ge)) % 8
    print("median end per XCD (blockIdx % 8): " + " ".join(f"{np.median(ge[xcd == x]):.2f}" for x in range(8)))
    print("median barrier per XCD:            " + " ".join(f"{np.median(gb[xcd == x]):.2f}" for x in range(8)))
    print("median start per XCD:              " + " ".join(f"{np.median(gs[xcd == x]):.2f}" for x in range(8)))
    print("median start->barrier per XCD:     " + " ".join(f"{np.median((gb - gs)[xcd == x]):.2f}" for x in range(8)))
    print("median barrier->end per XCD:       " + " ".join(f"{np.median((ge - gb)[xcd == x]):.2f}" for x in range(8)))
    # inside a workgroup: when its waves start (realtime, us after the workgroup's first wave), by wave slot
    ws = (g[:, :, 0] - g[:, :, 0].min(axis=1)[:, None]) / 100
    print("wave start within its workgroup, median by wave (us): " + " ".join(f"{v:.2f}" for v in np.median(ws, axis=0)))
    print(f"last wave start within its workgroup (us) percentiles {q}: "
          + " ".join(f"{x:.2f}" for x in np.percentile(ws.max(axis=1), q)))
    if a.diag:   # the prologue-stamp build: flight 12 tables arrived, ahead 11 / control 12 argument segment, control 13 loads issued
        fl, ah, ct = g[:, (rw[:wpg] == 0)], g[:, (role[:wpg] == 2)], g[:, (role[:wpg] == 1)]
        print(f"(diagnostic build) flight: start -> tables arrived median {np.median((fl[:, :, 12] - fl[:, :, 0]) / 100):.2f} us; "
              f"ahead: start -> argument segment median {np.median((ah[:, :, 11] - ah[:, :, 0]) / 100):.2f} us")
        print(f"(diagnostic build) control: start -> loads issued median {np.median((ct[:, :, 13] - ct[:, :, 0]) / 100):.2f} us, "
              f"-> argument segment {np.median((ct[:, :, 12] - ct[:, :, 0]) / 100):.2f} us")
    pre = (g[:, :, 15] - g[:, :, 0]) / 100           # each wave: its start to the barrier it passed
    print("wave start -> barrier, median by wave (us): " + " ".join(f"{v:.2f}" for v in np.median(pre, axis=0)))
    r0, r1 = s[:, 0], s[:, 7]
    t0 = r0.min()
    print(f"realtime (us): starts spread {(r0.max() - t0) / 100:.2f}, ends {(r1.min() - t0) / 100:.2f} .. "
          f"{(r1.max() - t0) / 100:.2f}; median wave life {np.median(r1 - r0) / 100:.2f}")


if __name__ == "__main__":
    main()
