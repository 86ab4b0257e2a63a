"""k_policy_act against the torch ActorCritic, error per wave slot of the 256-thread workgroup (GPU).

VERDICT r2 #5: the round-2 packed layer-1 experiment (two hidden units per v_pk_fma_f32, packed head sums)
gave a value head off by up to 6e-4 on one wave of four.  This rebuilds that experiment
(-DB747_L1_VALU=1 -DB747_L1_PACKED=1, csrc/b747_policy.h) and reports, per obs_dim and head, the largest
|kernel - torch| for envs in wave slot 0..3 of their workgroup (env // 64 % 4), for each --lib given.
Run: python tools/exp_l1_packed.py --lib tools/ab2/v_base.so --lib tools/ab2/v_pk.so"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(lib, ns):
    import numpy as np
    import torch
    import b747_rl_ctrl_amd._lib as Lm
    Lm.LIB_PATH = os.path.abspath(lib)
    from b747_rl_ctrl_amd.ppo import ActorCritic
    L = Lm.lib()
    torch.manual_seed(0)
    for od in (3, 5, 7, 8, 10):
        pol = ActorCritic(od).cuda()
        with torch.no_grad():
            for prm in pol.parameters():
                prm.add_(0.05 * torch.randn_like(prm))
        fp = pol.flat_params()
        flat = torch.zeros(L.b747_policy_num_params(od), device="cuda")
        flat[:fp.numel()].copy_(fp)
        Lm.check(L.b747_policy_pack(flat.data_ptr(), od, None), "pack")
        for n in ns:
            obs = torch.randn(n, od, device="cuda")
            noise = torch.randn(n, device="cuda")
            out = {k: torch.empty(n, device="cuda") for k in ("act", "logp", "val", "env")}
            Lm.check(L.b747_policy_act(flat.data_ptr(), od, n, obs.data_ptr(), noise.data_ptr(), 0, None, 0, 0,
                                       None, out["act"].data_ptr(), out["logp"].data_ptr(),
                                       out["val"].data_ptr(), out["env"].data_ptr(), -1.0, 1.0, None), "policy")
            torch.cuda.synchronize()
            with torch.no_grad():
                mean, value = pol(obs)
                act = mean.squeeze(-1) + pol.log_std.exp() * noise
            ea = (out["act"] - act).abs().cpu().numpy()
            ev = (out["val"] - value).abs().cpu().numpy()
            slot = (np.arange(n) // 64) % 4
            lane_hi = (np.arange(n) % 64) >= 32
            row = []
            for s in range(4):
                m = slot == s
                row.append(f"slot{s} pi {ea[m].max():.1e} vf {ev[m].max():.1e}")
            worst_v = int(np.argmax(ev))
            print(f"od {od:2d} n {n:6d}: " + " | ".join(row) +
                  f" | worst vf env {worst_v} (wave {worst_v // 64}, lane {worst_v % 64}, upper half {bool(lane_hi[worst_v])}), "
                  f"envs > 2e-5: pi {int((ea > 2e-5).sum())} vf {int((ev > 2e-5).sum())}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", required=True)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--n", type=int, action="append")
    a = ap.parse_args()
    ns = a.n or [3000, 65536]
    if a.child:
        one(a.lib[0], ns)
        return
    for lib in a.lib:   # one process per library (the ctypes handle is per process)
        print(f"== {os.path.basename(lib)}", flush=True)
        cmd = [sys.executable, "-u", __file__, "--child", "--lib", lib] + sum((["--n", str(n)] for n in ns), [])
        r = subprocess.run(cmd, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
