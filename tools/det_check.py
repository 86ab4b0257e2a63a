"""Diagnostic (GPU): config-specialised vs generic env kernel on identical inputs, several action seeds;
reports every output that differs (step, env, values)."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,  # noqa: E402
                              ResetRefMode, RewardType, _lib)
mk = lambda: BatchControllerEnv(4096, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                                CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                                disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=1.0, sample_time=None, seed=11)


def run(on, acts):
    _lib.lib().b747_set_specialization(on)
    e = mk()
    obs, xs = [], []
    for t in range(acts.shape[0]):
        o, r, d, _ = e.step(acts[t])
        obs.append(torch.cat([o, r[:, None]], 1).clone())
        xs.append(e.X.clone())
    torch.cuda.synchronize()
    return torch.stack(obs), torch.stack(xs)


for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    g = torch.Generator(device="cuda").manual_seed(seed)
    acts = torch.rand(200, 4096, device="cuda", generator=g) * 2 - 1
    (o1, x1), (o0, x0) = run(1, acts), run(0, acts)
    bo, bx = (o1 != o0).nonzero(), (x1 != x0).nonzero()
    print(f"seed {seed}: obs/reward diffs {bo.shape[0]}, X diffs {bx.shape[0]}")
    for s, i, j in bo[:4].tolist():
        print(f"   step {s} env {i} col {j}: spec {o1[s, i, j].item()!r} generic {o0[s, i, j].item()!r}; "
              f"row spec {o1[s, i].tolist()} generic {o0[s, i].tolist()}")
    for s, j, i in bx[:4].tolist():
        print(f"   X step {s} comp {j} env {i}: {x1[s, j, i].item()!r} vs {x0[s, j, i].item()!r}")
_lib.lib().b747_set_specialization(1)
