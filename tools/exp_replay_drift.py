"""Diagnostic (not a test): how the bench kernels' obs / reward deviate from the env oracle over free-running
windows of W env steps at tk = 20 s (the shadow windows of tests/test_gpu_episode_replay.py).
Prints, per window, the largest absolute deviation of each obs component and of the reward, the batch's
largest |value| of that component at the same step (its scale), and the env / step where the worst one sits."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle_lib as O  # noqa: E402
from test_gpu_episode_replay import _load_oracle_state  # noqa: E402
from test_gpu_fullsize import _bench_env, _device_draws  # noqa: E402


def main(kernel="rollout", W=100, N=65536, steps=2100):
    from b747_rl_ctrl_amd import _lib
    _lib.lib().b747_set_specialization(1)
    env = _bench_env(N, 77, 20.0)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=20.0)
    full.reset(*_device_draws(env))
    g = torch.Generator(device="cuda").manual_seed(6)
    obs_seq = torch.empty(W, N, 3, device="cuda")
    rew_seq = torch.empty(W, N, device="cuda")
    done_seq = torch.empty(W, N, dtype=torch.uint8, device="cuda")
    for w in range(steps // W):
        _load_oracle_state(env, full)
        acts = torch.rand(W, N, device="cuda", generator=g) * 2 - 1
        if kernel == "rollout":
            env.rollout(acts, obs_seq, rew_seq, done_seq)
        else:
            for t in range(W):
                o, r, d, _ = env.step(acts[t])
                obs_seq[t].copy_(o); rew_seq[t].copy_(r); done_seq[t].copy_(d)
        a_h = acts.cpu().numpy()
        worst = np.zeros(4); scale = np.zeros(4); where = [None] * 4; rel = np.zeros(4)
        for t in range(W):
            o_ref, r_ref, d_ref = full.step(a_h[t])
            d = done_seq[t].cpu().numpy().astype(bool)
            o = obs_seq[t].cpu().numpy()
            if d.any():
                o = np.where(d[:, None], env.terminal_obs.cpu().numpy(), o)
            r = rew_seq[t].cpu().numpy()
            for c in range(4):
                got, ref = (o[:, c], o_ref[:, c]) if c < 3 else (r, r_ref.astype(np.float32))
                err = np.abs(got.astype(np.float64) - ref)
                j = int(np.argmax(err))
                if err[j] > worst[c]:
                    worst[c], where[c] = err[j], (t, j, float(got[j]), float(ref[j]))
                scale[c] = max(scale[c], float(np.abs(ref).max()))
                rel[c] = max(rel[c], float(np.max(err / (np.abs(ref) * 2e-6 + 1e-7))))
            if d.any():
                full.reset(*_device_draws(env), mask=d)
        print(f"window {w:2d}: " + "  ".join(f"c{c} err {worst[c]:.2e} scale {scale[c]:.2e} tolx {rel[c]:.2f} at {where[c]}"
                                            for c in range(4)), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "rollout", int(sys.argv[2]) if len(sys.argv) > 2 else 100)
