"""Debug helper: per-env divergence of GPU vs oracle trajectories."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import oracle_lib as O
from test_gpu_model import _gpu_model, _init_both

b = O.random_batch(512, seed=5)
m = _gpu_model(b); _init_both(m, b)
for s in range(20):
    m.step(100); O.oracle_step(b, 100)
    torch.cuda.synchronize()
    g = m.sig.cpu().numpy(); r = b.sig
    scale = np.maximum(np.abs(r).max(axis=1, keepdims=True), 1e-300)
    per_env = np.nanmax(np.abs(g - r) / scale, axis=0)
    gx = m.X.cpu().numpy(); per_env_x = np.nanmax(np.abs(gx - b.X) / np.maximum(np.abs(b.X).max(axis=1, keepdims=True), 1e-300), axis=0)
    worst = np.argsort(-per_env)[:4]
    print((s + 1) * 100, 'sig max %.2e  p99 %.2e  median %.2e | X max %.2e  memdiff %d' % (
        per_env.max(), np.quantile(per_env, 0.99), np.median(per_env), per_env_x.max(), (m.mem.cpu().numpy() != b.mem).sum()),
        'worst envs', [(int(i), int(b.flags[i]), '%.1e' % per_env[i]) for i in worst], flush=True)
    if s == 19:
        i = worst[0]; j = int(np.nanargmax(np.abs(g[:, i] - r[:, i]) / scale[:, 0]))
        print('worst env', i, 'field', O.SIG_NAMES[j], g[j, i], r[j, i], 'theta', r[9, i], 'Vx', r[7, i], 'y', r[6, i])
