"""Probe: per-call latency of b747_rl_ctrl_amd/model_simple.so (the DLL ABI over a 1-env GPU batch)
beside the CPU oracle's DLL-ABI library, both driven through ctypes like core/model.py."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_model_simple_shim import ORACLE_SHIM, SHIM, Model  # noqa: E402

N = 3000
for name, path in (("gpu shim", SHIM), ("cpu oracle", ORACLE_SHIM)):
    m = Model(path)
    m.d.model_simple_initialize()
    for _ in range(50):
        m.d.model_simple_step()
    t0 = time.perf_counter()
    for _ in range(N):
        m.d.model_simple_step()
    dt = (time.perf_counter() - t0) / N
    print(f"{name}: {dt * 1e6:.1f} us per model_simple_step -> {1 / dt:.3e} steps/s", flush=True)
