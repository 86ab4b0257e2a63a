#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched B747 pitch simulation on MI355X.

Metric (BASELINE.json): env steps/sec (batched B747 pitch sim) at 1/2/4/8 MI355X vs CPU ctypes
baseline.  Workload (BASELINE.json configs[2], per GPU; configs[3] = the same x 8 GPUs):
65,536 envs per GPU, randomized trim/initial-condition sweep (core/controller.py:148-191
distributions: h0~U(1000,11000), Vx~U(100,265), Vy~U(-20,20), wz0~U(-1e-3,1e-3),
vartheta_ref=+-U(1,10) deg, aero_err~N([-.1,.1,-.1,-.1,.1],0.5)), fixed-step RK4 (h = 0.01 s).
One bench "step" = one env step of every env = one model_simple_step (ode4 step of 0.01 s,
the Controller default sample_time = dt, core/controller.py:110) = one kernel launch.

Launch:  python bench.py [--gpus N --steps K --warmup W]        (N=1)
         python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...  (N>1)
Each rank simulates its own 65,536 envs (weak scaling, env ids offset by rank); there is no
collective on the data path -- only a barrier and a max-reduce of the timings.
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ENVS_PER_GPU = 65536
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def bytes_per_env_step(x_f64: bool, with_sig: bool) -> int:
    """Algorithmic HBM bytes of one b747_model_step(n_steps=1) per env."""
    xb = 8 if x_f64 else 4
    state = 18 * xb + 9 * 8 + 4 + 1          # X, disc, k, mem
    params = 8 + 8 + 8 + 1 + 5 * 4           # deltaz, vartheta, h_zh, flags, aero_err
    sig = 31 * 8 if with_sig else 0
    return state + params + state + sig      # read state+params, write state (+ read-out)


def make_workload(n, seed, x_f64, device):
    from b747_rl_ctrl_amd import BatchModel, F_PID_SS, F_RP
    g = torch.Generator(device="cpu").manual_seed(seed)
    u = lambda lo, hi: (lo + (hi - lo) * torch.rand(n, generator=g, dtype=torch.float64))
    m = BatchModel(n, device=device, x_f64=x_f64, use_PID_SS=True, use_PID_CS=False)
    s0 = torch.stack([torch.zeros(n, dtype=torch.float64), u(1000, 11000), u(100, 265), u(-20, 20),
                      torch.zeros(n, dtype=torch.float64), u(-1e-3, 1e-3)], 1)
    m.state0 = s0.to(device)
    sign = torch.where(torch.rand(n, generator=g) < 0.5, -1.0, 1.0).to(torch.float64)
    ref = sign * u(np.pi / 180, 10 * np.pi / 180)
    mean = torch.tensor([-0.1, 0.1, -0.1, -0.1, 0.1], dtype=torch.float32)
    ae = mean + 0.5 * torch.randn(n, 5, generator=g, dtype=torch.float32)
    m.aero_err = ae.to(device)
    m.initialize()
    m.vartheta_zh = ref.to(device)     # AUTO ctrl type: SS PID tracks the pitch command
    m.flags.fill_(F_RP | F_PID_SS)
    return m


def reduce_max(value, dist, device):
    """MAX of a per-rank wall time over all ranks (the slowest rank defines the step time)."""
    if dist is None or not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(seconds_target=15.0):
    """Oracle (fp64 restatement, OpenMP over envs) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    threads = min(16, os.cpu_count() or 1)
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    b = O.random_batch(4096, seed=0, modes=O.F_RP | O.F_PID_SS)
    O.oracle_initialize(b)
    O.oracle_step(b, 5)                                 # warm-up
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds_target and steps < 2000:
        O.oracle_step(b, 25)
        steps += 25
    dt = time.perf_counter() - t0
    return {"value": round(b.n * steps / dt, 1), "unit": "env-steps/s", "cores": threads,
            "kind": "port", "sample": f"4096 envs x {steps} steps of the config-3 sweep, fp64 oracle "
                                      f"(oracle/b747_oracle.c), OpenMP over envs"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--x32", action="store_true", help="store X in fp32 (compute stays fp64)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import b747_rl_ctrl_amd  # noqa: F401  (fails loudly if libb747.so is missing)
    x_f64 = not args.x32
    m = make_workload(args.envs, seed=1000 + rank, x_f64=x_f64, device=device)

    for _ in range(args.warmup):
        m.step(1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        m.step(1)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps          # avg per launch, on the launch stream
    wall = reduce_max(wall, dist, device)
    if not torch.isfinite(m.X).all():
        raise RuntimeError("non-finite state after the timed region")

    total_steps = args.envs * args.steps * world
    value = total_steps / wall
    bpe = bytes_per_env_step(x_f64, with_sig=False)
    achieved = bpe * args.envs / (kern_ms * 1e-3) / 1e9
    out = {
        "metric": "env steps/sec (batched B747 pitch sim)",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (randomized trim/IC sweep, config-3 distributions, seeded per rank)",
        "config": {"workload": "configs[2]: 65536 envs/GPU randomized IC sweep, fixed-dt RK4 h=0.01s, "
                               "AUTO ctrl (SS PID tracks +-U(1,10) deg pitch command), 1 env-step/launch",
                   "envs_per_gpu": args.envs, "global_envs": args.envs * world,
                   "state_storage": "f64" if x_f64 else "f32", "parallelism": f"env-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                     "kernel": "k_model_step", "bytes_per_env_step": bpe,
                     "kernel_avg_us": round(kern_ms * 1e3, 3)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline()
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
