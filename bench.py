#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched B747 pitch-control environment on MI355X.

Metric (BASELINE.json): env steps/sec (batched B747 pitch sim) at 1/2/4/8 MI355X vs the CPU ctypes
baseline.  Workload = BASELINE.json configs[2] per GPU (configs[3] = the same on 8 GPUs):
  65,536 envs per GPU, ControllerEnv(PID_LIKE obs, CLASSIC reward, norm_obs, norm_act,
  MANUAL ctrl, DIRECT_CONTROL, reset_ref_mode=CONST, AERO_DISTURBANCE, tk=20 s), randomized
  trim/IC sweep on every reset (core/controller.py:148-191 distributions, Philox per global env
  id), actions U(-1,1) (x 17 deg by norm_act), auto-reset on done.
One bench "step" = ControllerEnv.step for every env with sample_time = dt (the Controller default,
core/controller.py:110): one model_simple_step (ode4, h = 0.01 s) + obs + reward + done (+ reset),
fused into ONE kernel launch (b747_env_step).  The K timed launches are captured in a HIP graph
(torch.cuda.CUDAGraph) so the host is out of the loop; every step's obs/reward/done is written
to HBM, exactly as a policy would consume it.

Launch:  python bench.py [--gpus N --steps K --warmup W]                          (N = 1)
         python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...    (N > 1)
Each rank owns 65,536 envs with global ids rank*65536 + i (weak scaling); there is no collective
on the data path, only a barrier and a MAX-reduce of the wall time.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ENVS_PER_GPU = 65536
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
PEAK_F64_TFLOPS = 78.6     # MI355X FP64 vector (spec; half the 157.3 TF FP32 vector rate)


# algorithmic bytes of one env step per env (fp32 SoA state, PID_LIKE obs, one ode4
# step per launch): 144 B read (X 72, discrete state 36, step counter + flag word 8, action 4,
# command 4, aero multipliers 20) + 133 B written (state 116, obs 12, reward 4, done 1).
ALGO_BYTES_PER_ENV_STEP = 277
ALGO_READ_BYTES_PER_ENV_STEP = 144


def env_bytes_per_step(x_f64: bool, obs_dim: int, ctrl=False, osc=False, add_mode=False, tf_reward=False,
                       ang_vel=False, single_step=True) -> float:
    """Bytes of one b747_env_step per env as STORED by this implementation: every
    field the kernel reads and writes for one env step (env_load / env_store in csrc/b747_lanes.h,
    which touch a controller slot only where the configuration uses it); the rare reset traffic
    (1 per 2000 steps) is left out.  Defaults = the bench workload (MANUAL, DIRECT, CLASSIC, CONST
    refs).  fp64 X / discrete state make this larger than the algorithmic 277 B of SURVEY 8(d).
    single_step: the one-step kernel of the FAST variant (the bench's), which skips the pitch-plane
    quaternion's constant q1 = q2 = 0 (16 B each way) and writes back only what the DLL step changed:
    one U_com history slot of four (-24 B) and the DSS pair on its 0.05 s tick only (-16 B x 4/5)."""
    xb = 8 if x_f64 else 4
    model = 18 * xb + 9 * 8 + 4 + 1                     # X, disc, k, mem
    model_w = model
    if single_step:
        model -= 2 * xb                                  # q1, q2 neither read nor written
        model_w = model - 3 * 8 - 16 * 4 / 5
    slot = 8                                             # ep_return
    slot += 8 if ang_vel else 0                          # deltaz
    slot += 8 if add_mode else 0                         # upid
    slot += 8 if tf_reward else 0                        # tp
    read = model + slot + 1 + 1 + 5 * 8 + 4              # + flags, ref_kind, aero_err (f64, ABI v7), action
    read += (7 if osc else 1) * 8 + (8 if ctrl else 0) + 8   # ref[0] (+ ref[1..6]) (+ ref[7]) (f64), h_zh
    write = model_w + slot + obs_dim * 4 + 4 + 1         # + obs, reward, done
    write += 8 if ctrl else 0                            # h_zh
    return read + write


def cpu_info():
    """Host CPU model and logical core count (the CPU baselines state both)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count()}


def committed_profile(name):
    """A JSON summary this round committed under profiles/ (tools/pmc_summary.py), or None."""
    for rnd in ("r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", rnd, name)
        if os.path.exists(path):
            return json.load(open(path)), f"profiles/{rnd}/{name}"
    return None, None


def make_env(n, rank, x_f64, device, seed=2024, variant="fast"):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=20, sample_time=None,
                              seed=seed, device=device, x_f64=x_f64, env_offset=rank * n, variant=variant)


def reduce_max(value, dist, device):
    """MAX of a per-rank wall time over all ranks (the slowest rank defines the step time)."""
    if dist is None or not dist.is_initialized():
        return value
    if dist.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(envs_per_rank, steps, world, wall_max):
    """Whole-job env-steps/s: every rank steps its own envs_per_rank envs `steps` times, and the slowest
    rank's wall time (reduce_max) is the job's time (weak scaling)."""
    return envs_per_rank * steps * world / wall_max


def cpu_baseline(seconds=12.0):
    """The reference's single-env ctypes path, restated: core/model.py-style ctypes Model over the
    DLL-ABI oracle library (oracle/build/model_simple.so) driven by Controller/ControllerEnv mirrors
    (oracle/ref_env.py), same env config as the GPU workload, 1 host core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import ref_env as R
    c = R.RefController(3, 0, 0, tk=20, sample_time=None)
    e = R.RefControllerEnv(0, 0, True, True, c)
    rng = np.random.default_rng(0)
    draws = lambda: {"state0": [0, rng.uniform(1000, 11000), rng.uniform(100, 265), rng.uniform(-20, 20), 0,
                                rng.uniform(-1e-3, 1e-3)], "kind": "const",
                     "ref": rng.uniform(math.pi / 180, 10 * math.pi / 180) * rng.choice([-1, 1]),
                     "aero_err": rng.normal([-0.1, 0.1, -0.1, -0.1, 0.1], 0.5)}
    e.reset(draws())
    acts = rng.uniform(-1, 1, 4096).astype(np.float32)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(200):
            _, _, d = e.step(acts[steps % 4096])
            steps += 1
            if d:
                e.reset(draws())
    dt = time.perf_counter() - t0
    return {"value": round(steps / dt, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"1 env x {steps} env steps (sample_time = dt, auto-reset at tk = 20 s) through the ctypes "
                      f"DLL ABI (oracle/build/model_simple.so) + Python Controller/ControllerEnv restatement"}


def host_threads():
    """The host threads this job may use: OMP_NUM_THREADS when the launcher set it (the GPU box sets it
    to the job's CPU share), else every CPU in the process's affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else len(os.sched_getaffinity(0))


def cpu_baseline_batched(seconds=10.0, n=16384):
    """All host cores of the job: the GPU line's env workload (ControllerEnv PID_LIKE / CLASSIC / MANUAL-DIRECT,
    CONST references, AERO errors, sample_time = dt, tk = 20 s, auto-reset) through the C restatement of the
    reference's env loop over the fp64 oracle (oracle/b747_oracle_env.c), OpenMP over envs; a bounded sample
    of n envs stepped until `seconds` have passed (resets draw with numpy, outside the timed steps)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    threads = host_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    import numpy as np
    import oracle_lib as O
    rng = np.random.default_rng(0)

    def draws(m):
        s0 = np.stack([np.zeros(m), rng.uniform(1000, 11000, m), rng.uniform(100, 265, m), rng.uniform(-20, 20, m),
                       np.zeros(m), rng.uniform(-1e-3, 1e-3, m)])
        ref = np.zeros((8, m), np.float32)
        ref[0] = rng.uniform(math.pi / 180, 10 * math.pi / 180, m) * rng.choice([-1.0, 1.0], m)
        aero = rng.normal([[-0.1], [0.1], [-0.1], [-0.1], [0.1]], 0.5, (5, m)).astype(np.float32)
        return s0, ref, np.zeros(m, np.uint8), aero

    E = O.EnvOracle(n, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=20.0)
    E.reset(*draws(n))
    acts = rng.uniform(-1, 1, (64, n)).astype(np.float32)
    E.step(acts[0])
    steps, busy = 0, 0.0
    while busy < seconds and steps < 4000:
        t0 = time.perf_counter()
        _, _, done = E.step(acts[steps % 64])
        busy += time.perf_counter() - t0
        steps += 1
        if done.any():
            E.reset(*draws(n), mask=done)
    value = n * steps / busy
    nproc = os.cpu_count() or threads
    return {"value": round(value, 1), "unit": "env-steps/s", "cores": threads,
            "cores_basis": "the job's host-thread share (OMP_NUM_THREADS on the GPU box), not every CPU of the host",
            "value_at_nproc_extrapolated": round(value / threads * nproc, 1) if threads else None,
            "extrapolation": f"linear per-thread scaling to all {nproc} host CPUs (not measured: the box caps a "
                             "job at its thread share)",
            "kind": "port",
            "sample": f"{n} envs x {steps} env steps of the bench workload (sample_time = dt, auto-reset at tk = 20 s) "
                      f"through the C env restatement over the fp64 oracle (oracle/b747_oracle_env.c), OpenMP"}


def isolated_launch_us(env, actions, n=60):
    """Diagnostic: mean duration of ONE b747_env_step launch measured in isolation, HIP events (no
    system fence) recorded on the launch stream around each launch (b747_env_time_steps).  The
    event pair adds ~2-4 us of its own, so the roofline uses the timed-region events instead."""
    ms = env.time_steps(actions[:n])
    return float(ms.mean()) * 1e3


def rollout_rate(env, actions, k=100, reps=3):
    """Secondary line: the same env steps with k pre-sampled actions per launch (b747_env_rollout,
    state kept in registers across the k steps, every step's obs/reward/done written)."""
    n = env.n
    k = min(k, actions.shape[0])
    obs_seq = torch.empty(k, n, env.obs_dim, device=actions.device)
    rew_seq = torch.empty(k, n, device=actions.device)
    done_seq = torch.empty(k, n, dtype=torch.uint8, device=actions.device)
    env.rollout(actions[:k], obs_seq, rew_seq, done_seq)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        env.rollout(actions[:k], obs_seq, rew_seq, done_seq)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (reps * k)
    return {"steps_per_launch": k, "value": round(n / dt, 1), "us_per_step": round(dt * 1e6, 3)}


def storage_f32_rate(n, rank, device, variant, actions, k=200):
    """Secondary line: the same per-step launches with X stored in fp32 -- the SoA layout the north star
    and SURVEY 8(d)'s 277 B assume; every stage still computes in fp64 (loaded into fp64 registers, rounded
    once per step by the store; tests/test_gpu_split.py).  The headline keeps fp64 storage."""
    env = make_env(n, rank, False, device, variant=variant)
    k = min(k, actions.shape[0])
    for t in range(5):
        env.step(actions[t])
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for t in range(k):
            env.step(actions[t])
    graph.replay()                   # untimed: the first replay uploads the graph
    torch.cuda.synchronize()
    dts = []
    for _ in range(3):               # the fastest of 3 replays: one short replay is exposed to host hiccups
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        dts.append((time.perf_counter() - t0) / k)
    dt = min(dts)
    return {"state_storage": "f32", "steps": k, "value": round(n / dt, 1), "us_per_step": round(dt * 1e6, 3),
            "bytes_per_env_step_stored": round(env_bytes_per_step(False, env.obs_dim, single_step=variant == "fast"), 1)}


def ppo_rollout_rate(n, rank, x_f64, device, variant, steps=64, reps=2):
    """BASELINE configs[4]: 65,536 envs + on-GPU PPO rollout (SB3-default MlpPolicy 64-64 tanh,
    separate pi/vf): per step policy forward + Gaussian sample + clip + fused env step, the
    whole rollout captured in one HIP graph.  End-to-end env-steps/s (b747_rl_ctrl_amd/ppo.py)."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = make_env(n, rank, x_f64, device, seed=99, variant=variant)
    ppo = PPO(env, PPOConfig(n_steps=steps), seed=0)
    ppo.last_obs.copy_(env.obs)
    ppo.collect_rollouts(steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ppo.collect_rollouts(steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (reps * steps)
    return {"workload": "configs[4]: 65536 envs + PPO rollout (policy fwd + sample + env step), HIP graph",
            "value": round(n / dt, 1), "us_per_step": round(dt * 1e6, 3), "rollout_steps": steps}


def measured_profile(x_f64, variant, envs):
    """Per-launch HBM bytes (rocprofv3 PMC FETCH_SIZE x 2 + WRITE_SIZE) and SQ counters of the env-step
    kernel from the committed profile summaries (tools/pmc_summary.py) when they were taken on this
    exact workload; otherwise Nones."""
    if not (x_f64 and variant == "fast"):
        return None, None, None, None
    d, src = committed_profile("env_step_pmc_traffic.json")
    if d is None or d.get("envs") != envs:
        return None, None, None, None
    sq, _ = committed_profile("env_step_sq_counters.json")
    return d["traffic_bytes_per_launch"], src, (sq or {}).get("per_wave"), (sq or {}).get("waves")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--x32", action="store_true", help="store X in fp32 (compute stays fp64)")
    ap.add_argument("--eager", action="store_true", help="no HIP graph: one Python call per step")
    ap.add_argument("--variant", default="fast", choices=["fast", "faithful"],
                    help="fast (default): identities for sin/cos/pow; faithful: the DLL's operation order")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) for real runs")
    ap.add_argument("--no-rollout", action="store_true",
                    help="skip the secondary lines (multi-step launches, config-5 PPO rollout, fp32 X storage)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU (torch.distributed.run); --dist-backend gloo with ranks sharing a GPU
    # only rehearses the multi-rank code path on a one-GPU box
    gpu = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    device = torch.device("cuda", gpu)
    torch.cuda.set_device(device)

    import b747_rl_ctrl_amd  # noqa: F401  (raises if libb747.so is missing -- no fallback)
    x_f64 = not args.x32
    env = make_env(args.envs, rank, x_f64, device, variant=args.variant)
    g = torch.Generator(device=device).manual_seed(77 + rank)
    actions = torch.rand(args.steps + args.warmup, args.envs, generator=g, device=device) * 2 - 1

    for t in range(args.warmup):
        env.step(actions[t])
    torch.cuda.synchronize()
    graph = None
    if not args.eager:
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for t in range(args.steps):
                env.step(actions[args.warmup + t])
        torch.cuda.synchronize()

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph is not None:            # one untimed replay: the first replay of a graph pays its upload
        graph.replay()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # the start event goes on the idle stream (where the graph replays / eager steps launch) before the
    # clock starts: its host call is instrumentation, not step work (tools/exp_fixed.py: at K = 20 it
    # put ~7 us of host latency in front of the first launch)
    ev0.record()
    t0 = time.perf_counter()
    if graph is not None:
        graph.replay()
    else:
        for t in range(args.steps):
            env.step(actions[args.warmup + t])
    ev1.record()
    torch.cuda.synchronize()
    # each rank's clock stops when its own K steps have drained; the closing barrier (an RCCL all-reduce
    # under nccl) then runs outside the region and the MAX over ranks below is the slowest rank's time
    # from the common start
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
    wall = reduce_max(wall, dist, device)
    region_event_us = ev0.elapsed_time(ev1) * 1e3 / args.steps   # per launch, on the launch stream

    if not torch.isfinite(env.obs).all() or not torch.isfinite(env.reward).all():
        raise RuntimeError("non-finite obs/reward after the timed region")
    region_us = wall / args.steps * 1e6          # per launch incl. the launch-to-launch gap
    kern_us = region_event_us                    # HIP events over the timed region / K
    iso_us = isolated_launch_us(env, actions)
    # the secondary lines are per-GPU figures: measured at N = 1 only, so that a multi-rank run stays short
    secondary = not args.no_rollout and world == 1
    roll = rollout_rate(env, actions) if secondary else None
    ppo = ppo_rollout_rate(args.envs, rank, x_f64, device, args.variant) if secondary else None
    x32 = storage_f32_rate(args.envs, rank, device, args.variant, actions) if secondary and x_f64 else None
    steps_done = int(env.k.min().item())  # sanity: envs advanced (auto-reset keeps k < 2000)
    stored = round(env_bytes_per_step(x_f64, env.obs_dim, single_step=args.variant == "fast"), 1)
    algo = ALGO_BYTES_PER_ENV_STEP
    achieved = algo * args.envs / (kern_us * 1e-6) / 1e9
    achieved_read = ALGO_READ_BYTES_PER_ENV_STEP * args.envs / (kern_us * 1e-6) / 1e9
    traffic, traffic_src, sq, sq_waves = measured_profile(x_f64, args.variant, args.envs)
    valu_frac = None
    if sq and sq.get("SQ_WAVE_CYCLES"):
        # per SIMD: a wave's VALU-active share x the waves each of the 1,024 SIMDs runs (256 CUs x 4) -- the
        # single-step kernel puts two waves (flight + control) of the same 64 envs on every SIMD
        waves_per_simd = max(1.0, float(sq_waves or 1024) / 1024.0)
        valu_frac = round(sq["SQ_ACTIVE_INST_VALU"] * waves_per_simd / sq["SQ_WAVE_CYCLES"], 3)
    out = {
        "metric": "env steps/sec (batched B747 pitch sim)",
        "value": round(aggregate_rate(args.envs, args.steps, world, wall), 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: config-3 randomized IC/reference/aero-error sweep (Philox per global env id), "
                "actions U(-1,1)",
        "config": {"workload": "configs[2]: 65536 envs/GPU ControllerEnv(PID_LIKE, CLASSIC, MANUAL, DIRECT, "
                               "reset CONST, AERO disturbance, tk=20 s), sample_time=dt: 1 fused env-step "
                               "launch = 1 ode4 step of 0.01 s + obs/reward/done/auto-reset",
                   "envs_per_gpu": args.envs, "global_envs": args.envs * world,
                   "state_storage": "f64" if x_f64 else "f32", "launch": "eager" if args.eager else "hipgraph",
                   "variant": args.variant,
                   "parallelism": f"env-shard x{world}", "min_k": steps_done},
        # frac against SURVEY 8(d)'s algorithmic bytes; the kernel's binding resource is reported beside it
        # "bound" is the roofline KIND this line is priced against (the contract's hbm | mfma: the path has no
        # matrix work); what the counters show actually binds the kernel is "bound_measured"
        "roofline": {"bound": "hbm", "bound_measured": "latency: the flight wave's dependent fp64 chain per RK4 stage "
                                                       "and the two waves' fp64 VALU issue, not HBM bandwidth",
                     "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "k_env_step_split", "bytes_per_env_step": algo,
                     "bytes_per_launch": algo * args.envs,
                     "read_bytes_per_env_step": ALGO_READ_BYTES_PER_ENV_STEP,
                     "hbm_read_frac": round(achieved_read / PEAK_HBM_GBS, 4),
                     "bytes_per_env_step_stored": stored,
                     "traffic_over_algorithmic": round(traffic / (algo * args.envs), 3) if traffic else None,
                     "kernel_avg_us": round(kern_us, 3), "launch_period_us": round(region_us, 3),
                     "isolated_launch_us": round(iso_us, 3),
                     "valu_issue_frac": valu_frac,
                     "measured_binder": "fp64 VALU issue of the two waves per SIMD (65,536 envs = 1,024 flight + "
                                        "1,024 control waves) and the serial load -> compute -> store -> "
                                        "kernel-boundary timeline (DESIGN.md 4), not HBM bandwidth"},
        "rollout": roll,
        "ppo_rollout": ppo,
        "storage_f32": x32,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        for key, fn in (("cpu_baseline", cpu_baseline), ("cpu_baseline_batched", cpu_baseline_batched)):
            try:
                out[key] = fn() | cpu_info()
            except Exception as e:  # report, never hide
                out[key] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
