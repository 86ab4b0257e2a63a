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

Launch:  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks itself, one per GPU)
         python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...    (the driver's form)
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
    one U_com history slot of four (-24 B) and the DSS pair on its 0.05 s tick only (-16 B x 4/5), and reads three
    of the four history slots on that tick only (-8 B - 24 B x 4/5)."""
    xb = 8 if x_f64 else 4
    model = 18 * xb + 9 * 8 + 4 + 1                     # X, disc, k, mem
    model_w = model
    if single_step:
        # X without q1, q2; disc: x_dss, y_dss, rl_prevY, e_prev, ed_prev read, the three history slots the delay
        # reads only on the 0.05 s DSS tick (b747_split.h Hist3); written: rl_prevY, e_prev, ed_prev, one history
        # slot, the DSS pair on its tick
        model = 16 * xb + 5 * 8 + 3 * 8 / 5 + 4 + 1
        model_w = 16 * xb + 3 * 8 + 8 + 2 * 8 / 5 + 4 + 1
    slot = 4                                             # ep_return (float, ABI 10)
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
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", rnd, name)
        if os.path.exists(path):
            return json.load(open(path)), f"profiles/{rnd}/{name}"
    return None, None


def make_env(n, rank, x_f64, device, seed=2024, variant="fast", sample_time=None):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=20, sample_time=sample_time,
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


REPS = 3   # every secondary line: one untimed replay, then REPS timed ones, each timed alone; the median is reported


def timed_replays(run, reps=REPS):
    """Seconds of `reps` calls of run(), each bracketed by synchronizes (after one untimed call)."""
    run()
    torch.cuda.synchronize()
    dts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
    return dts


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])


def graph_of(fn, device):
    """fn() captured in one HIP graph (torch.cuda.CUDAGraph) on a side stream."""
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        fn()
    torch.cuda.synchronize()
    return graph


def rate_line(n, units, dts, dll_per_env_step=1, **extra):
    """A secondary line from per-replay seconds: each replay = `units` env steps of every one of n envs."""
    dt = median(dts) / units
    out = {"value": round(n / dt, 1), "us_per_step": round(dt * 1e6, 3),
           "replays_us_per_step": [round(d / units * 1e6, 3) for d in dts], "timing": f"median of {len(dts)} replays"}
    if dll_per_env_step != 1:
        out["dll_steps_per_s"] = round(n * dll_per_env_step / dt, 1)
    return extra | out


def rollout_rate(env, k=100, seed=5):
    """Secondary line: the same env steps with k pre-sampled actions per launch (b747_env_rollout,
    state kept in registers across the k steps, every step's obs/reward/done written).  Its own k rows of
    actions, so the launch holds k steps whatever --steps / --warmup are."""
    n, dev = env.n, env.X.device
    g = torch.Generator(device=dev).manual_seed(seed)
    actions = torch.rand(k, n, generator=g, device=dev) * 2 - 1
    obs_seq = torch.empty(k, n, env.obs_dim, device=dev)
    rew_seq = torch.empty(k, n, device=dev)
    done_seq = torch.empty(k, n, dtype=torch.uint8, device=dev)
    dts = timed_replays(lambda: env.rollout(actions, obs_seq, rew_seq, done_seq))
    return rate_line(n, k, dts, int(env.cfg.n_sub), steps_per_launch=k)


def storage_f32_rate(n, rank, device, variant, k=100, seed=6):
    """Secondary line: the same per-step launches with X stored in fp32 -- the SoA layout the north star
    and SURVEY 8(d)'s 277 B assume; every stage still computes in fp64 (loaded into fp64 registers, rounded
    once per step by the store; tests/test_gpu_split.py).  The headline keeps fp64 storage."""
    env = make_env(n, rank, False, device, variant=variant)
    g = torch.Generator(device=device).manual_seed(seed)
    actions = torch.rand(k, n, generator=g, device=device) * 2 - 1   # its own k launches, whatever --steps is
    for t in range(5):
        env.step(actions[t])

    def steps():
        for t in range(k):
            env.step(actions[t])
    graph = graph_of(steps, device)
    return rate_line(n, k, timed_replays(graph.replay), state_storage="f32", steps=k,
                     bytes_per_env_step_stored=round(env_bytes_per_step(False, env.obs_dim,
                                                                       single_step=variant == "fast"), 1))


def ppo_rollout_rate(n, rank, x_f64, device, variant, steps=64, sample_time=None):
    """BASELINE configs[4]: 65,536 envs + on-GPU PPO rollout (SB3-default MlpPolicy 64-64 tanh,
    separate pi/vf): per step policy forward + Gaussian sample + clip + fused env step (b747_ppo_rollout:
    the whole rollout in one launch + the batched value pass).  End-to-end env-steps/s (b747_rl_ctrl_amd/ppo.py)."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = make_env(n, rank, x_f64, device, seed=99, variant=variant, sample_time=sample_time)
    ppo = PPO(env, PPOConfig(n_steps=steps), seed=0)
    ppo.last_obs.copy_(env.obs)
    dts = timed_replays(lambda: ppo.collect_rollouts(steps))
    return rate_line(n, steps, dts, int(env.cfg.n_sub),
                     workload="configs[4]: 65536 envs + PPO rollout (policy fwd + sample + env step)",
                     rollout_steps=steps, fused_kernel=bool(ppo.rollout_kernel))


def ppo_training_rate(n, rank, device, variant, steps=64, iterations=2):
    """End-to-end PPO training throughput in the units of the only throughput the reference publishes, SB3's
    time/fps (env steps per wall-clock second of learn(), rollouts AND updates: BASELINE.md 1, 323-360 env-steps/s
    on its 4-process CPU setup): main.py's sample_time = 0.05 on the config-5 env, one iteration = a 64-step
    rollout of every env (b747_ppo_rollout) + GAE + PPO.train (10 epochs, minibatches of 65,536, SB3's other
    defaults).  The update dominates; a separate number, not the headline."""
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    env = make_env(n, rank, True, device, seed=98, variant=variant, sample_time=0.05)
    ppo = PPO(env, PPOConfig(n_steps=steps, batch_size=65536), seed=0)
    ppo.last_obs.copy_(env.obs)

    def iteration():
        ppo.collect_rollouts(steps)
        ppo.compute_gae(steps)
        ppo.train(steps)
    iteration()                                   # untimed: allocator, kernels, graphs
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iterations):
        iteration()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iterations
    return {"value": round(n * steps / dt, 1), "unit": "env-steps/s (SB3 time/fps semantics: rollout + update)",
            "s_per_iteration": round(dt, 4), "envs": n, "rollout_steps": steps, "sample_time": 0.05,
            "epochs": ppo.cfg.n_epochs, "batch_size": ppo.cfg.batch_size,
            "reference_time_fps": "323-360 env-steps/s (tensorboard.xlsx, PID_LIKE runs, final value; BASELINE.md 1)"}


def mixed_rates(n, rank, device, k=100, seed=8):
    """Secondary line: the MIXED variant (include/b747.h B747_VARIANT_MIXED) -- FAST with the two-wave kernels'
    flight aerodynamics in fp32, state / attitude / integration / control fp64.  Its gates (tests/test_gpu_mixed.py,
    DESIGN.md 5): per step from the oracle's state, FAST's replay bar (2e-6 relative + 1e-7 absolute + 1e-7 of the
    batch's scale; measured <= 0.28 of it); free-running over the 20 s episode, quantiles of the deviation.  The
    headline stays on FAST fp64.  Per-step launches (K in
    one HIP graph), K env steps per launch, and the config-5 PPO rollout."""
    env = make_env(n, rank, True, device, variant="mixed")
    g = torch.Generator(device=device).manual_seed(seed)
    actions = torch.rand(k, n, generator=g, device=device) * 2 - 1
    for t in range(5):
        env.step(actions[t])

    def steps():
        for t in range(k):
            env.step(actions[t])
    graph = graph_of(steps, device)
    step = rate_line(n, k, timed_replays(graph.replay), launches=k, api="b747_env_step")
    step["kernel_avg_us"] = step["us_per_step"]
    step["roofline_frac"] = round(ALGO_BYTES_PER_ENV_STEP * n / (step["us_per_step"] * 1e-6) / 1e9 / PEAK_HBM_GBS, 4)
    return {"variant": "mixed", "precision": "fp32 flight aerodynamics, fp64 state/attitude/integration/control; "
                                            "per step from the oracle's state within 2e-6 relative + 1e-7 absolute + "
                                            "1e-7 of the batch scale (tests/test_gpu_mixed.py); but over the recorded "
                                            "2,000-step closed-loop step test the quality metric is 1.9e-5 off the "
                                            "reference's record (tests/test_gpu_tb_pin.py), beyond the north star's "
                                            "1e-5: opt-in only, not the headline",
            "step": step, "rollout": rollout_rate(env), "ppo_rollout": ppo_rollout_rate(n, rank, True, device, "mixed")}


def main05_rates(n, rank, device, variant, k=40):
    """"with main.py's sample_time = 0.05, one env step is 5 such steps; report that separately"
    (/root/reference/main.py:18, core/controller.py:258-264).  The bench workload at sample_time = 0.05:
    per-step launches (b747_env_step, one env step = 5 DLL steps, K of them in one HIP graph), K env steps per
    launch (b747_env_rollout) and the config-5 PPO rollout; env-steps/s and DLL-steps/s each."""
    env = make_env(n, rank, True, device, variant=variant, sample_time=0.05)
    g = torch.Generator(device=device).manual_seed(55)
    actions = torch.rand(k, n, generator=g, device=device) * 2 - 1
    for t in range(5):
        env.step(actions[t])

    def steps():
        for t in range(k):
            env.step(actions[t])
    graph = graph_of(steps, device)
    step = rate_line(n, k, timed_replays(graph.replay), int(env.cfg.n_sub), launches=k, api="b747_env_step")
    roll = rollout_rate(env, k=20)
    ppo = ppo_rollout_rate(n, rank, True, device, variant, steps=64, sample_time=0.05)
    return {"sample_time": 0.05, "dll_steps_per_env_step": int(env.cfg.n_sub), "unit": "env-steps/s (dll_steps_per_s beside)",
            "step": step, "rollout": roll, "ppo_rollout": ppo}


def config2_rates(device, k=100):
    """BASELINE configs[1]: 4,096 envs of the raw model (core/model.py Model, the DLL step API: b747_model_step with
    the 31 output signals written every step), MANUAL with the rate limiter on and both PIDs off, the default initial
    state, a held elevator step deltaz = -(1 + i mod 10) deg (tests/test_gpu_model.py
    test_config2_4096_envs_step_elevator_2000_steps).  The small-batch regime that replaces the reference's 4-env
    SubprocVecEnv (/root/reference/neural/agent.py:65,74): per-step launches (K in one HIP graph; each env over three
    waves, k_model_step_split) and K DLL steps in one launch (the same three waves with the state in registers across
    the steps, k_model_steps_split)."""
    from b747_rl_ctrl_amd import F_RP, BatchModel
    n = 4096
    m = BatchModel(n, device=device)
    m.flags.fill_(F_RP)
    m._deltaz.copy_(-(1.0 + torch.arange(n, device=device, dtype=torch.float64) % 10) * math.pi / 180.0)
    m.step(5)

    def steps():
        for _ in range(k):
            m.step(1)
    graph = graph_of(steps, device)
    step = rate_line(n, k, timed_replays(graph.replay), launches=k, api="b747_model_step(n_steps=1)")
    multi = rate_line(n, k, timed_replays(lambda: m.step(k)), steps_per_launch=k, api=f"b747_model_step(n_steps={k})")
    if not torch.isfinite(m.X).all():
        raise RuntimeError("config 2: non-finite state")
    return {"workload": "configs[1]: 4096 envs, fixed-dt RK4 (h = 0.01 s), held elevator step -(1 + i mod 10) deg, "
                        "MANUAL + rate limiter, default state0; every step's 31 DLL output signals written",
            "envs": n, "unit": "env-steps/s (one env step = one DLL step)", "step": step, "multi_step": multi}


def measured_profile(x_f64, variant, envs):
    """Per-launch HBM bytes (rocprofv3 PMC FETCH_SIZE x 2 + WRITE_SIZE) and SQ counters of the env-step
    kernel from the committed profile summaries (tools/pmc_summary.py) when they were taken on this
    exact workload; otherwise Nones."""
    if not (x_f64 and variant == "fast"):
        return None, None, None, None, None
    d, src = committed_profile("env_step_pmc_traffic.json")
    if d is None or d.get("envs") != envs:
        return None, None, None, None, None
    sq, sq_src = committed_profile("env_step_sq_counters.json")
    return d["traffic_bytes_per_launch"], src, (sq or {}).get("per_wave"), (sq or {}).get("waves"), sq_src


def rank_launch_cmd(argv, n, port):
    """The torch.distributed.run command that starts n ranks of this script on one node (127.0.0.1
    rendezvous), each with the same arguments; WORLD_SIZE / RANK / LOCAL_RANK come from the launcher."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """`python bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU) through
    torch.distributed.run and return its exit code; rank 0 prints the JSON line.  Runs before this process
    makes any GPU call (torch.cuda.device_count() does not initialise the device on this image)."""
    import socket
    import subprocess
    have = torch.cuda.device_count()
    if args.dist_backend == "nccl" and have < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {have} visible (RCCL runs one rank "
                         f"per GPU; --dist-backend gloo rehearses several ranks on fewer GPUs)")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")    # dmabuf IPC only on this pool (RCCL)
    return subprocess.run(rank_launch_cmd(argv, args.gpus, port), env=env).returncode


def check_world(args, world):
    """--gpus must be the number of ranks the job actually runs: fail loudly instead of printing a
    1-GPU line for an N-GPU request."""
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}; start N ranks with "
                         f"`python bench.py --gpus N` or torch.distributed.run --nproc-per-node N ... --gpus N")


def binder_note(valu_frac, sq, src):
    """What the committed SQ counters (tools/pmc_summary.py) say binds the per-step kernel, or None."""
    if not sq or not sq.get("SQ_WAVE_CYCLES"):
        return None
    wait = sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"]
    return {"source": src, "valu_issue_frac_per_simd": valu_frac, "wait_any_frac_per_wave": round(wait, 3),
            "reading": "fp64 VALU issue of the waves sharing a SIMD plus each wave's dependent-latency / memory waits "
                       "(DESIGN.md 4): HBM bandwidth is not what binds" if valu_frac and valu_frac < 0.8 else
                       "VALU issue bound"}


def budget_floor():
    """The per-step kernel's measured time budget (profiles/<round>/env_step_budget.json: phase stamps, SQ counters,
    fp64 VALU mix), or None."""
    d, src = committed_profile("env_step_budget.json")
    if d is None:
        return None
    out = {"source": src}
    out.update({k: v["value"] for k, v in d["terms"].items()})
    if "reading" in d:
        out["reading"] = d["reading"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--x32", action="store_true", help="store X in fp32 (compute stays fp64)")
    ap.add_argument("--eager", action="store_true", help="no HIP graph: one Python call per step")
    ap.add_argument("--variant", default="fast", choices=["fast", "faithful", "mixed"],
                    help="fast (default): identities for sin/cos/pow; faithful: the DLL's operation order; mixed: fast "
                         "with the flight aerodynamics in fp32 (tests/test_gpu_mixed.py gates)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) for real runs")
    ap.add_argument("--no-rollout", action="store_true",
                    help="skip the secondary lines (multi-step launches, config-5 PPO rollout, fp32 X storage)")
    ap.add_argument("--no-main05", action="store_true", help="skip the sample_time = 0.05 lines (main.py:18)")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU-only rehearsal of the rank launch: every rank joins a gloo group, all-reduces its rank "
                         "count and prints one JSON line; no GPU is touched (tests/test_bench_launcher.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if args.launch_check:
            args.dist_backend = "gloo"
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    check_world(args, world)
    if args.launch_check:
        import torch.distributed as tdist
        if world > 1:
            tdist.init_process_group("gloo")
        t = torch.ones(1)
        if world > 1:
            tdist.all_reduce(t)
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world,
                          "ranks_seen": tdist.get_world_size() if world > 1 else 1, "all_reduce": float(t)}), flush=True)
        if world > 1:
            tdist.destroy_process_group()
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU (torch.distributed.run); --dist-backend gloo with ranks sharing a GPU
    # only rehearses the multi-rank code path on a one-GPU box
    gpu = local % max(1, torch.cuda.device_count())
    # under a launcher (WORLD_SIZE set) every rank joins the group, a single one included: the N=1 point of a
    # scaling run then takes the same RCCL init / barrier / MAX path as N = 2..8
    if "WORLD_SIZE" in os.environ:
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
    ranks_seen = dist.get_world_size() if dist else 1
    # two more replays of the same graph after the timed region, for the spread a single replay hides (the
    # secondary lines report medians of such replays); `value` stays the one timed region above
    spread = [round(d / args.steps * 1e6, 3) for d in timed_replays(graph.replay, 2)] if graph is not None else None

    if not torch.isfinite(env.obs).all() or not torch.isfinite(env.reward).all():
        raise RuntimeError("non-finite obs/reward after the timed region")
    region_us = wall / args.steps * 1e6          # per launch incl. the launch-to-launch gap
    kern_us = region_event_us                    # HIP events over the timed region / K
    iso_us = isolated_launch_us(env, actions)
    # the secondary lines are per-GPU figures: measured at N = 1 only, so that a multi-rank run stays short
    secondary = not args.no_rollout and world == 1
    roll = rollout_rate(env) if secondary else None
    ppo = ppo_rollout_rate(args.envs, rank, x_f64, device, args.variant) if secondary else None
    x32 = storage_f32_rate(args.envs, rank, device, args.variant) if secondary and x_f64 else None
    m05 = main05_rates(args.envs, rank, device, args.variant) if secondary and not args.no_main05 else None
    train = ppo_training_rate(args.envs, rank, device, args.variant) if secondary and x_f64 else None
    mixed = mixed_rates(args.envs, rank, device) if secondary and args.variant == "fast" and x_f64 else None
    cfg2 = config2_rates(device) if secondary else None
    steps_done = int(env.k.min().item())  # sanity: envs advanced (auto-reset keeps k < 2000)
    stored = round(env_bytes_per_step(x_f64, env.obs_dim, single_step=args.variant == "fast"), 1)
    algo = ALGO_BYTES_PER_ENV_STEP
    achieved = algo * args.envs / (kern_us * 1e-6) / 1e9
    achieved_read = ALGO_READ_BYTES_PER_ENV_STEP * args.envs / (kern_us * 1e-6) / 1e9
    traffic, traffic_src, sq, sq_waves, sq_src = measured_profile(x_f64, args.variant, args.envs)
    valu_frac = None
    if sq and sq.get("SQ_WAVE_CYCLES"):
        # per SIMD: a wave's VALU-active share x the waves each of the 1,024 SIMDs runs (256 CUs x 4) -- the
        # single-step kernel puts three waves (flight, ahead, control) of the same 64 envs on every SIMD
        waves_per_simd = max(1.0, float(sq_waves or 1024) / 1024.0)
        valu_frac = round(sq["SQ_ACTIVE_INST_VALU"] * waves_per_simd / sq["SQ_WAVE_CYCLES"], 3)
    out = {
        "metric": "env steps/sec (batched B747 pitch sim)",
        "value": round(aggregate_rate(args.envs, args.steps, world, wall), 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "dist_backend": dist.get_backend() if dist else None,
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
        # matrix work); what the committed counters show actually binds the kernel is in "binder"
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "k_env_step_split", "bytes_per_env_step": algo,
                     "bytes_per_launch": algo * args.envs,
                     "read_bytes_per_env_step": ALGO_READ_BYTES_PER_ENV_STEP,
                     "hbm_read_frac": round(achieved_read / PEAK_HBM_GBS, 4),
                     "bytes_per_env_step_stored": stored,
                     "traffic_over_algorithmic": round(traffic / (algo * args.envs), 3) if traffic else None,
                     "kernel_avg_us": round(kern_us, 3), "launch_period_us": round(region_us, 3),
                     "isolated_launch_us": round(iso_us, 3), "replays_after_us_per_step": spread,
                     "valu_issue_frac": valu_frac,
                     "binder": binder_note(valu_frac, sq, sq_src),
                     "floor_us": budget_floor() if args.envs == ENVS_PER_GPU and x_f64 and args.variant == "fast" else None},
        "rollout": roll,
        "ppo_rollout": ppo,
        "storage_f32": x32,
        "sample_time_0.05": m05,
        "ppo_training": train,
        "variant_mixed": mixed,
        "config2": cfg2,
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
