"""The GPU env against the reference DLL's own recorded closed-loop tests (tests/golden/tb_transfer_first_log.json;
tests/tb_transfer.py and tests/test_tb_transfer_pin.py are the CPU side).

ControlTestCallback (neural/callbacks.py:60-100) runs through b747_rl_ctrl_amd.evaluate.run_step_tests on the
GPU with each recorded run's own initial policy (weights reconstructed from torch's generator history, 17 of the
18 runs), for every variant: settling time within one DLL sample of one reference (0.0025 s in the 4-reference
mean), overshoot and quality within 1e-6 relative of the recorded values, and the 48 metrics the CPU oracle
reproduces bit for bit in float32 (all but the SPEED_MODE open-loop quality) equal in float32 too (measured: 48 of
51 for FAST and FAITHFUL, worst 3.0e-7).  The 17 runs hold 7 distinct trajectories (a process's later runs start
from its first run's seeded policy), i.e. 21 distinct metrics, 19 of them float32-equal.  The first
run of the reference's process (generator state unknown) and every other run lie inside the range of 64 product
ActorCritic initialisations run as one 256-env batch.

The same rows' rollout/ep_rew_mean (the 20 stochastic training episodes of each run's first rollout, see
tests/tb_transfer.py oracle_first_rollout) replayed through BatchControllerEnv with every episode's reset draws
loaded and the replayed action noise: within 1e-6 relative of the records for every variant, at least 16 of 17
(17 distinct trajectories) equal in float32 (measured 16 / 16 for FAST / FAITHFUL, worst 5.5e-7).  That covers the train
env's CONST / OSCILLATING / HYBRID episodes (including HYBRID's SEMI_MANUAL altitude-PID episodes), the CLASSIC
reward and all three action modes on the GPU path.

The recorded configurations (fixed-reference tests, no disturbance, ADD modes, HYBRID / OSCILLATING resets) run
the one-wave kernels, where MIXED is FAST.  MIXED's fp32 aerodynamics lives in the two-wave kernels of the bench /
training specialization; test_gpu_bench_kernels_reproduce_the_recorded_step_tests (below) sets the three PID_LIKE
DIRECT_CONTROL runs up so that they fly those kernels -- the bench's own k_env_step_split and k_rollout_split -- for
FAST and MIXED alike."""
import numpy as np
import pytest
import torch

import tb_transfer as T

pytestmark = pytest.mark.gpu

POLICIES = 64


def _run(group, policy, replicas=1, variant="fast"):
    from b747_rl_ctrl_amd import CtrlMode, ObservationType
    from b747_rl_ctrl_amd.evaluate import run_step_tests
    obs_name, mode_name = group
    mode, amax = T.MODES[mode_name]
    return run_step_tests(policy, T.REFS, state0=T.STATE0.tolist(), tk=T.TK,
                          observation_type=ObservationType(T.OBS[obs_name]), ctrl_mode=CtrlMode(mode),
                          sample_time=T.SAMPLE_TIME, replicas=replicas, action_max=amax, variant=variant)


def _means(out, replicas):
    """the callback's float32 means over the 4 references, per replica"""
    per = lambda k: out[k].reshape(replicas, len(T.REFS)).mean(1).to(torch.float32).cpu().numpy()
    return np.stack([per(k) for k in T.KEYS], 1)          # [replicas, 3]


def _device_policy(weights):
    (w0, b0), (w1, b1), (w2, b2) = [(w.cuda(), b.cuda()) for w, b in weights]

    def act(obs):
        h = torch.tanh(torch.tanh(obs @ w0.T + b0) @ w1.T + b1)
        return (h @ w2.T + b2)[:, 0].clamp(-1, 1)
    return act


def _initial_policies(obs_dim):
    """the deterministic actions of POLICIES freshly initialised ActorCritics, env j -> policy j // 4"""
    from b747_rl_ctrl_amd.ppo import ActorCritic
    nets = []
    for s in range(POLICIES):
        torch.manual_seed(1000 + s)
        nets.append(ActorCritic(obs_dim))
    lin = [[m for m in n.pi_net if isinstance(m, torch.nn.Linear)] + [n.action_net] for n in nets]
    W = [torch.stack([l[i].weight.detach() for l in lin]).cuda() for i in range(3)]
    B = [torch.stack([l[i].bias.detach() for l in lin]).cuda() for i in range(3)]

    def act(obs):
        x = obs.reshape(POLICIES, len(T.REFS), obs_dim)
        for i in range(3):
            x = torch.einsum("pho,pro->prh", W[i], x) + B[i][:, None, :]
            x = torch.tanh(x) if i < 2 else x
        return x.reshape(-1).clamp(-1, 1)
    return act


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_gpu_reproduces_the_recorded_runs(variant):
    runs = T.load_fixture()
    done, exact, total, worst, distinct = {}, 0, 0, 0.0, {}
    for name in sorted(runs):
        w = T.reference_weights(name)
        if w is None:
            continue
        key = T.split_run(name) + (T.previous_obs(name),)
        if key not in done:
            done[key] = _means(_run(T.split_run(name), _device_policy(w), variant=variant), 1)[0]
        m, v = done[key], runs[name]
        assert abs(m[0] - v["settling_time"]) <= 0.0025 + 1e-6, (name, m, v)
        err = T.rel_err(m, v)
        assert max(err[1:]) <= 1e-6, (name, variant, m, v, err)
        eq = T.f32_equal(m, v)
        exact, total, worst = exact + sum(eq), total + 3, max(worst, max(err))
        distinct[tuple(v[k] for k in T.KEYS)] = sum(eq)
    # 17 runs, but runs after their process's first share its th.manual_seed(1) policy (env/ctrl_env.py:76-78): the
    # records hold 7 distinct trajectories (21 distinct metrics)
    dexact = sum(distinct.values())
    print(f"\n{variant}: {exact} of {total} recorded metrics ({dexact} of {3 * len(distinct)} distinct, "
          f"{len(distinct)} trajectories) equal in float32, worst relative error {worst:.1e}")
    assert total == 51 and len(distinct) == 7
    assert exact >= 48 and dexact >= 19            # measured (rounds 4-6): 48 of 51, 19 of 21 distinct


@pytest.mark.parametrize("group", sorted({T.split_run(n) for n in T.load_fixture()}), ids=lambda g: "-".join(g))
def test_recorded_runs_inside_the_gpu_initial_policy_range(group):
    runs = T.load_fixture()
    out = _run(group, _initial_policies(T.OBS_DIM[group[0]]), replicas=POLICIES)
    m = _means(out, POLICIES)
    lo, hi = m.min(0), m.max(0)
    for name, v in runs.items():
        if T.split_run(name) == group:
            for j, k in enumerate(T.KEYS):
                assert T.within(v[k], lo[j], hi[j], 0.25), (name, k, v[k], lo[j], hi[j])
    print(f"\n{group}: GPU initial-policy range settling [{lo[0]:.4f}, {hi[0]:.4f}] overshoot [{lo[1]:.6f}, "
          f"{hi[1]:.6f}] quality [{lo[2]:.7f}, {hi[2]:.7f}]")


def _gpu_first_rollouts(group, names, variant):
    """the first training rollout of each recorded run in `names` (one (obs, ctrl mode) group) on the GPU, through
    the integration surface neural/agent.py trains on -- B747VecEnv (SubprocVecEnv + VecMonitor) over
    BatchControllerEnv: env 4r + w is run r's worker w; every episode's reset draws are loaded into the env
    (reset_ref_mode None: state0, reference, ctrl flags for HYBRID's SEMI_MANUAL / MANUAL switch) and all envs reset
    together at the 400-step episode boundary; actions = the reconstructed initial actor's mean (on the GPU) + the
    replayed noise, clipped; the episode returns are step_wait's infos[i]["episode"]["r"] (VecMonitor's float32
    accumulation, done by the kernels) and the mean SB3's safe_mean of them.  -> float32 ep_rew_mean per run"""
    from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, RewardType
    from b747_rl_ctrl_amd import B747VecEnv, ep_rew_mean
    from b747_rl_ctrl_amd._lib import F_PID_CS, F_RP
    obs_name, mode_name = group
    mode, amax = T.MODES[mode_name]
    runs = len(names)
    n = 4 * runs
    # SEMI_MANUAL: the env's altitude command slot is live (HYBRID episodes fly the CS PID); each env's
    # control flags are then set per episode, MANUAL (F_RP) or SEMI_MANUAL (F_RP | F_PID_CS)
    env = BatchControllerEnv(n, ObservationType(T.OBS[obs_name]), RewardType.CLASSIC, True, True,
                             CtrlType.SEMI_MANUAL, CtrlMode(mode), reset_ref_mode=None, tk=T.TK, sample_time=T.SAMPLE_TIME,
                             action_max=amax, auto_reset=False, variant=variant)
    venv = B747VecEnv(env)
    reps = [T.reference_rollout_noise(nm) for nm in names]
    draws = [T.worker_draws(nm) for nm in names]
    W = [torch.stack([r[0][i][0] for r in reps]).cuda() for i in range(3)]
    B = [torch.stack([r[0][i][1] for r in reps]).cuda() for i in range(3)]
    noise = torch.cat([r[1] for r in reps], 1).cuda()                   # [2048, n]
    od = T.OBS_DIM[obs_name]

    def mean(obs):
        x = torch.as_tensor(obs, device="cuda").reshape(runs, 4, od)
        for i in range(3):
            x = torch.einsum("pho,pro->prh", W[i], x) + B[i][:, None, :]
            x = torch.tanh(x) if i < 2 else x
        return x.reshape(-1)

    def load_episode(e):
        for j in range(n):
            d = draws[j // 4][e]
            env.state0[:, j] = torch.as_tensor(d["state0"], dtype=torch.float64)
            env.flags[j] = F_RP | (F_PID_CS if d.get("hybrid_ctrl") else 0)
            if d["kind"] == "osc":
                env.ref[1:7, j] = torch.as_tensor(d["osc"], dtype=torch.float64)
                env.ref_kind[j] = 1
            else:
                env.ref[0, j] = d["ref"]
                env.ref_kind[j] = 0
            if "h" in d:
                env.ref[7, j] = d["h"]
        return venv.reset()

    obs = load_episode(0)
    episodes = [[] for _ in range(runs)]                                   # VecMonitor records in finishing order
    for call in range(T.ROLLOUT_STEPS):
        a = (mean(obs) + noise[call]).clamp(-1, 1)
        obs, rew, done, infos = venv.step(a.cpu().numpy()[:, None])
        if (call + 1) % 400 == 0:
            assert bool(done.all())
            for j in range(n):
                assert infos[j]["episode"]["l"] == 400 and isinstance(infos[j]["episode"]["r"], np.float32)
                episodes[j // 4].append(infos[j]["episode"])
            obs = load_episode((call + 1) // 400)
        else:
            assert not bool(done.any())
    return [float(ep_rew_mean(eps)) for eps in episodes]


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_gpu_reproduces_the_recorded_first_rollouts(variant):
    runs = T.load_fixture()
    groups = {}
    for name in sorted(runs):
        if T.reference_rollout_noise(name) is not None:
            groups.setdefault(T.split_run(name), []).append(name)
    exact, worst = 0, 0.0
    for group, names in groups.items():
        for name, m in zip(names, _gpu_first_rollouts(group, names, variant)):
            v = runs[name]["ep_rew_mean"]
            err = abs(m - v) / abs(v)
            print(f"\n{name}: GPU {m!r} recorded {v!r} rel {err:.1e}", end="")
            exact += bool(np.float32(m) == np.float32(v))
            worst = max(worst, err)
    print(f"\n{variant}: {exact} of 17 first-rollout ep_rew_mean equal in float32, worst relative error {worst:.1e}")
    # every first rollout is its own trajectory (its own replayed noise and reset draws): 17 distinct records;
    # measured (round 5-6, VecMonitor's float32 returns in the kernels): 16 of 17 for FAST and FAITHFUL
    assert worst <= 1e-6 and exact >= 16


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_gpu_training_replay_tracks_the_record(variant):
    """The reference's recorded training (tests/tb_training.py) with the GPU in every role: the product PPO's
    two-launch rollout path (b747_policy_act sampling with the replayed noise, b747_env_rollout stepping the 4
    workers' BatchControllerEnv), its update on the GPU, the test callbacks through run_step_tests.  The first
    3 iterations (3 x 8,192 env steps, 2 updates of 1,280 minibatches) meet the CPU replay's gates."""
    import tb_training as TT
    rec = TT.load_curves(TT_RUN)
    rp = TT.TrainingReplay(TT_RUN, "gpu", variant)
    exact = total = 0
    for _ in range(3):
        step, entry = rp.step_iteration()
        cmp_ = TT.check_entry(entry, rec, step)
        exact += sum(c[2] for c in cmp_.values())
        total += len(cmp_)
        print(f"\n{variant} step {step}: " + " ".join(f"{t.split('/')[1]}={'=' if c[2] else f'{c[3]:.0e}'}"
                                                     for t, c in sorted(cmp_.items())), end="")
    print(f"\n{variant}: {exact} of {total} recorded values equal in float32")
    assert total == 4 + 12 + 12
    assert exact >= {"fast": 16, "faithful": 17}[variant]   # measured (round 5, VecMonitor's float32 returns): 16 / 17


TT_RUN = "PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2"


# ---------------------------------------------------------------------------------------------------------------
# The bench's own two-wave kernels against the same records (VERDICT r4 next #1a).  The recorded step tests run the
# one-wave kernels above (fixed references, no disturbance: not the training specialization).  The PID_LIKE
# DIRECT_CONTROL runs are the training configuration's observation / action / controller (two of the three have a
# reconstructed initial policy: HYBRID and OSCILLATING, 6 recorded metrics), so they run on the
# specialised two-wave kernels once the env is set up that way: CONST resets and the AERO disturbance with its
# drawn errors zeroed after the reset (aero_err = 0, the DLL default the test env flies), the test's state0 and
# reference loaded by a reset with reset mode None, then the configuration switched to the specialisation.
#   * k_env_step_split (the headline, b747_env_step at sample_time = dt): main.py's sample_time = 0.05 reproduced
#     by holding each action for 5 DLL steps (Controller.step injects the same command every sub-step);
#   * k_rollout_split<false, SUB> (b747_env_step at sample_time = 0.05: 5 DLL steps in one launch).
# Neither kernel records signals, so the pitch the callback's Storage keeps (the DLL's state_vartheta output of
# each DLL step) is the DLL's output map applied to the GPU state before each step: one oracle step (test-side
# checker) from the GPU's (X, disc, k, Memory) per DLL step, 2,000 x 12.  ITSE likewise.

def _spec_step_env(n, vrefs, amax, variant, sample_time):
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  RewardType)
    env = BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                             CtrlMode.DIRECT_CONTROL, reset_ref_mode=None,
                             disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=T.TK, sample_time=sample_time,
                             action_max=amax, variant=variant)
    env.set_state0(torch.tensor(T.STATE0, dtype=torch.float64))
    env.set_reference(vartheta=torch.tensor(vrefs, dtype=torch.float64))
    obs = env.reset().clone()
    env.aero_err.zero_()                       # the test env has no disturbance: the DLL's aero_err = 0
    env.cfg.reset_ref_mode = 0                 # CONST: the specialisation (no reset happens before t = tk)
    env.cfg.tk = T.TK + 0.005                  # no done at the episode's last DLL step: its ITSE is read afterwards
    return env, obs


def _dll_outputs(states, deltaz, vrefs, h_zh):
    """state_vartheta and ITSE after each DLL step: one oracle step from each GPU state (X, disc, k, mem)"""
    import oracle_lib as O
    X, disc, k, mem = states
    S, n = X.shape[0], X.shape[2]
    b = O.Batch(S * n)
    b.X[:] = X.transpose(1, 0, 2).reshape(18, S * n)
    b.disc[:] = disc.transpose(1, 0, 2).reshape(9, S * n)
    b.k[:] = k.reshape(-1).astype(np.uint32)
    b.mem[:] = mem.reshape(-1)
    b.deltaz[:] = deltaz.reshape(-1)
    b.vartheta[:] = np.tile(vrefs, S)
    b.h_zh[:] = np.tile(h_zh, S)
    b.flags[:] = O.F_RP
    O.oracle_step(b, 1)
    sig = b.sig.reshape(31, S, n)
    return sig[O.SIG_NAMES.index("sim_time")], sig[O.SIG_NAMES.index("vartheta")], sig[O.SIG_NAMES.index("ITSE")]


@pytest.mark.parametrize("variant", ["fast", "mixed"])
def test_gpu_bench_kernels_reproduce_the_recorded_step_tests(variant):
    import math
    import stepinfo_ref as SI
    runs = T.load_fixture()
    names = sorted(nm for nm in runs if T.split_run(nm) == ("PID_LIKE", "DIRECT_CONTROL")
                   and T.reference_weights(nm) is not None)
    assert len(names) == 2                     # (the CONST run is its process's first: initial policy unknown)
    mode, amax = T.MODES["DIRECT_CONTROL"]
    n = 4 * len(names)
    vrefs = np.array(T.REFS * len(names))
    W = [[w.cuda() for w, _ in T.reference_weights(nm)] for nm in names]
    B = [[b.cuda() for _, b in T.reference_weights(nm)] for nm in names]

    def policy(obs):                           # SB3 predict(deterministic): the actor mean, clipped to the box
        out = []
        for r in range(len(names)):
            x = obs[4 * r:4 * r + 4]
            x = torch.tanh(torch.tanh(x @ W[r][0].T + B[r][0]) @ W[r][1].T + B[r][1]) @ W[r][2].T + B[r][2]
            out.append(x[:, 0].clamp(-1, 1))
        return torch.cat(out)

    env, obs = _spec_step_env(n, vrefs, amax, variant, None)
    assert env.kernel() == "step_split"
    env5, obs5 = _spec_step_env(n, vrefs, amax, variant, T.SAMPLE_TIME)
    assert env5.kernel() == "rollout_split"
    steps = int(round(T.TK / 0.01))
    Xs, Ds, Ks, Ms, dz = (np.empty((steps, 18, n)), np.empty((steps, 9, n)), np.empty((steps, n), np.uint32),
                          np.empty((steps, n), np.uint8), np.empty((steps, n)))
    worst5 = worst5o = 0.0
    for u in range(steps):
        if u % 5 == 0:
            a = policy(obs)
            a32 = (a.to(torch.float64) * amax).to(torch.float32).to(torch.float64).cpu().numpy()   # env/ctrl_env.py:262
            obs5, _, _, _ = env5.step(a)       # the sample_time = 0.05 env: 5 DLL steps in one launch
        Xs[u], Ds[u] = env.X.cpu().numpy(), env.disc.cpu().numpy()
        Ks[u], Ms[u], dz[u] = env.k.cpu().numpy().astype(np.uint32), env.mem.cpu().numpy(), a32
        obs, _, done, _ = env.step(a)
        assert not bool(done.any())
        if u % 5 == 4:                         # both at the same DLL step: the same state
            g, r = env5.X.cpu().numpy(), env.X.cpu().numpy()
            span = np.maximum(np.abs(r).max(axis=1, keepdims=True), 1.0)
            worst5 = max(worst5, float(np.max(np.abs(g - r) / span)))
            worst5o = max(worst5o, float((obs5 - obs).abs().max()))
    ts, th, itse = _dll_outputs((Xs, Ds, Ks, Ms), dz, vrefs, env.h_zh.cpu().numpy())
    itse_end = itse[-1]
    got = {k: [] for k in T.KEYS}
    for j in range(n):
        info = SI.calc_stepinfo(list(th[:, j] * 180 / math.pi), vrefs[j] * 180 / math.pi, ts=list(ts[:, j]))
        got["settling_time"].append(info["settling_time"])
        got["overshoot"].append(abs(info["overshoot"]))
        got["quality"].append(math.exp(-60 * 0.1 * itse_end[j] / (T.TK * vrefs[j] ** 2)))
    worst, exact = 0.0, 0
    for r, nm in enumerate(names):
        rec = runs[nm]
        for k in T.KEYS:
            m = float(np.mean(got[k][4 * r:4 * r + 4]))
            rel = abs(m - rec[k]) / abs(rec[k])
            exact += bool(np.float32(m) == np.float32(rec[k]))
            print(f"\n{variant} {nm} {k}: GPU two-wave {m!r} recorded {rec[k]!r} rel {rel:.1e}", end="")
            if k == "settling_time":
                assert abs(m - rec[k]) <= 0.01 / 4 + 1e-9, (nm, k, m, rec[k])   # one DLL sample of one reference
            else:
                worst = max(worst, rel)
    print(f"\n{variant}: k_env_step_split {exact} of {3 * len(names)} recorded metrics float32-equal, worst overshoot / quality "
          f"relative error {worst:.1e}; k_rollout_split (sample_time 0.05) state within {worst5:.1e} of it, "
          f"observations within {worst5o:.1e}")
    # The two runs record ONE trajectory (the same th.manual_seed(1) policy, the open-loop response that never
    # settles: overshoot 63.09 %, settling 19.99 s), so this is one distinct triple compared twice.
    # measured (profiles/r05): FAST 6 of 6 float32-equal, worst 1.8e-8; MIXED 2 of 6 (the settling times), worst
    # 1.9e-5 -- quality = exp(-6 ITSE / ...) integrates MIXED's fp32-force error in the pitch error over the 20 s
    assert len({tuple(runs[nm][k] for k in T.KEYS) for nm in names}) == 1
    assert exact >= {"fast": 6, "mixed": 2}[variant]
    assert worst <= {"fast": 1e-7, "mixed": 1e-4}[variant]
    assert worst5 <= 1e-12 and worst5o <= 1e-6
