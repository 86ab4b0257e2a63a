"""The GPU env against the reference DLL's own recorded closed-loop tests (tests/golden/tb_transfer_first_log.json;
tests/tb_transfer.py and tests/test_tb_transfer_pin.py are the CPU side).

ControlTestCallback (neural/callbacks.py:60-100) runs through b747_rl_ctrl_amd.evaluate.run_step_tests on the
GPU with each recorded run's own initial policy (weights reconstructed from torch's generator history, 17 of the
18 runs), for every variant: settling time within one DLL sample of one reference (0.0025 s in the 4-reference
mean), overshoot and quality within 1e-6 relative of the recorded values, and at least the 45 metrics the CPU
oracle reproduces bit for bit in float32 (all but the SPEED_MODE open-loop quality) equal in float32 too
(measured: 48 of 51 for FAST and FAITHFUL, worst 3.0e-7, profiles/r04/pytest_gpu_tb_pin.log).  The first
run of the reference's process (generator state unknown) and every other run lie inside the range of 64 product
ActorCritic initialisations run as one 256-env batch.

The same rows' rollout/ep_rew_mean (the 20 stochastic training episodes of each run's first rollout, see
tests/tb_transfer.py oracle_first_rollout) replayed through BatchControllerEnv with every episode's reset draws
loaded and the replayed action noise: within 1e-6 relative of the records for every variant, at least 10 of 17
equal in float32 (measured 12 / 13 for FAST / FAITHFUL, worst 2.9e-7).  That covers the train
env's CONST / OSCILLATING / HYBRID episodes (including HYBRID's SEMI_MANUAL altitude-PID episodes), the CLASSIC
reward and all three action modes on the GPU path.

No MIXED case: MIXED's fp32 aerodynamics lives in the two-wave kernels of the bench / training specialization
(PID_LIKE, CLASSIC, MANUAL-DIRECT, CONST resets, AERO disturbance); the recorded configurations (fixed-reference
tests, no disturbance, ADD modes, HYBRID / OSCILLATING resets) all run the one-wave kernels, where MIXED is FAST.
MIXED is held to the north star's per-step gate in tests/test_gpu_mixed.py."""
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
    done, exact, total, worst = {}, 0, 0, 0.0
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
    print(f"\n{variant}: {exact} of {total} recorded metrics equal in float32, worst relative error {worst:.1e}")
    assert total == 51 and exact >= 45


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
    assert worst <= 1e-6 and exact >= 12         # round 4 (test-side float32 sums of the float32 rewards): 12 / 13


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
