"""The reference's recorded closed-loop test results replayed on the oracle (TEST INFRASTRUCTURE).

tests/golden/tb_transfer_first_log.json holds, for each of the 18 training runs in the reference's
tensorboard.xlsx, the first `transfer_custom/*` log point: ControlTestCallback.calc_stepinfo
(neural/callbacks.py:60-100) run by the reference on its DLL with the PPO policy still at its initial weights
(tests/golden/make_tb_fixture.py says why).  This module reruns that callback on the oracle:

  * the test env of main.py:57-72: tk 20 s, sample_time 0.05, norm obs/act, no disturbance, MANUAL control,
    action_max per ctrl mode (main.py:7-12), state0 [0, 11000, 250, 0, 0, 0] (main.py:124);
  * references +-5, +-10 deg (main.py:116), one fresh model each (callbacks.py:74-76, ctrl._init_model());
  * the Storage hook records pitch (deg) and time after every DLL step (core/controller.py:209-228) and
    calc_stepinfo (oracle/stepinfo_ref.py) + quality() (core/controller.py:334-336) score the episode;
  * the callback's means over the references, float32 as TensorBoard stores scalars.

The policy is SB3 1.4's default MlpPolicy (PPO's hyperparameters fall back to SB3 defaults, see the fixture
script): pi / vf MLPs [64, 64] with Tanh, orthogonal init (gain sqrt 2 hidden, 0.01 action head, zero biases),
deterministic action = mean clipped to the [-1, 1] box.  Its initial weights are reconstructed from torch's CPU
generator (`reference_weights`): main.py:133-152 trains the 18 runs one after another in one process, and each
ControlTestCallback builds a ControllerEnv, whose constructor calls th.manual_seed(1) (env/ctrl_env.py:75-78),
then loads a copy of the model (callbacks.py:70-72: one more policy construction).  The last test of a run is
at callback call 126,000 (500,000 timesteps -> 62 rollouts of 2048 x 4 = 126,976 calls, main.py:108, log
interval 1000); the 976 rollout steps after it each draw one [4, 1] Gaussian action sample; then the next run
builds its PPO policy.  So every run but the process's first starts from the same generator history:
  manual_seed(1) -> build policy(previous run's obs dim) -> 976 x normal_([4, 1]) -> build policy(obs dim).
That reproduces 17 of the 18 recorded runs (all but the first, PID_LIKE DIRECT CONST, whose generator state
at start is not recoverable).  For that one, and as a weight-free check for all, `band` draws many SB3-style
initialisations (numpy) and returns the metrics' range.  a = 0 (`zero_policy`) is the pure PID (ADD_*) /
open-loop (DIRECT) response.

The same row's rollout/ep_rew_mean is reproducible too (`oracle_first_rollout`): the 20 training episodes of
the first rollout (4 SubprocVecEnv workers x 5 episodes of 400 steps) take their resets from Python's `random`
seeded 1 in every worker (env/ctrl_env.py:76; `worker_draws`) and their actions from the initial actor's mean
plus the generator's Gaussian noise, which the replay continues past the weights (`reference_rollout_noise`).
That pins the train env's reset distributions (CONST / OSCILLATING / HYBRID with its SEMI_MANUAL switch), the
CLASSIC reward and the stochastic rollout semantics, not only the dynamics.

  python tests/tb_transfer.py [--seeds 16] [--out profiles/r04/tb_transfer_pin.txt]   (the full report)"""
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_env as R  # noqa: E402
from stepinfo_ref import calc_stepinfo  # noqa: E402

FIXTURE = os.path.join(HERE, "golden", "tb_transfer_first_log.json")
REFS = [5 * math.pi / 180, -5 * math.pi / 180, 10 * math.pi / 180, -10 * math.pi / 180]   # main.py:116
STATE0 = np.array([0, 11000, 250, 0, 0, 0], float)                                          # main.py:124
TK, SAMPLE_TIME = 20.0, 0.05                                                                # main.py:17,96
OBS = {"PID_LIKE": 0, "SPEED_MODE": 1}                  # env/ctrl_env.py ObservationType values
OBS_DIM = {"PID_LIKE": 3, "SPEED_MODE": 5}
MODES = {"DIRECT_CONTROL": (0, 17 * math.pi / 180),     # ctrl mode value, action_max (main.py:7-12)
         "ADD_PROC_CONTROL": (1, 1.0),
         "ADD_DIRECT_CONTROL": (3, 10 * math.pi / 180)}
KEYS = ("settling_time", "overshoot", "quality")
# main.py:100-110 loop order (obs outer, ctrl mode, reset mode inner): the process's first run
FIRST_RUN = ("PID_LIKE", "DIRECT_CONTROL", "CONST")
TAIL_SAMPLES = 976                                      # 126,976 - 126,000 rollout steps after the last test
CALLBACK_INTERVAL = 1000                                # main.py:19 log_interval (callback calls)
ROLLOUT_STEPS = 2048                                    # SB3 PPO default n_steps (per worker)
EPISODES_PER_WORKER = ROLLOUT_STEPS // 400              # 400 env steps per episode (tk 20 s / 0.05 s)


def load_fixture():
    with open(FIXTURE) as f:
        return json.load(f)["runs"]


def split_run(name):
    """'PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2' -> ('PID_LIKE', 'ADD_DIRECT_CONTROL')"""
    obs, rest = name.split("_MANUAL_")
    mode = next(m for m in MODES if rest.startswith(m + "_"))
    return obs, mode


def reset_mode(name):
    return name.split("_MANUAL_")[1].split("_CONTROL_")[1].split("_")[0]


def previous_obs(name):
    """obs type of the run main.py trained just before this one (the loop order of main.py:100-110)"""
    obs = split_run(name)[0]
    first_of_obs = split_run(name)[1] == "DIRECT_CONTROL" and reset_mode(name) == "CONST"
    return "PID_LIKE" if (obs == "SPEED_MODE" and first_of_obs) else obs


def zero_policy(obs):
    return np.float32(0.0)


def _sb3_build(obs_dim, full=False):
    """ActorCriticPolicy._build of SB3 1.4 with net_arch [dict(pi=[64, 64], vf=[64, 64])]: the nn.Linear
    constructions in MlpExtractor's order (pi0, vf0, pi1, vf1), action_net, value_net, then the orthogonal
    init through module.apply (policy_net then value_net, then action_net 0.01, value_net 1)"""
    import torch
    from torch import nn
    pi0, vf0, pi1, vf1 = nn.Linear(obs_dim, 64), nn.Linear(obs_dim, 64), nn.Linear(64, 64), nn.Linear(64, 64)
    act, val = nn.Linear(64, 1), nn.Linear(64, 1)
    for m, g in ((pi0, math.sqrt(2)), (pi1, math.sqrt(2)), (vf0, math.sqrt(2)), (vf1, math.sqrt(2)), (act, 0.01),
                 (val, 1.0)):
        nn.init.orthogonal_(m.weight, gain=g)
        with torch.no_grad():
            m.bias.fill_(0.0)
    mods = (pi0, pi1, act, vf0, vf1, val) if full else (pi0, pi1, act)
    return [(m.weight.detach().clone(), m.bias.detach().clone()) for m in mods]


def _replay_generator(name, rollout_calls=0, full=False):
    """torch's CPU generator history of recorded run `name` (see the module docstring): its initial actor
    weights, then the Gaussian noise of its first `rollout_calls` rollout steps [calls, 4] (one [4, 1] sample
    per step; the test callbacks at calls 1000 and 2000 re-seed and build a model copy after their step).
    Uses (and restores) the global generator."""
    import torch
    obs, mode = split_run(name)
    saved = torch.random.get_rng_state()
    try:
        torch.manual_seed(1)                                         # env/ctrl_env.py:78
        _sb3_build(OBS_DIM[previous_obs(name)])                      # the callback's model copy
        for _ in range(TAIL_SAMPLES):
            torch.empty(4, 1).normal_()                              # Normal.rsample of 4 workers' actions
        weights = _sb3_build(OBS_DIM[obs], full)
        noise = []
        for call in range(1, rollout_calls + 1):
            noise.append(torch.empty(4, 1).normal_()[:, 0].clone())
            if call % CALLBACK_INTERVAL == 0:                        # ControlTestCallback after this step
                torch.manual_seed(1)
                _sb3_build(OBS_DIM[obs])
        return weights, (torch.stack(noise) if noise else None)
    finally:
        torch.random.set_rng_state(saved)


def reference_weights(name):
    """The initial actor weights [(W, b)] x 3 of recorded run `name`; None for the process's first run."""
    if (split_run(name) + (reset_mode(name),)) == FIRST_RUN:
        return None
    return _replay_generator(name)[0]


def reference_rollout_noise(name):
    """(weights, noise [2048, 4] float32) of the first rollout of run `name`; None for the first run."""
    if (split_run(name) + (reset_mode(name),)) == FIRST_RUN:
        return None
    return _replay_generator(name, ROLLOUT_STEPS)


def reset_draws(rnd, mode, vmax=10 * math.pi / 180):
    """Controller.reset's random draws (core/controller.py:145-176) from the Python generator `rnd`, in the
    reference's order, as an oracle/ref_env.py draws dict"""
    h0, vx, vy, wz0 = rnd.uniform(1000, 11000), rnd.uniform(100, 265), rnd.uniform(-20, 20), rnd.uniform(-0.001, 0.001)
    d = {"state0": np.array([0, h0, vx, vy, 0, wz0]), "kind": "const", "ref": 0.0}
    if mode == "CONST":
        ref = rnd.uniform(-vmax, -1 * math.pi / 180)
        d["ref"] = ref * rnd.choice([1.0, -1.0])
    elif mode == "OSCILLATING":
        a1 = rnd.uniform(0, vmax)
        a2 = rnd.uniform(0, vmax - a1)
        a3 = rnd.uniform(0, vmax - a1 - a2)
        d["kind"], d["osc"] = "osc", (a1, a2, a3, rnd.uniform(0.01, 0.5), rnd.uniform(0.01, 0.5), rnd.uniform(0.01, 0.5))
    else:                                                            # HYBRID
        d["hybrid_ctrl"] = rnd.choice([True, False])
        if d["hybrid_ctrl"]:
            d["h"] = h0 + rnd.uniform(-1000, 1000)
        else:
            d["ref"] = rnd.uniform(-vmax, vmax)
    return d


def worker_draws(name, episodes=EPISODES_PER_WORKER + 1):
    """the reset draws of one worker's first `episodes` training episodes: every worker constructs its
    ControllerEnv with random.seed(1) (env/ctrl_env.py:76), whose constructor resets once (:96), and SB3's
    learn() resets again before the first step; all 4 workers therefore draw the same sequence"""
    import random
    rnd = random.Random(1)
    mode = reset_mode(name)
    reset_draws(rnd, mode)                                           # ControllerEnv.__init__'s reset
    return [reset_draws(rnd, mode) for _ in range(episodes)]


def oracle_first_rollout(name, record=False):
    """The 20 training episodes of run `name`'s first rollout on the oracle: SubprocVecEnv's 4 workers
    (neural/agent.py:63-81), each step's action = the initial actor's mean + the replayed noise (std 1),
    clipped to the box (SB3 collect_rollouts), auto-reset at done; returns accumulated in float32 as
    VecMonitor does.  -> (returns [20] in finishing order, their float32 mean = rollout/ep_rew_mean) and, with
    record, SB3's RolloutBuffer contents: obs [2048, 4, od] (what the policy saw), unclipped actions, float32
    rewards, dones [2048, 4] and the bootstrap observation [4, od]"""
    import torch
    obs_name, mode_name = split_run(name)
    mode, amax = MODES[mode_name]
    weights, noise = reference_rollout_noise(name)
    (w0, b0), (w1, b1), (w2, b2) = weights
    draws = worker_draws(name)
    envs = [R.RefControllerEnv(OBS[obs_name], 0, True, True,
                               R.RefController(3, mode, None, None, tk=TK, sample_time=SAMPLE_TIME, action_max=amax))
            for _ in range(4)]
    ep = [0] * 4
    obs = np.stack([e.reset(draws[0]) for e in envs])
    acc = np.zeros(4, np.float32)
    returns = []
    od = OBS_DIM[obs_name]
    buf = {"obs": np.zeros((ROLLOUT_STEPS, 4, od), np.float32), "act": np.zeros((ROLLOUT_STEPS, 4), np.float32),
           "rew": np.zeros((ROLLOUT_STEPS, 4), np.float32), "done": np.zeros((ROLLOUT_STEPS, 4), bool)}
    for call in range(ROLLOUT_STEPS):
        with torch.no_grad():
            x = torch.as_tensor(obs).float()
            mean = torch.tanh(torch.tanh(x @ w0.T + b0) @ w1.T + b1) @ w2.T + b2
            sample = (mean[:, 0] + noise[call] * 1.0).numpy()
            act = np.clip(sample, -1, 1)
        if record:
            buf["obs"][call], buf["act"][call] = x.numpy(), sample
        nxt = []
        for i, e in enumerate(envs):
            o, r, d = e.step(act[i])
            if record:
                buf["rew"][call, i], buf["done"][call, i] = r, d
            acc[i] = np.float32(np.float64(acc[i]) + r)   # VecMonitor: float32 returns += float64 rewards (arrays)
            if d:
                returns.append(float(acc[i]))
                acc[i] = 0
                ep[i] += 1
                o = e.reset(draws[ep[i]])
            nxt.append(o)
        obs = np.stack(nxt)
    m = float(np.mean(np.asarray(returns, np.float32)))   # SB3 safe_mean over the float32 "r" values: float32
    if record:
        buf["last_obs"] = obs.astype(np.float32)
        return returns, m, buf
    return returns, m


class _HostEnv:
    """what PPO reads of an env when its rollout buffers are filled from outside (CPU)"""

    class _Box:
        low, high = -1.0, 1.0

    def __init__(self, n, obs_dim, device="cpu"):
        import torch
        self.n, self.obs_dim, self.device, self.action_space = n, obs_dim, torch.device(device), self._Box()


def replay_first_update(name):
    """SB3's first PPO update of run `name` through the product's PPO (b747_rl_ctrl_amd/ppo.py, torch path on
    the CPU): the policy at the reconstructed initial weights (actor and critic), the rollout buffer from
    oracle_first_rollout, values and log-probs from that policy, GAE, then PPO.train with SB3 1.4's defaults
    (batch 64, 10 epochs, Adam 3e-4 / eps 1e-5, clip 0.2, max_grad_norm 0.5) and SB3's minibatch order:
    np.random.permutation over the env-major flattening (RolloutBuffer.get / swap_and_flatten), from NumPy's
    global generator as the test callback at call 2000 left it, np.random.seed(0) (env/ctrl_env.py:77).
    -> PPO.train's statistics (SB3's train/* keys)"""
    import torch
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    obs_name = split_run(name)[0]
    od = OBS_DIM[obs_name]
    weights = _replay_generator(name, full=True)[0]
    _, _, buf = oracle_first_rollout(name, record=True)
    ppo = PPO(_HostEnv(4, od), PPOConfig(n_steps=ROLLOUT_STEPS, batch_size=64), fused=False)
    p = ppo.policy
    with torch.no_grad():
        for lin, (w, b) in zip((p.pi_net[0], p.pi_net[2], p.action_net, p.vf_net[0], p.vf_net[2], p.value_net),
                               weights):
            lin.weight.copy_(w)
            lin.bias.copy_(b)
        p.log_std.zero_()
        ppo.obs_buf.copy_(torch.from_numpy(buf["obs"]))
        ppo.act_buf[..., 0].copy_(torch.from_numpy(buf["act"]))
        ppo.rew_buf.copy_(torch.from_numpy(buf["rew"]))
        ppo.done_buf.copy_(torch.from_numpy(buf["done"]))
        ppo.last_obs.copy_(torch.from_numpy(buf["last_obs"]))
        mean, value = p(ppo.obs_buf)
        ppo.val_buf.copy_(value)
        ppo.logp_buf.copy_(p.log_prob(mean, ppo.act_buf))
    ppo.compute_gae(ROLLOUT_STEPS)
    rs = np.random.RandomState(0)

    def sb3_order(epoch, T, n):
        j = rs.permutation(T * n)                 # SB3 flat index j = env * T + t
        return torch.from_numpy((j % T) * n + j // T)
    return ppo.train(ROLLOUT_STEPS, minibatch_order=sb3_order)


def torch_policy(weights):
    """deterministic SB3 predict: mean of the actor, clipped to the [-1, 1] box, float32"""
    import torch
    (w0, b0), (w1, b1), (w2, b2) = weights

    def act(obs):
        with torch.no_grad():
            x = torch.as_tensor(np.asarray(obs, np.float32))
            h = torch.tanh(w1 @ torch.tanh(w0 @ x + b0) + b1)
            return np.float32(np.clip(float((w2 @ h + b2)[0]), -1.0, 1.0))
    return act


def init_policy(seed, obs_dim):
    """A deterministic SB3-default actor at initialisation drawn with numpy (only pi's path matters)."""
    rng = np.random.default_rng(seed)

    def ortho(rows, cols, gain):          # torch.nn.init.orthogonal_: QR of a Gaussian, sign-fixed
        a = rng.standard_normal((max(rows, cols), min(rows, cols)))
        q, r = np.linalg.qr(a)
        q *= np.sign(np.diag(r))
        q = q if rows >= cols else q.T
        return (gain * q[:rows, :cols]).astype(np.float32)
    w1, w2, w3 = ortho(64, obs_dim, math.sqrt(2)), ortho(64, 64, math.sqrt(2)), ortho(1, 64, 0.01)

    def act(obs):
        h = np.tanh(w1 @ obs.astype(np.float32))
        h = np.tanh(w2 @ h)
        return np.float32(np.clip((w3 @ h)[0], -1.0, 1.0))
    return act


def run_test(obs_name, mode_name, policy, sample_time=SAMPLE_TIME, use_rp=True, aero_err=None):
    """ControlTestCallback.calc_stepinfo on the oracle -> (settling_time, overshoot, quality): the means over
    the references (float64, as the callback appends them to its window; TensorBoard stores float32)"""
    mode, amax = MODES[mode_name]
    times, overs, quals = [], [], []
    for vref in REFS:
        ctrl = R.RefController(3, mode, None, None, tk=TK, sample_time=sample_time, action_max=amax)
        if not use_rp:
            ctrl.model.use_RP = 0.0
        env = R.RefControllerEnv(OBS[obs_name], 0, True, True, ctrl)
        t, th = [], []

        def rec(m):
            t.append(m.time)
            th.append(float(np.nan_to_num(m.state[4])) * 180 / math.pi)
        obs = env.reset({"state0": STATE0, "kind": "const", "ref": vref, "aero_err": aero_err})
        done = False
        while not done:
            obs, _, done = env.step(policy(np.asarray(obs, np.float32)), rec)
        info = calc_stepinfo(th, ctrl.vartheta_ref * 180 / math.pi, ts=t)
        times.append(info["settling_time"])
        overs.append(abs(info["overshoot"]))
        quals.append(ctrl.quality())
    return tuple(float(np.mean(v)) for v in (times, overs, quals))


def band(obs_name, mode_name, seeds):
    """(min, max) over `seeds` initial policies of each metric, as arrays [settling, overshoot, quality]"""
    r = np.array([run_test(obs_name, mode_name, init_policy(s, OBS_DIM[obs_name])) for s in range(seeds)],
                 np.float32).astype(np.float64)          # as TensorBoard would store them
    return r.min(0), r.max(0)


def within(value, lo, hi, slack):
    """value in [lo, hi] widened on each side by `slack` x the band width (a finite draw of initial
    policies under-covers the range of all of them)"""
    w = hi - lo
    return lo - slack * w - 1e-12 <= value <= hi + slack * w + 1e-12


def rel_err(got, recorded):
    """per metric |got - recorded| / |recorded|"""
    return [abs(got[j] - recorded[k]) / abs(recorded[k]) for j, k in enumerate(KEYS)]


def f32_equal(got, recorded):
    """per metric: the float32 TensorBoard would store is the recorded one, bit for bit"""
    return [bool(np.float32(got[j]) == np.float32(recorded[k])) for j, k in enumerate(KEYS)]


def main(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    runs = load_fixture()
    lines = ["ControlTestCallback first log point: the reference's DLL runs (tensorboard.xlsx) vs the oracle", "",
             "1. Each run's own initial policy (torch generator history reconstructed, tests/tb_transfer.py):"]
    exact = total = 0
    worst = 0.0
    for name, v in runs.items():
        w = reference_weights(name)
        if w is None:
            lines.append(f"  {name}: first run of the process, generator state unknown (range check only)")
            continue
        got = run_test(*split_run(name), torch_policy(w))
        eq, err = f32_equal(got, v), rel_err(got, v)
        exact += sum(eq)
        total += 3
        worst = max(worst, max(err))
        lines.append(f"  {name}: oracle settling {got[0]:.6f} overshoot {got[1]:.9f} quality {got[2]:.9g} | "
                     f"recorded {v['settling_time']:.6f} {v['overshoot']:.9f} {v['quality']:.9g} | float32-equal "
                     f"{eq} | rel err {max(err):.1e}")
    lines.append(f"  => {exact} of {total} recorded metrics reproduced bit for bit in float32; worst relative "
                 f"error {worst:.1e}")
    lines += ["", f"2. Range over {a.seeds} SB3-style initialisations (numpy draws) and the a = 0 response:"]
    groups = {}
    for name, v in runs.items():
        groups.setdefault(split_run(name), []).append((name, v))
    for (obs_name, mode_name), members in sorted(groups.items()):
        lo, hi = band(obs_name, mode_name, a.seeds)
        zero = run_test(obs_name, mode_name, zero_policy)
        lines.append(f"{obs_name} {mode_name}: oracle a=0 settling {zero[0]:.4f} overshoot {zero[1]:.6f} "
                     f"quality {zero[2]:.7f}")
        lines.append(f"  oracle initial-policy range: settling [{lo[0]:.4f}, {hi[0]:.4f}] overshoot "
                     f"[{lo[1]:.6f}, {hi[1]:.6f}] quality [{lo[2]:.7f}, {hi[2]:.7f}]")
        for name, v in members:
            ins = [bool(within(v[k], lo[j], hi[j], 0.0)) for j, k in enumerate(KEYS)]
            lines.append(f"  recorded {name[len(obs_name) + 8:]}: settling {v['settling_time']:.4f} overshoot "
                         f"{v['overshoot']:.6f} quality {v['quality']:.7f}  inside range: {ins}")
    lines += ["", "3. rollout/ep_rew_mean of the first rollout (20 training episodes, oracle_first_rollout):"]
    exact = 0
    worst = 0.0
    for name, v in runs.items():
        if reference_rollout_noise(name) is None:
            continue
        rets, m = oracle_first_rollout(name)
        eq = bool(np.float32(m) == np.float32(v["ep_rew_mean"]))
        err = abs(m - v["ep_rew_mean"]) / abs(v["ep_rew_mean"])
        exact += eq
        worst = max(worst, err)
        lines.append(f"  {name}: oracle {m:.9g} recorded {v['ep_rew_mean']:.9g} float32-equal {eq} rel err {err:.1e} "
                     f"(episode returns {min(rets):.2f}..{max(rets):.2f})")
    lines.append(f"  => {exact} of 17 reproduced bit for bit in float32; worst relative error {worst:.1e}")
    lines += ["", "4. Sensitivity (PID_LIKE ADD_DIRECT_CONTROL, the reconstructed policy; relative changes):"]
    name = "PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2"
    pol = torch_policy(reference_weights(name))
    base = run_test("PID_LIKE", "ADD_DIRECT_CONTROL", pol)
    for label, kw in (("rate limiter off (use_RP = 0)", {"use_rp": False}),
                      ("controller at the DLL rate (sample_time 0.01)", {"sample_time": 0.01}),
                      ("mz x 1.001 (aero_err[2] = 1e-3)", {"aero_err": [0, 0, 1e-3, 0, 0]}),
                      ("mz x (1 + 1e-5)", {"aero_err": [0, 0, 1e-5, 0, 0]}),
                      ("mz x (1 + 1e-6)", {"aero_err": [0, 0, 1e-6, 0, 0]}),
                      ("CX x (1 + 1e-5)", {"aero_err": [1e-5, 0, 0, 0, 0]}),
                      ("CY x (1 + 1e-5)", {"aero_err": [0, 1e-5, 0, 0, 0]}),
                      ("dCm/ddeltaz x (1 + 1e-5)", {"aero_err": [0, 0, 0, 1e-5, 0]}),
                      ("Kalpha x (1 + 1e-5)", {"aero_err": [0, 0, 0, 0, 1e-5]}),
                      ("main.py's aero_err_test applied", {"aero_err": [-0.1, 0.1, -0.1, -0.1, 0.1]})):
        r = run_test("PID_LIKE", "ADD_DIRECT_CONTROL", pol, **kw)
        d = [(r[j] - base[j]) / base[j] for j in range(3)]
        lines.append(f"  {label}: settling {d[0]:+.1e} overshoot {d[1]:+.1e} quality {d[2]:+.1e}; "
                     f"float32-equal to the record: {f32_equal(r, runs[name])}")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main(sys.argv[1:])
