"""Replay of a whole recorded training run of the reference (TEST INFRASTRUCTURE).

tests/tb_transfer.py reproduces the first log point of each training run in tensorboard.xlsx.  This module keeps
going: it replays main.py's PPO training of one run iteration by iteration -- SB3 1.4's learn() loop with the
product's PPO (b747_rl_ctrl_amd/ppo.py, torch path) as the learner -- and compares every log point the reference
recorded (tests/golden/tb_curves.json: rollout/ep_rew_mean, transfer_custom/*, train/*, 62 rows per run).

What is replayed, and from where:
  * the policy's initial weights and every Gaussian action sample: torch's global CPU generator
    (tb_transfer._replay_generator); each ControlTestCallback call (every 1000 vec-env steps,
    neural/callbacks.py:103-106) builds a ControllerEnv -- th.manual_seed(1), env/ctrl_env.py:78 -- and loads a
    model copy (one policy construction) before its test episodes;
  * the minibatch order of every update: np.random.permutation over SB3's env-major flattening from NumPy's
    global generator, which those callbacks re-seed with np.random.seed(0) (env/ctrl_env.py:77) -- every update
    of a run therefore sees the same 10 permutations;
  * the 4 SubprocVecEnv workers' reset draws: Python's random, seeded 1 in each worker (env/ctrl_env.py:76);
  * the envs themselves: the oracle (oracle/ref_env.py) for `backend="oracle"` (CPU), or the product's
    BatchControllerEnv with every episode's draws loaded for `backend="gpu"`;
  * the logging: VecMonitor's float32 episode returns, SB3's ep_info_buffer (last 100 episodes), the callback's
    30-entry windows of test means, PPO.train's train/* statistics of the previous update.

  python tests/tb_training.py [--run NAME] [--iterations 62] [--backend oracle|gpu] [--out FILE]"""
import collections
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import tb_transfer as T  # noqa: E402

CURVES = os.path.join(HERE, "golden", "tb_curves.json")
WINDOW = 30                                            # ControlTestCallback window_length (main.py:147)
EP_BUFFER = 100                                        # SB3 ep_info_buffer maxlen
N_ENVS = 4                                             # neural/agent.py:63 n_cpu


def load_curves(name):
    import json
    with open(CURVES) as f:
        return {tag: dict((s, v) for s, v in rows) for tag, rows in json.load(f)["runs"][name].items()}


class _OracleEnvs:
    """the 4 workers on the oracle"""

    def __init__(self, obs_name, mode, amax, draws):
        R = T.R
        self.envs = [R.RefControllerEnv(T.OBS[obs_name], 0, True, True,
                                        R.RefController(3, mode, None, None, tk=T.TK, sample_time=T.SAMPLE_TIME,
                                                        action_max=amax)) for _ in range(N_ENVS)]
        self.draws = draws

    def reset(self):
        return np.stack([e.reset(next(self.draws[i])) for i, e in enumerate(self.envs)]).astype(np.float32)

    def step(self, act):
        obs, rew, done = [], [], []
        for i, e in enumerate(self.envs):
            o, r, d = e.step(act[i])
            if d:
                o = e.reset(next(self.draws[i]))
            obs.append(o)
            rew.append(r)
            done.append(d)
        return np.stack(obs).astype(np.float32), np.array(rew), np.array(done)


class _GpuEnvs:
    """the 4 workers as one BatchControllerEnv: each episode's draws are loaded at its (synchronous) reset; the
    product PPO's rollout steps it (TrainingReplay._step_iteration_gpu)"""

    def __init__(self, obs_name, mode, amax, draws, variant="fast"):
        import torch
        from b747_rl_ctrl_amd import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, RewardType
        from b747_rl_ctrl_amd._lib import F_PID_CS, F_RP
        self.torch, self.F_PID_CS, self.F_RP = torch, F_PID_CS, F_RP
        # SEMI_MANUAL keeps the altitude-command slot live for HYBRID's CS-PID episodes; the flags are per episode
        self.variant = variant
        self.env = BatchControllerEnv(N_ENVS, ObservationType(T.OBS[obs_name]), RewardType.CLASSIC, True, True,
                                      CtrlType.SEMI_MANUAL, CtrlMode(mode), reset_ref_mode=None, tk=T.TK,
                                      sample_time=T.SAMPLE_TIME, action_max=amax, auto_reset=False, variant=variant)
        self.draws = draws

    def reset(self):
        env, torch = self.env, self.torch
        for j in range(N_ENVS):
            d = next(self.draws[j])
            env.state0[:, j] = torch.as_tensor(d["state0"], dtype=torch.float64)
            env.flags[j] = self.F_RP | (self.F_PID_CS if d.get("hybrid_ctrl") else 0)
            if d["kind"] == "osc":
                env.ref[1:7, j] = torch.as_tensor(d["osc"], dtype=torch.float64)
                env.ref_kind[j] = 1
            else:
                env.ref[0, j] = d["ref"]
                env.ref_kind[j] = 0
            if "h" in d:
                env.ref[7, j] = d["h"]
        return env.reset().cpu().numpy().copy()


def _draw_stream(name):
    """one worker's endless reset draws after its constructor's reset (all workers draw the same)"""
    import random
    rnd = random.Random(1)
    mode = T.reset_mode(name)
    T.reset_draws(rnd, mode)
    while True:
        yield T.reset_draws(rnd, mode)


class TrainingReplay:
    """main.py's training of recorded run `name`, one SB3 iteration (2048 steps x 4 workers + one update) at a
    time; `log` collects what SB3 would have logged at each dump (timestep -> {tag: value})."""

    def __init__(self, name, backend="oracle", variant="fast"):
        import torch
        from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
        assert T.reference_rollout_noise(name) is not None, "the process's first run: generator state unknown"
        self.torch, self.name = torch, name
        self.obs_name, self.mode_name = T.split_run(name)
        mode, amax = T.MODES[self.mode_name]
        self.od = T.OBS_DIM[self.obs_name]
        self._saved_rng = torch.random.get_rng_state()
        torch.manual_seed(1)                                   # the generator history up to this run's policy
        T._sb3_build(T.OBS_DIM[T.previous_obs(name)])
        for _ in range(T.TAIL_SAMPLES):
            torch.empty(4, 1).normal_()
        weights = T._sb3_build(self.od, full=True)
        self.gen = torch.random.get_rng_state()               # the run's own generator, swapped in while it runs
        self.dev = torch.device("cuda" if backend == "gpu" else "cpu")
        self.backend = backend
        draws = [_draw_stream(name) for _ in range(N_ENVS)]
        cfg = PPOConfig(n_steps=T.ROLLOUT_STEPS, batch_size=64)
        if backend == "gpu":
            # the product's rollout path: b747_policy_act (HIP policy, fed the replayed noise) + b747_env_rollout
            self.envs = _GpuEnvs(self.obs_name, mode, amax, draws, variant)
            self.ppo = PPO(self.envs.env, cfg, fused=True, rollout_kernel=False)
        else:
            self.envs = _OracleEnvs(self.obs_name, mode, amax, draws)
            self.ppo = PPO(T._HostEnv(N_ENVS, self.od), cfg, fused=False)
        p = self.ppo.policy
        with torch.no_grad():
            for lin, (w, b) in zip((p.pi_net[0], p.pi_net[2], p.action_net, p.vf_net[0], p.vf_net[2], p.value_net),
                                   weights):
                lin.weight.copy_(w)
                lin.bias.copy_(b)
            p.log_std.zero_()
        self.ppo.sync_params()
        torch.random.set_rng_state(self._saved_rng)           # (PPO's constructor re-seeds the global generator)
        self.obs = self.envs.reset()                           # SB3 _setup_learn's reset
        self.acc = np.zeros(N_ENVS, np.float32)               # VecMonitor episode_returns (float32)
        self.episodes = collections.deque(maxlen=EP_BUFFER)
        self.window = {k: collections.deque(maxlen=WINDOW) for k in T.KEYS}
        self.calls = 0
        self.iteration = 0
        self.train_stats = None
        self.log = {}
        self._test_cache = None

    def _actor(self):
        p = self.ppo.policy
        return [(l.weight.detach().clone(), l.bias.detach().clone())
                for l in (p.pi_net[0], p.pi_net[2], p.action_net)]

    def _callback(self):
        """ControlTestCallback.calc_stepinfo: seeds the generators, builds the model copy, tests the policy"""
        torch = self.torch
        torch.manual_seed(1)
        T._sb3_build(self.od)
        if self._test_cache is None:                          # the policy only changes at updates
            if self.backend == "gpu":
                self._test_cache = self._gpu_test()
            else:
                actor = [(w.cpu(), b.cpu()) for w, b in self._actor()]
                self._test_cache = T.run_test(self.obs_name, self.mode_name, T.torch_policy(actor))
        for k, v in zip(T.KEYS, self._test_cache):
            self.window[k].append(v)

    def _gpu_test(self):
        """the callback's 4 test episodes through evaluate.run_step_tests on the GPU (means over the references)"""
        from b747_rl_ctrl_amd import CtrlMode, ObservationType
        from b747_rl_ctrl_amd.evaluate import run_step_tests
        (w0, b0), (w1, b1), (w2, b2) = self._actor()
        torch = self.torch

        def act(obs):
            h = torch.tanh(torch.tanh(obs @ w0.T + b0) @ w1.T + b1)
            return (h @ w2.T + b2)[:, 0].clamp(-1, 1)
        mode, amax = T.MODES[self.mode_name]
        out = run_step_tests(act, T.REFS, state0=T.STATE0.tolist(), tk=T.TK,
                             observation_type=ObservationType(T.OBS[self.obs_name]), ctrl_mode=CtrlMode(mode),
                             sample_time=T.SAMPLE_TIME, action_max=amax, variant=self.envs.variant)
        return tuple(float(out[k].double().mean()) for k in T.KEYS)

    def step_iteration(self):
        torch = self.torch
        ppo, p = self.ppo, self.ppo.policy
        saved = torch.random.get_rng_state()
        torch.random.set_rng_state(self.gen)
        try:
            if self.backend == "gpu":
                return self._step_iteration_gpu()
            obs_buf = np.zeros((T.ROLLOUT_STEPS, N_ENVS, self.od), np.float32)
            act_buf = np.zeros((T.ROLLOUT_STEPS, N_ENVS), np.float32)
            rew_buf = np.zeros((T.ROLLOUT_STEPS, N_ENVS), np.float32)
            done_buf = np.zeros((T.ROLLOUT_STEPS, N_ENVS), bool)
            std = p.log_std.detach().exp()
            for t in range(T.ROLLOUT_STEPS):
                with torch.no_grad():
                    x = torch.from_numpy(self.obs).to(self.dev)
                    mean = p.action_net(p.pi_net(x))[:, 0]
                    eps = torch.empty(4, 1).normal_()[:, 0].to(self.dev)      # the CPU generator, as SB3 drew it
                    sample = (mean + eps * std).cpu().numpy()
                obs_buf[t], act_buf[t] = self.obs, sample
                self.obs, rew, done = self.envs.step(np.clip(sample, -1, 1))
                rew_buf[t], done_buf[t] = rew, done
                self.acc += rew
                for i in np.flatnonzero(done):
                    self.episodes.append(float(self.acc[i]))
                    self.acc[i] = 0
                self.calls += 1
                if self.calls % T.CALLBACK_INTERVAL == 0:
                    self._callback()
            step, entry = self._dump()
            with torch.no_grad():
                ppo.obs_buf.copy_(torch.from_numpy(obs_buf))
                ppo.act_buf[..., 0].copy_(torch.from_numpy(act_buf))
                ppo.rew_buf.copy_(torch.from_numpy(rew_buf))
                ppo.done_buf.copy_(torch.from_numpy(done_buf))
                ppo.last_obs.copy_(torch.from_numpy(self.obs))
                mean, value = p(ppo.obs_buf)
                ppo.val_buf.copy_(value)
                ppo.logp_buf.copy_(p.log_prob(mean, ppo.act_buf))
            self._update()
        finally:
            self.gen = torch.random.get_rng_state()
            torch.random.set_rng_state(saved)
        return step, entry

    def _dump(self):
        """what SB3's logger writes at the end of the rollout (timestep, {tag: value})"""
        self.iteration += 1
        step = self.iteration * T.ROLLOUT_STEPS * N_ENVS
        entry = {"rollout/ep_rew_mean": float(np.mean(np.asarray(self.episodes, np.float32)))}   # SB3 safe_mean
        entry.update({f"transfer_custom/{k}": float(np.mean(self.window[k])) for k in T.KEYS})
        if self.train_stats is not None:
            entry.update({f"train/{k}": v for k, v in self.train_stats.items()
                          if k not in ("policy_loss", "pg_term_scale", "kl_term_scale")})
            entry["scale/policy_gradient_loss"] = self.train_stats["pg_term_scale"]   # (not SB3 log values)
            entry["scale/approx_kl"] = self.train_stats["kl_term_scale"]
        self.log[step] = entry
        return step, entry

    def _update(self):
        """GAE and PPO.train in SB3's minibatch order (the callbacks' np.random.seed(0))"""
        torch = self.torch
        self.ppo.compute_gae(T.ROLLOUT_STEPS)
        rs = np.random.RandomState(0)

        def sb3_order(epoch, n_steps, n):
            j = rs.permutation(n_steps * n)
            return torch.from_numpy((j % n_steps) * n + j // n_steps)
        self.train_stats = self.ppo.train(T.ROLLOUT_STEPS, minibatch_order=sb3_order)
        self._test_cache = None

    def _step_iteration_gpu(self):
        """the rollout through the product's two-launch path (b747_policy_act with the replayed noise, then
        b747_env_rollout into the PPO buffers), the 400-step episode boundaries reloading the next draws;
        runs with the run's generator swapped in (see step_iteration)"""
        torch, ppo = self.torch, self.ppo
        noise = torch.empty(T.ROLLOUT_STEPS, N_ENVS)
        tests = 0
        for t in range(T.ROLLOUT_STEPS):                  # the generator's draws, callbacks interleaved
            noise[t] = torch.empty(4, 1).normal_()[:, 0]
            if (self.calls + t + 1) % T.CALLBACK_INTERVAL == 0:
                torch.manual_seed(1)
                T._sb3_build(self.od)
                tests += 1
        noise = noise.to(self.dev)
        for t in range(T.ROLLOUT_STEPS):
            ppo._rollout_step_fused(t, noise[t])
            if (self.calls + t + 1) % 400 == 0:          # every worker's episode ends here (tk 20 s, 0.05 s)
                assert bool(ppo.done_buf[t].all()), (self.calls + t + 1)
                # VecMonitor's episode "r": the kernels accumulate it as VecMonitor does (float32 + float64 reward)
                self.episodes.extend(float(r) for r in self.envs.env.ep_final_return.cpu().numpy())
                self.envs.reset()
        self.calls += T.ROLLOUT_STEPS
        ppo._end_rollout(T.ROLLOUT_STEPS)
        for _ in range(tests):                            # the policy is the same for every test of the rollout
            if self._test_cache is None:
                self._test_cache = self._gpu_test()
            for k, v in zip(T.KEYS, self._test_cache):
                self.window[k].append(v)
        step, entry = self._dump()
        self._update()
        return step, entry


def compare(entry, recorded, step):
    """per tag: (ours, recorded, float32-equal, relative error) where the record has the tag at `step`"""
    out = {}
    for tag, v in entry.items():
        if tag in recorded and step in recorded[tag]:
            r = recorded[tag][step]
            out[tag] = (v, r, bool(np.float32(v) == np.float32(r)), abs(v - r) / max(abs(r), 1e-30))
    return out


CANCEL_K = 2.0   # float32 units (1e-7) of the summed terms' magnitude allowed to approx_kl / the policy-gradient loss


def check_entry(entry, recorded, step, tight=1e-5):
    """the early-iteration gates of tests/test_tb_training.py: float32-rounding agreement with the record.
    approx_kl and the policy-gradient loss are means over 81,920 samples of signed O(1) terms (ratio, -1, -log ratio;
    A ratio) that cancel to O(1e-4 - 1e-3): their float32 rounding is set by the terms, not by the result, so they
    are held ABSOLUTELY to CANCEL_K x 1e-7 x the mean magnitude of the summed terms (entry["scale/..."], returned by
    PPO.train); explained variance and clip fraction absolute"""
    cmp_ = compare(entry, recorded, step)
    assert cmp_, step
    for tag, (ours, rec, _, rel) in cmp_.items():
        if tag in ("train/approx_kl", "train/policy_gradient_loss"):
            scale = entry["scale/" + tag.split("/")[1]]
            assert abs(ours - rec) <= CANCEL_K * 1e-7 * scale, (step, tag, ours, rec, abs(ours - rec) / (1e-7 * scale))
        elif tag == "train/explained_variance":
            assert abs(ours - rec) <= 1e-5, (step, tag, ours, rec)
        elif tag == "train/clip_fraction":
            assert abs(ours - rec) <= 1e-4, (step, tag, ours, rec)
        else:
            assert rel <= tight, (step, tag, ours, rec, rel)
    return cmp_


def main(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", default="PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2")
    ap.add_argument("--iterations", type=int, default=62)
    ap.add_argument("--backend", default="oracle", choices=("oracle", "gpu"))
    ap.add_argument("--variant", default="fast")
    ap.add_argument("--out", default=None)
    ap.add_argument("--json", default=None, help="also write every logged entry (timestep -> tag -> value)")
    ap.add_argument("--threads", type=int, default=0, help="torch intra-op threads (0: torch's default)")
    a = ap.parse_args(argv)
    import torch
    if a.threads:
        torch.set_num_threads(a.threads)
    rec = load_curves(a.run)
    rp = TrainingReplay(a.run, a.backend, a.variant)
    lines = [f"training replay of {a.run} ({a.backend}{'/' + a.variant if a.backend == 'gpu' else ''}) against "
             f"tensorboard.xlsx"]
    t0 = time.time()
    exact = total = 0
    for _ in range(a.iterations):
        step, entry = rp.step_iteration()
        cmp_ = compare(entry, rec, step)
        exact += sum(c[2] for c in cmp_.values())
        total += len(cmp_)
        worst = max((c[3] for c in cmp_.values()), default=0.0)
        cells = " ".join(f"{t.split('/')[1]}={'=' if c[2] else f'{c[3]:.0e}'}" for t, c in sorted(cmp_.items()))
        lines.append(f"  step {step:6d}: float32-equal {sum(c[2] for c in cmp_.values())}/{len(cmp_)} worst rel "
                     f"{worst:.1e} | {cells}")
        print(lines[-1], flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write("\n".join(lines) + f"\n  ({time.time() - t0:.0f} s so far)\n")
        if a.json:
            import json
            with open(a.json, "w") as f:
                json.dump({str(k): v for k, v in rp.log.items()}, f)
    lines.append(f"=> {exact} of {total} recorded values float32-equal over {a.iterations} iterations "
                 f"({time.time() - t0:.0f} s)")
    print(lines[-1])
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
