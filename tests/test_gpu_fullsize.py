"""Oracle-anchored tests of the kernels that produce the bench numbers, at the BASELINE sizes.

  configs[2]  k_env_steps kind 3 (the bench kernel, b747_env_step) on 65,536 envs for 300 steps
              with auto-resets: EVERY env is replayed through the C restatement of the reference's
              env loop (oracle/b747_oracle_env.c, bit-identical to ref_env: tests/test_oracle_env.py),
              and a subset of 128 envs (first and last wave, lanes 0 and 63, and a stride over the
              batch) through the Python restatement itself (oracle/ref_env.py over the DLL-ABI oracle
              library), with the actions and reset draws read back from the device.
  configs[4]  b747_ppo_rollout (k_rollout_split<true> + k_policy_value) on 65,536 envs for 64 steps: every env through the C
              restatement and the same subset through ref_env, driven by the rollout's own (clipped)
              actions; logp / value of every env and step against the fp32 torch ActorCritic.
  configs[3]  524,288 envs (8 x 65,536 per GPU) stepped as ONE batch and as 8 shards with
              env_offset = r * 65,536 on one GPU for 2,100 steps across the tk = 20 s auto-reset:
              X / disc / k / obs / reward / done / terminal obs must be bit-identical (the 8-GPU
              run is these shards on 8 devices; only its timing needs the hardware).
Tolerances as tests/test_gpu_env.py: float32 obs / reward within 2e-6 relative (+1e-7 absolute),
done flags and reset draws exact."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_lib as O  # noqa: E402
import ref_env as R  # noqa: E402

pytestmark = pytest.mark.gpu

RTOL, ATOL = 2e-6, 1e-7
N = 65536


def _subset(n=N):
    """128 envs: lanes 0-15 and 48-63 of the first and of the last wave (first and last workgroup),
    and 64 envs on a stride of 1021 (a prime: every lane position mod 64 appears)."""
    first = list(range(0, 16)) + list(range(48, 64))
    last = [n - 64 + j for j in first]
    mid = [(1021 * k + 64) % n for k in range(64)]
    idx = sorted(set(first + last + mid))
    assert len(idx) == 128 and 0 in idx and 63 in idx and n - 64 in idx and n - 1 in idx
    return np.array(idx)


def _bench_env(n, seed, tk, env_offset=0, sample_time=None, variant="fast"):
    """bench.py's workload (BASELINE configs[2]/[3]): the reference's training configuration."""
    from b747_rl_ctrl_amd import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,
                                  ResetRefMode, RewardType)
    return BatchControllerEnv(n, ObservationType.PID_LIKE, RewardType.CLASSIC, True, True, CtrlType.MANUAL,
                              CtrlMode.DIRECT_CONTROL, reset_ref_mode=ResetRefMode.CONST,
                              disturbance_mode=DisturbanceMode.AERO_DISTURBANCE, tk=tk, sample_time=sample_time,
                              seed=seed, env_offset=env_offset, variant=variant)


def _read_draws(env, idx):
    """The device's Controller.reset draws of envs idx (state0, ref, aero_err), as ref_env dicts."""
    s0 = env.state0[:, idx].cpu().numpy().T
    ref = env.ref[:, idx].cpu().numpy().T.astype(np.float64)
    ae = env.aero_err[:, idx].cpu().numpy().T.astype(np.float64)
    return [{"state0": s0[j], "kind": "const", "ref": float(ref[j, 0]), "h": float(ref[j, 7]), "aero_err": ae[j]}
            for j in range(len(idx))]


def _check_host_draws(draws, idx, seed, episodes):
    """The device draws are the host build's Philox draws for (seed, env id, episode)."""
    for d, i, e in zip(draws, idx, episodes):
        s0, ref, ae, _ = O.draw_resets(seed, int(i), 1, episode=int(e), mode=0, dist_mode=0)
        assert np.array_equal(d["state0"], s0[0]), f"env {i} episode {e}: state0 draw"
        assert d["ref"] == ref[0, 0], f"env {i} episode {e}: ref draw"
        np.testing.assert_allclose(d["aero_err"], ae[0], rtol=1e-14, atol=0,   # device log/cos vs host libm
                                   err_msg=f"env {i} episode {e}: aero_err draw")


def _device_draws(env):
    """Every env's current reset draws in the device layout (state0, ref, ref_kind, aero_err)."""
    return (env.state0.cpu().numpy(), env.ref.cpu().numpy(), env.ref_kind.cpu().numpy(), env.aero_err.cpu().numpy())


def _check_all(full, actions, obs, rew, done, term, env, t):
    """Step the C env restatement of all N envs with the same actions; compare every env's obs (the
    terminal one where an episode ended), reward and done; reset the finished ones with the device's draws."""
    o_ref, r_ref, d_ref = full.step(actions)
    d = done.cpu().numpy()
    assert np.array_equal(d, d_ref), f"step {t}: done differs in {np.flatnonzero(d != d_ref)[:10]}"
    o = np.where(d[:, None], term.cpu().numpy(), obs.cpu().numpy())
    np.testing.assert_allclose(o, o_ref, rtol=RTOL, atol=ATOL, err_msg=f"obs step {t}")
    np.testing.assert_allclose(rew.cpu().numpy(), r_ref.astype(np.float32), rtol=RTOL, atol=ATOL,
                               err_msg=f"reward step {t}")
    if d.any():
        full.reset(*_device_draws(env), mask=d)
    return int(d.sum())


def _ref_envs(draws, tk, sample_time):
    envs = []
    for d in draws:
        c = R.RefController(3, 0, 0, disturbance_mode=0, tk=tk, sample_time=sample_time)
        e = R.RefControllerEnv(0, 0, True, True, c)
        e.reset(d)
        envs.append(e)
    return envs


def test_bench_kernel_65536_envs_300_steps_replayed_through_ref_env():
    from b747_rl_ctrl_amd import _lib
    L = _lib.lib()
    assert L.b747_set_specialization(1) == 1          # the config-specialised kernel (kind 3) is on
    seed, tk = 2024, 1.0                              # 100 env steps per episode: 3 episodes in 300 steps
    env = _bench_env(N, seed, tk)
    idx = _subset()
    ti = torch.from_numpy(idx).cuda()
    draws = _read_draws(env, idx)
    _check_host_draws(draws, idx, seed, [0] * len(idx))
    refs = _ref_envs(draws, tk, None)
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=tk)   # every env, C restatement
    full.reset(*_device_draws(env))
    episodes = np.ones(len(idx), np.int64)
    g = torch.Generator(device="cuda").manual_seed(5)
    n_done = 0
    for t in range(300):
        a = torch.rand(N, device="cuda", generator=g) * 2 - 1
        obs, rew, done, info = env.step(a)
        _check_all(full, a.cpu().numpy(), obs, rew, done, info["terminal_observation"], env, t)
        a_h = a[ti].cpu().numpy()
        o_h, r_h, d_h = obs[ti].cpu().numpy(), rew[ti].cpu().numpy(), done[ti].cpu().numpy()
        term = info["terminal_observation"][ti].cpu().numpy()
        done_j = np.flatnonzero(d_h)
        fresh = _read_draws(env, idx[done_j]) if done_j.size else []
        for j, e in enumerate(refs):
            o_ref, r_ref, d_ref = e.step(a_h[j])
            assert bool(d_h[j]) == d_ref, f"step {t} env {idx[j]}: done {d_h[j]} vs {d_ref}"
            np.testing.assert_allclose(term[j] if d_ref else o_h[j], o_ref.astype(np.float32), rtol=RTOL, atol=ATOL,
                                       err_msg=f"obs step {t} env {idx[j]}")
            np.testing.assert_allclose(r_h[j], np.float32(r_ref), rtol=RTOL, atol=ATOL,
                                       err_msg=f"reward step {t} env {idx[j]}")
        for q, j in enumerate(done_j):
            assert np.all(o_h[j] == 0.0), "auto-reset observation is all zeros"
            _check_host_draws([fresh[q]], [idx[j]], seed, [episodes[j]])
            refs[j].reset(fresh[q])
            episodes[j] += 1
            n_done += 1
    assert n_done == 3 * len(idx)                     # every subset env finished 3 episodes
    assert int(env.episode.min()) == 4 and int(env.episode.max()) == 4   # ... and so did every env


def test_ppo_rollout_kernel_65536_envs_64_steps_replayed_through_ref_env():
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    seed, tk = 3, 0.4                                 # 40-step episodes: one auto-reset per env in 64 steps
    env = _bench_env(N, seed, tk, sample_time=0.01)
    idx = _subset()
    ti = torch.from_numpy(idx).cuda()
    draws = _read_draws(env, idx)
    first_all = _device_draws(env)
    ppo = PPO(env, PPOConfig(n_steps=64, batch_size=N), seed=1, rollout_kernel=True)
    assert ppo.rollout_kernel
    with torch.no_grad():
        for prm in ppo.policy.parameters():               # break the ortho-init symmetry / scale
            prm.add_(0.05 * torch.randn_like(prm))
    ppo.sync_params()
    ppo.collect_rollouts(64)
    torch.cuda.synchronize()
    # the second episode's draws are the host Philox draws of episode 1 (the device keeps them in state0)
    second = _read_draws(env, idx)
    _check_host_draws(second, idx, seed, [1] * len(idx))
    refs = _ref_envs(draws, tk, 0.01)
    # every env: the C env restatement driven by the rollout's own clipped actions
    full = O.EnvOracle(N, 0, 0, 0, flags=O.F_RP, sample_time=0.01, tk=tk)
    full.reset(*first_all)
    o_prev_all = np.zeros((N, 3), np.float32)
    for t in range(64):
        np.testing.assert_allclose(ppo.obs_buf[t].cpu().numpy(), o_prev_all, rtol=RTOL, atol=ATOL,
                                   err_msg=f"obs the policy saw, step {t}")
        a = ppo.act_buf[t, :, 0].clamp(-1, 1).cpu().numpy()
        o_ref, r_ref, d_ref = full.step(a)
        assert np.array_equal(ppo.done_buf[t].cpu().numpy(), d_ref), f"done step {t}"
        np.testing.assert_allclose(ppo.rew_buf[t].cpu().numpy(), r_ref.astype(np.float32), rtol=RTOL, atol=ATOL,
                                   err_msg=f"reward step {t}")
        o_prev_all = np.where(d_ref[:, None], 0.0, o_ref).astype(np.float32)
        if d_ref.any():
            full.reset(*_device_draws(env), mask=d_ref)
    obs_b, act_b = ppo.obs_buf[:, ti].cpu().numpy(), ppo.act_buf[:, ti, 0].cpu().numpy()
    rew_b, done_b = ppo.rew_buf[:, ti].cpu().numpy(), ppo.done_buf[:, ti].cpu().numpy()
    o_prev = np.zeros((len(idx), 3), np.float32)      # reset observation: all zeros
    for t in range(64):
        for j, e in enumerate(refs):
            np.testing.assert_allclose(obs_b[t, j], o_prev[j], rtol=RTOL, atol=ATOL,
                                       err_msg=f"obs the policy saw, step {t} env {idx[j]}")
            a = np.float32(min(max(act_b[t, j], -1.0), 1.0))          # SB3 clips to the action space
            o_ref, r_ref, d_ref = e.step(a)
            assert bool(done_b[t, j]) == d_ref, f"step {t} env {idx[j]}"
            np.testing.assert_allclose(rew_b[t, j], np.float32(r_ref), rtol=RTOL, atol=ATOL,
                                       err_msg=f"reward step {t} env {idx[j]}")
            o_prev[j] = o_ref.astype(np.float32)
            if d_ref:
                e.reset(second[j])
                o_prev[j] = 0.0
    assert int(ppo.done_buf.sum()) == N                # exactly one episode end per env
    # policy outputs of every env and step against the fp32 torch policy (kernel tanh: exp / rcp)
    with torch.no_grad():
        for t in range(0, 64, 7):
            mean, value = ppo.policy(ppo.obs_buf[t])
            lp = ppo.policy.log_prob(mean, ppo.act_buf[t])
            torch.testing.assert_close(value, ppo.val_buf[t], rtol=0, atol=2e-5)
            torch.testing.assert_close(lp, ppo.logp_buf[t], rtol=0, atol=2e-5)
            z = (ppo.act_buf[t, :, 0] - mean[:, 0]) / ppo.policy.log_std.exp()
            assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1) < 0.02   # N(0, 1) noise


def _bits(t):
    """Bit pattern of a tensor: bit-for-bit comparison that also holds for NaN (NaN != NaN)."""
    return t.contiguous().view({8: torch.int64, 4: torch.int32, 2: torch.int16, 1: torch.uint8}[t.element_size()])


def _same_bits(a, b, what):
    if not torch.equal(_bits(a), _bits(b)):
        diff = (_bits(a) != _bits(b))
        raise AssertionError(f"{what}: {int(diff.sum())} elements differ (non-finite: {int((~torch.isfinite(a)).sum())} "
                             f"vs {int((~torch.isfinite(b)).sum())})")


def test_config4_524288_envs_equal_eight_shards_bit_for_bit():
    seed, n, shards = 2024, 8 * N, 8
    full = _bench_env(n, seed, 20)
    parts = [_bench_env(N, seed, 20, env_offset=r * N) for r in range(shards)]
    for r, p in enumerate(parts):
        assert torch.equal(p.state0, full.state0[:, r * N:(r + 1) * N])
    g = torch.Generator(device="cuda").manual_seed(9)
    bad = torch.zeros(4, dtype=torch.int64, device="cuda")
    for t in range(2100):
        a = torch.rand(n, device="cuda", generator=g) * 2 - 1
        o, r_, d, info = full.step(a)
        for r, p in enumerate(parts):
            sl = slice(r * N, (r + 1) * N)
            po, pr, pd, pinfo = p.step(a[sl])
            bad[0] += (_bits(po) != _bits(o[sl])).sum()
            bad[1] += (_bits(pr) != _bits(r_[sl])).sum()
            bad[2] += (pd != d[sl]).sum()
            bad[3] += ((_bits(pinfo["terminal_observation"]) != _bits(info["terminal_observation"][sl])).any(1) & pd).sum()
        if t % 100 == 99 or t == 2000:
            for r, p in enumerate(parts):
                sl = slice(r * N, (r + 1) * N)
                for name in ("X", "disc"):
                    _same_bits(getattr(p, name), getattr(full, name)[:, sl], f"step {t} shard {r} {name}")
                for name in ("k", "mem", "episode", "ep_return"):
                    _same_bits(getattr(p, name), getattr(full, name)[sl], f"step {t} shard {r} {name}")
    assert bad.tolist() == [0, 0, 0, 0], f"obs / reward / done / terminal obs mismatches {bad.tolist()}"
    assert int(full.episode.min()) == 2 and int(full.episode.max()) == 2   # every env crossed the tk = 20 s reset
