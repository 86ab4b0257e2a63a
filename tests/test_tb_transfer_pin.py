"""Trajectory-level pin of the oracle to the reference DLL's own recorded output (CPU).

The reference ships no test vectors and its DLL may not be executed here, but its
tensorboard.xlsx records what ControlTestCallback measured on the DLL: 18 training runs' closed-loop
step-response tests (4 episodes of 2,000 DLL steps each; settling time, overshoot, quality), the first of them
taken with the PPO policy at its initial weights (tests/golden/make_tb_fixture.py).  tests/tb_transfer.py
reconstructs those weights from torch's generator history for 17 of the runs and reruns the callback on the
oracle.

Gates: the 45 metrics of the 15 closed-loop and PID_LIKE open-loop runs are the recorded float32 values bit for
bit; the two SPEED_MODE open-loop (DIRECT) runs' settling time and overshoot too, and their quality within 1e-6
relative (measured 2.2e-7 / 4.9e-7: exp(-6 ITSE / (tk vref^2)) of an uncontrolled 2,000-step divergence carries
the libm differences between the reference's Windows CRT and glibc); the first run of the reference's process
(its generator state is not recoverable) lies inside the range of 8 SB3-style initialisations.  The gate has
teeth: the pitching moment scaled by 1 + 1e-5 already moves the reproduced quality off the record.

The same rows' rollout/ep_rew_mean -- 20 stochastic training episodes of the train env per run, random resets
from Python's generator, the CLASSIC reward, the initial actor plus replayed Gaussian noise -- is reproduced
within 1e-6 relative, 16 of the 17 bit for bit in float32 (each run's first rollout is its own trajectory; the
step-response records of the 17 runs hold only 7 distinct trajectories, since a process's later runs start from its
first run's seeded policy).  Full report: profiles/r05/tb_transfer_pin.txt."""
import numpy as np
import pytest

import tb_transfer as T


@pytest.fixture(scope="module")
def runs():
    return T.load_fixture()


def _unique_reproducible(runs):
    """one run per distinct (obs, ctrl mode, previous obs) -- the others are the same computation"""
    seen, out = set(), []
    for name in sorted(runs):
        if (T.split_run(name) + (T.reset_mode(name),)) == T.FIRST_RUN:
            continue
        key = T.split_run(name) + (T.previous_obs(name),)
        if key not in seen:
            seen.add(key)
            out.append(name)
    return out


def _group(runs, name):
    key = T.split_run(name) + (T.previous_obs(name),)
    return [n for n in runs if (T.split_run(n) + (T.reset_mode(n),)) != T.FIRST_RUN
            and T.split_run(n) + (T.previous_obs(n),) == key]


def test_fixture_is_the_first_log_point_of_all_18_runs(runs):
    assert len(runs) == 18
    groups = {}
    for name, v in runs.items():
        assert v["step"] == 8192 and v["ep_len_mean"] == 400.0
        groups.setdefault(T.split_run(name), []).append(name)
    assert sorted(len(m) for m in groups.values()) == [3] * 6       # 2 obs types x 3 ctrl modes x 3 reset modes


def test_reconstructed_weights_are_deterministic_and_leave_the_generator_alone():
    import torch
    torch.manual_seed(123)
    before = torch.random.get_rng_state()
    a = T.reference_weights("PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2")
    b = T.reference_weights("PID_LIKE_MANUAL_ADD_PROC_CONTROL_HYBRID_None_1")
    assert torch.equal(torch.random.get_rng_state(), before)
    assert all(torch.equal(x, y) for (x, _), (y, _) in zip(a, b))
    c = T.reference_weights("SPEED_MODE_MANUAL_DIRECT_CONTROL_CONST_None_1")     # previous run PID_LIKE
    d = T.reference_weights("SPEED_MODE_MANUAL_DIRECT_CONTROL_HYBRID_None_1")
    assert c[0][0].shape == (64, 5) and not torch.equal(c[0][0], d[0][0])
    assert T.reference_weights("PID_LIKE_MANUAL_DIRECT_CONTROL_CONST_None_2") is None


@pytest.mark.parametrize("name", _unique_reproducible(T.load_fixture()))
def test_oracle_reproduces_the_recorded_run(runs, name):
    got = T.run_test(*T.split_run(name), T.torch_policy(T.reference_weights(name)))
    open_loop_speed = T.split_run(name) == ("SPEED_MODE", "DIRECT_CONTROL")
    for member in _group(runs, name):
        eq, err = T.f32_equal(got, runs[member]), T.rel_err(got, runs[member])
        if open_loop_speed:
            assert eq[:2] == [True, True] and err[2] <= 1e-6, (member, got, runs[member], err)
        else:
            assert eq == [True, True, True], (member, got, runs[member], err)


def test_first_run_inside_the_initial_policy_range(runs):
    lo, hi = T.band("PID_LIKE", "DIRECT_CONTROL", 8)
    v = runs["PID_LIKE_MANUAL_DIRECT_CONTROL_CONST_None_2"]
    for j, k in enumerate(T.KEYS):
        assert T.within(v[k], lo[j], hi[j], 0.5), (k, v[k], lo[j], hi[j])


def test_a_1e5_pitching_moment_error_fails_the_pin(runs):
    name = "PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2"
    off = T.run_test("PID_LIKE", "ADD_DIRECT_CONTROL", T.torch_policy(T.reference_weights(name)),
                     aero_err=[0, 0, 1e-5, 0, 0])
    assert not all(T.f32_equal(off, runs[name]))
    assert max(T.rel_err(off, runs[name])) > 5e-7


def _reproducible_names():
    return [n for n in sorted(T.load_fixture()) if (T.split_run(n) + (T.reset_mode(n),)) != T.FIRST_RUN]


def test_worker_draws_follow_pythons_generator_seeded_1():
    import math
    import random
    rnd = random.Random(1)
    first = [rnd.uniform(1000, 11000) for _ in range(1)]
    d = T.worker_draws("PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2", episodes=2)
    assert d[0]["state0"][1] != first[0]            # the constructor's reset consumed the first draw set
    assert all(1000 <= x["state0"][1] <= 11000 and 1 * math.pi / 180 <= abs(x["ref"]) <= 10 * math.pi / 180
               for x in d)
    h = T.worker_draws("PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_HYBRID_None_1", episodes=6)
    assert {x["hybrid_ctrl"] for x in h} == {True, False}


def test_oracle_reproduces_the_recorded_first_rollouts(runs):
    """rollout/ep_rew_mean: 20 stochastic training episodes per run (reset draws, CLASSIC reward, action noise);
    with SB3 1.4's own float32 semantics (VecMonitor, safe_mean) 16 of 17 float32-equal, the last within 5.5e-7
    (libm last bits)"""
    exact = 0
    for name in _reproducible_names():
        rets, m = T.oracle_first_rollout(name)
        v = runs[name]["ep_rew_mean"]
        assert len(rets) == 20
        assert abs(m - v) <= 1e-6 * abs(v), (name, m, v)
        exact += bool(np.float32(m) == np.float32(v))
    assert exact >= 16   # VecMonitor's float32(return + float64 reward) and SB3's float32 mean (round 4's float32 sums: 13)
