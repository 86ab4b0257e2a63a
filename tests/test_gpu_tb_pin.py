"""The GPU env against the reference DLL's own recorded closed-loop tests (tests/golden/tb_transfer_first_log.json,
see tests/tb_transfer.py and tests/test_tb_transfer_pin.py for the CPU side).

ControlTestCallback (neural/callbacks.py:60-100) runs through b747_rl_ctrl_amd.evaluate.run_step_tests on the
GPU: (1) with a = 0 (the DLL's PID / open-loop response) for every variant, equal to the oracle's a = 0 episodes
(settling time within one DLL sample per reference, overshoot and quality 1e-6 relative) and on the recorded
runs within the initial-policy gate; (2) with 64 SB3-default initial policies (the product's ActorCritic, one per
4-reference block of a 256-env batch) per (obs type, ctrl mode) group: all 18 recorded runs lie inside the range
the GPU produces."""
import math

import numpy as np
import pytest
import torch

import tb_transfer as T

pytestmark = pytest.mark.gpu

KEYS = ("settling_time", "overshoot", "quality")
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
    return np.stack([per(k) for k in KEYS], 1)          # [replicas, 3]


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


@pytest.mark.parametrize("variant", ["fast", "faithful", "mixed"])
def test_pid_response_matches_the_oracle_and_the_recorded_runs(variant):
    runs = T.load_fixture()
    group = ("PID_LIKE", "ADD_DIRECT_CONTROL")
    out = _run(group, lambda o: torch.zeros(o.shape[0], device=o.device), variant=variant)
    mode, amax = T.MODES[group[1]]
    for j, vref in enumerate(T.REFS):         # per reference against the oracle's a = 0 episode
        c = T.R.RefController(3, mode, None, None, tk=T.TK, sample_time=T.SAMPLE_TIME, action_max=amax)
        e = T.R.RefControllerEnv(0, 0, True, True, c)
        t, th = [], []
        e.reset({"state0": T.STATE0, "kind": "const", "ref": vref, "aero_err": None})
        done = False
        while not done:
            _, _, done = e.step(np.float32(0), lambda m: (t.append(m.time), th.append(m.state[4] * 180 / math.pi)))
        info = T.calc_stepinfo(th, vref * 180 / math.pi, ts=t)
        assert abs(float(out["settling_time"][j]) - info["settling_time"]) <= 0.0100001
        assert float(out["overshoot"][j]) == pytest.approx(abs(info["overshoot"]), rel=1e-6)
        assert float(out["quality"][j]) == pytest.approx(c.quality(), rel=1e-6)
    m = _means(out, 1)[0]
    for name, v in runs.items():
        if T.split_run(name) == group:
            assert np.float32(m[0]) == np.float32(v["settling_time"])
            assert abs(m[1] - v["overshoot"]) <= 1e-4 * v["overshoot"], (m, v)    # the a != 0 spread: 6e-5
            assert abs(m[2] - v["quality"]) <= 3e-5 * v["quality"], (m, v)        # 2.5e-5


@pytest.mark.parametrize("group", sorted({T.split_run(n) for n in T.load_fixture()}), ids=lambda g: "-".join(g))
def test_recorded_runs_inside_the_gpu_initial_policy_range(group):
    runs = T.load_fixture()
    od = len(T.R.OBS_MAX[T.OBS[group[0]]])
    out = _run(group, _initial_policies(od), replicas=POLICIES)
    m = _means(out, POLICIES)
    lo, hi = m.min(0), m.max(0)
    for name, v in runs.items():
        if T.split_run(name) == group:
            for j, k in enumerate(KEYS):
                assert T.within(v[k], lo[j], hi[j], 0.25), (name, k, v[k], lo[j], hi[j])
    print(f"\n{group}: GPU initial-policy range settling [{lo[0]:.4f}, {hi[0]:.4f}] overshoot [{lo[1]:.6f}, "
          f"{hi[1]:.6f}] quality [{lo[2]:.7f}, {hi[2]:.7f}]")
