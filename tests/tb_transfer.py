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

The policy: SB3 1.4 MlpPolicy defaults (PPO hyperparameters fall back to SB3 defaults, see the fixture
script) -- separate pi / vf MLPs [64, 64] with Tanh, orthogonal init (gain sqrt 2 hidden, 0.01 action head,
zero biases), deterministic action = mean, clipped to the [-1, 1] action box.  The reference's weights are
unknown, so `band` draws many such initialisations and returns the range of the metrics they produce: the
reference's values must lie in it.  a = 0 (`zero_policy`) is the pure PID (ADD_*) / open-loop (DIRECT) case.

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
MODES = {"DIRECT_CONTROL": (0, 17 * math.pi / 180),     # ctrl mode value, action_max (main.py:7-12)
         "ADD_PROC_CONTROL": (1, 1.0),
         "ADD_DIRECT_CONTROL": (3, 10 * math.pi / 180)}


def load_fixture():
    with open(FIXTURE) as f:
        return json.load(f)["runs"]


def split_run(name):
    """'PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2' -> ('PID_LIKE', 'ADD_DIRECT_CONTROL')"""
    obs, rest = name.split("_MANUAL_")
    mode = next(m for m in MODES if rest.startswith(m + "_"))
    return obs, mode


def zero_policy(obs):
    return np.float32(0.0)


def init_policy(seed, obs_dim):
    """A deterministic SB3-default actor at initialisation (only pi's path matters for predict)."""
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
    """ControlTestCallback.calc_stepinfo on the oracle -> (settling_time, overshoot, quality) float32 means"""
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
    return tuple(float(np.float32(np.mean(v))) for v in (times, overs, quals))


def band(obs_name, mode_name, seeds):
    """(min, max) over `seeds` initial policies of each metric, as arrays [settling, overshoot, quality]"""
    r = np.array([run_test(obs_name, mode_name, init_policy(s, len(R.OBS_MAX[OBS[obs_name]])))
                  for s in range(seeds)])
    return r.min(0), r.max(0)


def within(value, lo, hi, slack):
    """value in [lo, hi] widened on each side by `slack` x the band width (a finite draw of initial
    policies under-covers the range of all of them)"""
    w = hi - lo
    return lo - slack * w - 1e-12 <= value <= hi + slack * w + 1e-12


def main(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    runs = load_fixture()
    lines = [f"ControlTestCallback first log point: the reference's DLL runs (tensorboard.xlsx) vs the oracle "
             f"with {a.seeds} SB3-default initial policies and with a = 0", ""]
    groups = {}
    for name, v in runs.items():
        groups.setdefault(split_run(name), []).append((name, v))
    for (obs_name, mode_name), members in sorted(groups.items()):
        lo, hi = band(obs_name, mode_name, a.seeds)
        zero = run_test(obs_name, mode_name, zero_policy)
        lines.append(f"{obs_name} {mode_name}: oracle a=0 settling {zero[0]:.4f} overshoot {zero[1]:.6f} "
                     f"quality {zero[2]:.7f}")
        lines.append(f"  oracle initial-policy band: settling [{lo[0]:.4f}, {hi[0]:.4f}] overshoot "
                     f"[{lo[1]:.6f}, {hi[1]:.6f}] quality [{lo[2]:.7f}, {hi[2]:.7f}]")
        for name, v in members:
            ins = [within(v[k], lo[j], hi[j], 0.0) for j, k in enumerate(("settling_time", "overshoot", "quality"))]
            lines.append(f"  reference {name[len(obs_name) + 8:]}: settling {v['settling_time']:.4f} overshoot "
                         f"{v['overshoot']:.6f} quality {v['quality']:.7f}  inside band: {ins}")
    lines += ["", "Sensitivity of the a = 0 PID_LIKE ADD_DIRECT_CONTROL result to restatement changes:"]
    base = run_test("PID_LIKE", "ADD_DIRECT_CONTROL", zero_policy)
    for label, kw in (("rate limiter off (use_RP = 0)", {"use_rp": False}),
                      ("controller at the DLL rate (sample_time 0.01)", {"sample_time": 0.01}),
                      ("mz x 1.001 (aero_err[2] = 1e-3)", {"aero_err": [0, 0, 1e-3, 0, 0]}),
                      ("CX x 1.001 (aero_err[0] = 1e-3)", {"aero_err": [1e-3, 0, 0, 0, 0]}),
                      ("dCm/ddeltaz x 1.001 (aero_err[3] = 1e-3)", {"aero_err": [0, 0, 0, 1e-3, 0]}),
                      ("main.py's aero_err_test applied", {"aero_err": [-0.1, 0.1, -0.1, -0.1, 0.1]})):
        r = run_test("PID_LIKE", "ADD_DIRECT_CONTROL", zero_policy, **kw)
        lines.append(f"  {label}: settling {r[0]:.4f} ({r[0] - base[0]:+.4f}) overshoot {r[1]:.6f} "
                     f"({(r[1] - base[1]) / base[1]:+.2e} rel) quality {r[2]:.7f} ({(r[2] - base[2]) / base[2]:+.2e} rel)")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main(sys.argv[1:])
