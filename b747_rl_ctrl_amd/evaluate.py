"""Batched step-response evaluation.

The reference evaluates a policy during training with `ControlTestCallback.calc_stepinfo`
(neural/callbacks.py:60-100): for each pitch reference in a list it resets ONE env at a fixed
state0 (MANUAL control, constant reference), runs the deterministic policy to tk with the
Controller's Storage recording every DLL step (core/controller.py:209-228), then computes
`calc_stepinfo` (tools/general.py:46-61) on the recorded pitch and `quality()`
(core/controller.py:334-336).  Here all test episodes run as one batch on the GPU (one env per
reference, optionally replicated) and the step-response metrics are reductions over the
recorded [T, N] pitch history.

Semantics kept from calc_stepinfo(ys, y_base, error_band=0.05, ts):
  overshoot      (max ys if y_base > 0 else min ys) - y_base) / y_base * 100; NaN if y_base == 0
  rise_time      ts[first i < T-1 with (ys[i]-ys[0])/(y_base-ys[0]) >= 1-band] - ts[0]; NaN if none
  settling_time  ts[last i outside the [1-band, 1+band] ratio band] - ts[0]; NaN if none
  static_error   |ys[-1] - y_base|
(None in the reference -> NaN here; the reference raises ZeroDivisionError when y_base == ys[0],
which gives NaN/inf ratios here.)
"""
import math
from typing import Callable, Dict, Optional, Sequence

import torch

from .ctrl_env import BatchControllerEnv, CtrlMode, CtrlType, ObservationType, RewardType


def stepinfo(ys: torch.Tensor, y_base: torch.Tensor, ts: torch.Tensor, error_band: float = 0.05,
             length: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """calc_stepinfo for N step responses at once: ys [T, N], y_base [N], ts [T] or [T, N]; length [N]
    (optional): env j's series is its first length[j] rows (an episode that ended early)."""
    T = ys.shape[0]
    ys = ys.to(torch.float64)
    y_base = torch.as_tensor(y_base, dtype=torch.float64, device=ys.device).expand(ys.shape[1])
    ts = torch.as_tensor(ts, dtype=torch.float64, device=ys.device)
    if ts.dim() == 1:
        ts = ts[:, None].expand_as(ys)
    L = torch.full_like(y_base, T, dtype=torch.int64) if length is None else \
        torch.as_tensor(length, device=ys.device).to(torch.int64).clamp(1, T)
    nan = torch.full_like(y_base, math.nan)
    idx = torch.arange(T, device=ys.device)[:, None].expand_as(ys)
    valid = idx < L
    peak = torch.where(y_base > 0, torch.where(valid, ys, -math.inf).max(0).values,
                       torch.where(valid, ys, math.inf).min(0).values)
    overshoot = torch.where(y_base != 0, (peak - y_base) / y_base * 100, nan)
    ratio = (ys - ys[0]) / (y_base - ys[0])
    risen = (ratio >= 1 - error_band) & (idx < L - 1)
    first = torch.where(risen, idx, T).min(0).values
    rise_time = torch.where(first < T, ts.gather(0, first.clamp(max=T - 1)[None])[0] - ts[0], nan)
    outside = ((ratio <= 1 - error_band) | (ratio >= 1 + error_band)) & valid
    last = torch.where(outside, idx, -1).max(0).values
    settling_time = torch.where(last >= 0, ts.gather(0, last.clamp(min=0)[None])[0] - ts[0], nan)
    y_end = ys.gather(0, (L - 1)[None])[0]
    return {"overshoot": overshoot, "rise_time": rise_time, "settling_time": settling_time,
            "static_error": (y_end - y_base).abs()}


def quality(itse: torch.Tensor, vartheta_ref: torch.Tensor, tk: float) -> torch.Tensor:
    """Controller.quality() (core/controller.py:334-336): exp(-60*0.1*ITSE / (tk * vref^2))."""
    return torch.exp(-60 * 0.1 * itse / (tk * vartheta_ref ** 2))


def run_step_tests(policy: Callable[[torch.Tensor], torch.Tensor], vartheta_ref: Sequence[float],
                   state0: Sequence[float] = (0, 11000, 250, 0, 0, 0), tk: float = 60.0,
                   observation_type: ObservationType = ObservationType.PID_LIKE,
                   reward_type: RewardType = RewardType.CLASSIC, ctrl_mode: Optional[CtrlMode] = CtrlMode.DIRECT_CONTROL,
                   norm_obs: bool = True, norm_act: bool = True, sample_time: Optional[float] = None,
                   replicas: int = 1, device="cuda", **env_kwargs) -> Dict[str, torch.Tensor]:
    """ControlTestCallback.calc_stepinfo for every reference at once.

    policy: deterministic actions [N] from observations [N, obs_dim] (device tensors).
    Returns per-env tensors (N = len(vartheta_ref) * replicas): settling_time, overshoot (abs, as
    the callback takes it), rise_time, static_error, quality, and the callback's means over the
    references ("mean_settling_time", "mean_overshoot", "mean_quality")."""
    refs = torch.tensor(list(vartheta_ref) * replicas, dtype=torch.float64, device=device)
    n = refs.numel()
    env = BatchControllerEnv(n, observation_type, reward_type, norm_obs, norm_act, CtrlType.MANUAL, ctrl_mode,
                             reset_ref_mode=None, tk=tk, sample_time=sample_time, auto_reset=False,
                             device=device, **env_kwargs)
    env.set_state0(torch.tensor(state0, dtype=torch.float64))
    env.set_reference(vartheta=refs)
    env.record_signals(True)
    obs = env.reset()
    steps = int(math.ceil(tk / env.sample_time - 1e-9))
    ns = int(env.cfg.n_sub)
    theta = torch.empty(steps, ns, n, dtype=torch.float64, device=device)
    ts = torch.empty(steps, ns, n, dtype=torch.float64, device=device)
    # the callback steps each episode `while not done` (neural/callbacks.py:77-80): an env that ends early
    # (use_limiter) keeps stepping here with the batch, but its series and ITSE stop at its first done
    ended = torch.zeros(n, dtype=torch.bool, device=device)
    length = torch.full((n,), steps * ns, dtype=torch.int64, device=device)
    itse = torch.zeros(n, dtype=torch.float64, device=device)
    for t in range(steps):
        obs, _, done, _ = env.step(policy(obs))
        theta[t] = torch.nan_to_num(env.signal("state_vartheta"))   # state getter, core/model.py:200
        ts[t] = env.signal("sim_time")
        live = ~ended
        itse = torch.where(live, env.signal("ITSE")[-1], itse)
        length = torch.where(live & done, (t + 1) * ns, length)
        ended = ended | done
    theta, ts = theta.reshape(steps * ns, n), ts.reshape(steps * ns, n)   # one row per DLL step
    # Storage keeps degrees for angles (core/controller.py:219-227); overshoot is unit-free
    # score against the command the dynamics ran with (b747_env_batch.ref, float64 since ABI v7)
    vref = env.ref[0].to(torch.float64)
    info = stepinfo(theta * (180 / math.pi), vref * 180 / math.pi, ts, length=length)   # (x*180)/pi like Storage
    q = quality(itse, vref, tk)
    out = {"settling_time": info["settling_time"], "overshoot": info["overshoot"].abs(),
           "rise_time": info["rise_time"], "static_error": info["static_error"], "quality": q,
           "done": ended.clone(), "length": length}
    out["mean_settling_time"] = out["settling_time"].mean()
    out["mean_overshoot"] = out["overshoot"].mean()
    out["mean_quality"] = q.mean()
    return out
