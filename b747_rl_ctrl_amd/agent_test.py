"""The agent's test flow on the GPU: `ControllerAgent.test`, `_test_env` and `_unwrap_env`
(neural/agent.py:84-86, 230-411) for every reference value at once.

The reference runs, per reference value, one PID-baseline episode per set of PID gains and one
episode per neural controller, each on ONE env with its Controller's Storage recording every DLL
step, then tabulates `stepinfo_SS` / `stepinfo_CS` and `quality()` (core/controller.py:334-358).
Here each (controller, gain set) is one BatchControllerEnv whose envs are the reference values, so
a whole test is a handful of batched episodes:

  pid_baseline_env   the env the reference derives for the baseline (neural/agent.py:303-309):
                     MANUAL -> AUTO, SEMI_MANUAL -> FULL_AUTO, ctrl_mode None, sample_time = dt,
                     Storage on, a fresh model (here: a fresh batch)
  set_pid_coefs      neural/agent.py:296-301: PID_CS when the CS loop is on, else PID_SS (the gains
                     are batch-wide DLL parameters, so each gain set gets its own batch)
  test_episodes      _test_env (neural/agent.py:230-257) for N references: reset at state0, constant
                     pitch (or altitude) command, num_interactions steps, 'rew' recorded one env step
                     late like the reference's _post_step wrapper
  controller_test    ControllerAgent.test: the table rows per reference value and the merged Storage
                     (PID columns, then `<column>__<model name>` for each neural controller), saved
                     as CSV when output_dir is given (xlsx needs openpyxl, absent here)

Policies are callables obs [N, obs_dim] -> action [N] (the deterministic `model.predict`).
"""
import math
import os
from typing import Callable, Dict, List, Optional, Sequence

import torch

from .ctrl_env import BatchControllerEnv, CtrlType
from .evaluate import stepinfo
from .storage import Storage
from .vec_env import B747VecEnv

Policy = Callable[[torch.Tensor], torch.Tensor]
TABLE_COLUMNS = ["Устройство", "σ, [%]", "tпп, [с]", "tв, [с]", "Δ", "Q, [-]"]   # neural/agent.py:322


def unwrap_env(env) -> BatchControllerEnv:
    """Agent._unwrap_env (neural/agent.py:84-86): the environment object behind the VecEnv wrapper."""
    return env.env if isinstance(env, B747VecEnv) else env


def set_pid_coefs(env: BatchControllerEnv, coefs: Sequence[float]) -> BatchControllerEnv:
    """neural/agent.py:296-301: the CS gains when the altitude loop is on, else the SS gains."""
    use_ctrl = env.ctrl_type in (CtrlType.SEMI_MANUAL, CtrlType.FULL_AUTO)
    target = env.consts.PID_CS if use_ctrl else env.consts.PID_SS
    for j in range(4):
        target[j] = float(coefs[j])
    return env


def pid_baseline_env(n: int, env_kwargs: dict, device="cuda") -> BatchControllerEnv:
    """The PID baseline the reference derives from the first env (neural/agent.py:303-309)."""
    kw = dict(env_kwargs)
    ct = kw.pop("ctrl_type")
    kw.pop("ctrl_mode", None)
    kw.update(reset_ref_mode=None, sample_time=None, auto_reset=False)
    ctrl_type = CtrlType.AUTO if ct == CtrlType.MANUAL else CtrlType.FULL_AUTO
    env = BatchControllerEnv(n, kw.pop("observation_type"), kw.pop("reward_type"), kw.pop("norm_obs"),
                             kw.pop("norm_act"), ctrl_type, None, device=device, **kw)
    env.use_storage = True
    return env


def test_episodes(env: BatchControllerEnv, ref_values: Sequence[float], state0: Optional[Sequence[float]],
                  num_interactions: int, policy: Optional[Policy] = None) -> BatchControllerEnv:
    """_test_env for env i = ref_values[i]: reset at state0, hold the command, step num_interactions
    times (policy None: the PID flies, action None)."""
    refs = torch.as_tensor(list(ref_values), dtype=torch.float64, device=env.device)
    assert refs.numel() == env.n
    use_ctrl = env.ctrl_type in (CtrlType.SEMI_MANUAL, CtrlType.FULL_AUTO)
    env.use_storage = True
    env.storage.clear_all()
    if state0 is not None:
        env.set_state0(torch.as_tensor(state0, dtype=torch.float64))
    if use_ctrl:                                  # env.ctrl.h_func = lambda _: ref_value
        env.set_reference(h=refs)
    else:                                         # env.ctrl.vartheta_func = lambda _: ref_value
        env.set_reference(vartheta=refs)
    obs = env.reset()
    rew = torch.full((env.n,), math.nan, dtype=torch.float64, device=env.device)   # `rew = None` at first
    for _ in range(num_interactions):
        action = None if policy is None else policy(obs)
        obs, r, _, _ = env.step(action)
        env.storage.record("rew", rew)            # the wrapper records the previous step's reward
        rew = r.to(torch.float64)
    return env


def episode_info(env: BatchControllerEnv) -> Dict[str, torch.Tensor]:
    """stepinfo_SS / stepinfo_CS and quality() of every env after test_episodes
    (core/controller.py:334-358): calc_stepinfo over the recorded DLL steps."""
    cols = env.storage.columns()
    use_ctrl = env.ctrl_type in (CtrlType.SEMI_MANUAL, CtrlType.FULL_AUTO)
    if use_ctrl:
        info = stepinfo(cols["y"], cols["hzh"][-1], cols["t"])
    else:
        info = stepinfo(cols["vartheta"], cols["vartheta_ref"][-1], cols["t"])
    from .model import SIG
    itse = env.sig[-1, SIG["ITSE"]]
    # Controller.vartheta_ref in radians: the CS PID's output signal, or the pitch command parameter
    vref = torch.where((env.flags & 2).bool(), env.sig[-1, SIG["vartheta_zh"]], env.rec_params[0])
    info["quality"] = torch.exp(-60 * 0.1 * itse / (env.tk * vref ** 2))
    return info


def _row(name, info, j, unit):
    g = lambda k: float(info[k][j])
    return {"Устройство": name, "σ, [%]": g("overshoot"), "tпп, [с]": g("settling_time"), "tв, [с]": g("rise_time"),
            f"Δ, {unit}": g("static_error"), "Q, [-]": g("quality")}


def controller_test(ref_values: Sequence[float], env_kwargs: Dict[str, dict], policies: Dict[str, Policy],
                    state0: Optional[Sequence[float]] = None, pid_coefs: Sequence[Sequence[float]] = (),
                    no_neural: bool = False, output_dir: Optional[str] = None, device="cuda"):
    """ControllerAgent.test (neural/agent.py:259-411).  env_kwargs: model name -> BatchControllerEnv
    keyword arguments (observation_type, reward_type, norm_obs, norm_act, ctrl_type, ctrl_mode, tk, ...);
    policies: model name -> deterministic policy.  Returns (rows per reference value, Storage per
    reference value); with output_dir, writes the reference's files: data_<ref>.xlsx (the Storage, with charts,
    and its _big copy), data_<ref>_info.xlsx and data_<kind>_info_mean.xlsx."""
    n = len(ref_values)
    first = next(iter(env_kwargs.values()))
    env_pid = pid_baseline_env(n, first, device=device)
    use_ctrl = env_pid.ctrl_type == CtrlType.FULL_AUTO
    unit = "[м]" if use_ctrl else "[град]"
    base = "CУ ПИД" if use_ctrl else "СС ПИД"                 # neural/agent.py:315
    if len(pid_coefs) == 0:
        pid_coefs = [list(env_pid.consts.PID_CS if use_ctrl else env_pid.consts.PID_SS)]
    names = lambda i: f"{base}{f' [{i + 1}]' if len(pid_coefs) > 1 else ''}"
    rows: List[List[dict]] = [[] for _ in range(n)]
    stores: List[Optional[Storage]] = [None] * n
    num_pid = int(env_pid.tk / env_pid.dt)
    for i, coefs in enumerate(pid_coefs):
        e = env_pid if i == 0 else pid_baseline_env(n, first, device=device)
        set_pid_coefs(e, coefs)
        test_episodes(e, ref_values, state0, num_pid)
        info = episode_info(e)
        for j in range(n):
            s = e.storage.storage(j)
            if stores[j] is None:
                stores[j] = s
                if len(pid_coefs) > 1:
                    stores[j].set_suffix(names(i))
            else:
                stores[j].merge(s, names(i))
            rows[j].append(_row(names(i), info, j, unit))
    if not no_neural:
        for name, kw in env_kwargs.items():
            kw = dict(kw)
            e = BatchControllerEnv(n, kw.pop("observation_type"), kw.pop("reward_type"), kw.pop("norm_obs"),
                                   kw.pop("norm_act"), kw.pop("ctrl_type"), kw.pop("ctrl_mode"),
                                   **{**kw, "reset_ref_mode": None, "auto_reset": False}, device=device)
            test_episodes(e, ref_values, state0, int(e.tk / e.sample_time), policies[name])
            info = episode_info(e)
            for j in range(n):
                stores[j].merge(e.storage.storage(j), name)
                rows[j].append(_row(name, info, j, unit))
    if output_dir:
        # neural/agent.py:393-408: per reference data_<tag>.xlsx (Storage.save with its charts, + _big copy) and
        # data_<tag>_info.xlsx, then data_<kind>_info_mean.xlsx (b747_rl_ctrl_amd.xlsx writes the workbooks)
        import pandas as pd
        from .xlsx import write_frame
        os.makedirs(output_dir, exist_ok=True)
        kind = "h" if use_ctrl else "vartheta"
        tables = []
        for j, ref in enumerate(ref_values):
            tag = f"h_{ref}" if use_ctrl else f"vartheta_{ref * 180 / math.pi}"
            df = pd.DataFrame(rows[j]).set_index("Устройство")
            write_frame(os.path.join(output_dir, f"data_{tag}_info.xlsx"), df)
            tables.append(df)
            stores[j].save(os.path.join(output_dir, f"data_{tag}.xlsx"), base="t")
        allt = pd.concat(tables)
        allt["σ, [%]"] = allt["σ, [%]"].abs()
        write_frame(os.path.join(output_dir, f"data_{kind}_info_mean.xlsx"), allt.groupby(allt.index).mean())
    return rows, stores
