"""BatchControllerEnv -- N copies of the reference's `env.ctrl_env.ControllerEnv`, one launch per step.

Mirrors env/ctrl_env.py:61-282 (ControllerEnv) and core/controller.py:43-360 (Controller):
same enums and values, same constructor arguments, same observation layouts / normalisation,
reward functions, action modes, sub-stepping (round(sample_time/dt) DLL steps per env step),
done logic and random resets.  `step()` is one fused HIP kernel (b747_env_step) per env step;
obs / reward / done stay on the GPU as torch tensors.  With auto_reset=True (default) it
behaves like an SB3 VecEnv: finished envs are reset inside the same launch, `obs` holds the reset
observation and `info["terminal_observation"]` the last one of the finished episode.

No CPU fallback: without libb747.so or a ROCm GPU the constructor raises.
"""
import ctypes
import math
from enum import Enum
from typing import Optional

import torch

from . import _lib
from ._lib import F_PID_CS, F_PID_SS, F_RP, NAERO, NDISC, NX


class ObservationType(Enum):   # env/ctrl_env.py:16-22
    PID_LIKE = 0
    SPEED_MODE = 1
    PID_AERO = 2
    PID_SPEED_AERO = 3
    MODEL_STATE = 4


class RewardType(Enum):        # env/ctrl_env.py:24-30
    CLASSIC = 0
    PID_LIKE = 1
    QUALITY = 2
    MINIMAL = 3
    TF_REFERENCE = 4


class CtrlType(Enum):          # core/controller.py:14-19
    FULL_AUTO = 0
    AUTO = 1
    SEMI_MANUAL = 2
    MANUAL = 3


class CtrlMode(Enum):          # core/controller.py:21-26
    DIRECT_CONTROL = 0
    ADD_PROC_CONTROL = 1
    ANG_VEL_CONTROL = 2
    ADD_DIRECT_CONTROL = 3


class ResetRefMode(Enum):      # core/controller.py:28-32
    CONST = 0
    OSCILLATING = 1
    HYBRID = 2


class DisturbanceMode(Enum):   # core/controller.py:34-36
    AERO_DISTURBANCE = 0


OBS_MAX = {  # env/ctrl_env.py:200-214
    ObservationType.PID_LIKE: [60 * math.pi, math.pi, math.pi],
    ObservationType.SPEED_MODE: [60 * math.pi, math.pi, math.pi, 500, 100],
    ObservationType.PID_SPEED_AERO: [60 * math.pi, math.pi, math.pi, 500, 100, 0.5, 2, 0.6, 0.05, 1.0],
    ObservationType.PID_AERO: [60 * math.pi, math.pi, math.pi, 0.5, 2, 0.6, 0.05, 1.0],
    ObservationType.MODEL_STATE: [10 * math.pi / 180, 12000, 15000, 500, 100, math.pi, math.pi],
}


def _calc_exp_k(rk: float, xk: float) -> float:  # tools/general.py:32-33
    return -math.log(rk) / xk


class Box:
    """Minimal gym.spaces.Box stand-in (gym is not a dependency of the hot path)."""

    def __init__(self, low, high, shape, dtype="float32"):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


class BatchControllerEnv:
    """Vectorised ControllerEnv on one MI355X.  Constructor = ControllerEnv(observation_type,
    reward_type, norm_obs, norm_act, *Controller args) with `n` envs in front and device options
    at the end."""

    def __init__(self, n: int, observation_type: ObservationType, reward_type: RewardType, norm_obs: bool,
                 norm_act: bool, ctrl_type: CtrlType, ctrl_mode: Optional[CtrlMode],
                 reset_ref_mode: Optional[ResetRefMode] = None, disturbance_mode: Optional[DisturbanceMode] = None,
                 tk: float = 60, sample_time: Optional[float] = None, action_max: float = 17 * math.pi / 180,
                 vartheta_max: float = 10 * math.pi / 180, use_limiter: bool = False, aero_err=None,
                 reward_config: Optional[dict] = None, seed: int = 0, device="cuda", x_f64: bool = True,
                 auto_reset: bool = True, env_offset: int = 0, state0=None, variant: str = "fast"):
        if not torch.cuda.is_available():
            raise _lib.B747Error("BatchControllerEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        assert ctrl_mode is not None or ctrl_type in (CtrlType.AUTO, CtrlType.FULL_AUTO), \
            "ctrl_mode may be None only when the SS PID is in the loop (core/controller.py:104)"
        if reset_ref_mode is not None:
            assert ctrl_type in (CtrlType.SEMI_MANUAL, CtrlType.MANUAL), \
                "random resets need the neural SS controller in the loop (core/controller.py:145)"
        self._L = _lib.lib()
        assert variant in ("fast", "faithful", "mixed")
        self.variant = {"fast": _lib.VARIANT_FAST, "faithful": _lib.VARIANT_FAITHFUL, "mixed": _lib.VARIANT_MIXED}[variant]
        self.n, self.device = int(n), _lib.resolve_device(device)
        self.observation_type, self.reward_type = observation_type, reward_type
        self.norm_obs, self.norm_act = bool(norm_obs), bool(norm_act)
        self.ctrl_type, self.ctrl_mode = ctrl_type, ctrl_mode
        self.reset_ref_mode, self.disturbance_mode = reset_ref_mode, disturbance_mode
        self.dt = 0.01
        self.sample_time = sample_time if sample_time else self.dt
        assert self.sample_time >= self.dt, "sample_time must be >= dt (core/controller.py:111)"
        self.tk, self.action_max, self.vartheta_max = float(tk), float(action_max), float(vartheta_max)
        self.use_limiter = bool(use_limiter)
        self.obs_dim = int(self._L.b747_env_obs_dim(observation_type.value))

        cfg = _lib.EnvConfig()
        _lib.check(self._L.b747_env_config_default(ctypes.byref(cfg), observation_type.value, reward_type.value),
                   "b747_env_config_default")
        cfg.ctrl_type = ctrl_type.value
        cfg.ctrl_mode = -1 if ctrl_mode is None else ctrl_mode.value
        cfg.reset_ref_mode = -1 if reset_ref_mode is None else reset_ref_mode.value
        cfg.disturbance_mode = -1 if disturbance_mode is None else disturbance_mode.value
        cfg.norm_obs, cfg.norm_act, cfg.use_limiter = int(self.norm_obs), int(self.norm_act), int(self.use_limiter)
        cfg.auto_reset = int(auto_reset)
        cfg.sample_time = self.sample_time
        cfg.n_sub = int(round(self.sample_time / self.dt))
        cfg.tk, cfg.action_max, cfg.vartheta_max = self.tk, self.action_max, self.vartheta_max
        if aero_err is not None:
            cfg.aero_fixed = 1
            for j in range(NAERO):
                cfg.aero_err_fixed[j] = float(aero_err[j])
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.cfg = cfg
        if reward_config:
            self.set_rew_config(reward_config)
        self.consts = _lib.default_consts()

        dev, f64, f32 = self.device, torch.float64, torch.float32
        z = lambda *shape, dt=f64: torch.zeros(*shape, dtype=dt, device=dev)
        self.X = z(NX, n, dt=f64 if x_f64 else f32)
        self.x_f64 = bool(x_f64)
        self.disc, self.k, self.mem = z(NDISC, n), z(n, dt=torch.int32), z(n, dt=torch.uint8)
        self.deltaz, self.vartheta, self.upid, self.tp = z(n), z(n), z(n), z(n)
        self.h_zh = torch.full((n,), 11000.0, dtype=f64, device=dev)
        use_ctrl = ctrl_type in (CtrlType.SEMI_MANUAL, CtrlType.FULL_AUTO)       # core/controller.py:129-131
        manual_stab = ctrl_type in (CtrlType.MANUAL, CtrlType.SEMI_MANUAL)
        fl = F_RP | (F_PID_CS if use_ctrl else 0) | (0 if manual_stab else F_PID_SS)
        self.flags = torch.full((n,), fl, dtype=torch.uint8, device=dev)
        self.aero_err = z(NAERO, n, dt=f64)       # the DLL's double aero_err[5]; float64 draws (ABI v7)
        self.ref = z(8, n, dt=f64)                # the reference's Python-float references
        self.ref_kind = z(n, dt=torch.uint8)
        s0 = torch.tensor([0.0, 11000.0, 259.1667, 0.0, 0.0, 0.0], dtype=f64, device=dev)   # DLL default state0
        self.state0 = s0[:, None].repeat(1, n).contiguous()
        if state0 is not None:
            self.set_state0(state0)
        self.episode = z(n, dt=torch.int32)
        self.ep_return, self.ep_len = z(n, dt=torch.float32), z(n, dt=torch.int32)   # (float32-valued: VecMonitor)
        self.ep_final_return, self.ep_final_len = z(n), z(n, dt=torch.int32)
        self.action = z(n, dt=f32)
        self.obs, self.reward = z(n, self.obs_dim, dt=f32), z(n, dt=f32)
        self.done = z(n, dt=torch.bool)   # the kernel writes 0/1 bytes (torch.bool storage)
        self.terminal_obs = z(n, self.obs_dim, dt=f32)
        self.sig = None                     # [n_sub, 31, N] f64 model signals, see record_signals()
        self.rec_params = None              # [3, N] f64 vartheta / h_zh / deltaz of the last step (recording)
        self.ep_stats = None                # [3, N] f64 episode accumulators, see track_episodes()
        self.storage = None                 # BatchStorage while use_storage is on (Controller.storage)
        self._use_storage = False
        self.env_offset = int(env_offset)

        if self.norm_act:
            self.action_space = Box(-1.0, 1.0, (1,))
        else:
            self.action_space = Box(-self.action_max, self.action_max, (1,))
        om = OBS_MAX[observation_type]
        self.observation_space = Box(-1.0, 1.0, (self.obs_dim,)) if self.norm_obs else \
            Box([-v for v in om], om, (self.obs_dim,))
        self.reset()

    # ------------------------------------------------------------------ plumbing --
    def _batch(self) -> _lib.EnvBatch:
        """The C-ABI descriptor; buffers never move, so it is built once and cached."""
        b = getattr(self, "_b", None)
        if b is None:
            b = _lib.EnvBatch()
            b.n, b.env_offset, b.x_f64, b.obs_dim = self.n, self.env_offset, int(self.x_f64), self.obs_dim
            b.variant = self.variant
            for f in _lib._ENV_PTRS:
                t = getattr(self, f)
                setattr(b, f, t.data_ptr() if t is not None else None)
            self._b = b
            self._bref = ctypes.byref(b)
            self._cref, self._kref = ctypes.byref(self.cfg), ctypes.byref(self.consts)
        return b

    def record_signals(self, on: bool = True):
        """Make every step also write the 31 exported model signals after each of its DLL steps
        to `self.sig` [n_sub, 31, N] (rows in model.SIG order) -- what Controller._post_step
        records into its Storage (core/controller.py:209-228); off again with on=False."""
        n_sub = int(self.cfg.n_sub)
        self.sig = torch.zeros(n_sub, _lib.NSIG, self.n, dtype=torch.float64, device=self.device) if on else None
        self.rec_params = torch.zeros(3, self.n, dtype=torch.float64, device=self.device) if on else None
        self._b = None                      # rebuild the cached C descriptor

    def track_episodes(self, on: bool = True):
        """Make the step kernel add every finished episode to per-env device accumulators
        `self.ep_stats` [3, N] (count, return sum, length sum; b747_env_batch.ep_stats) -- the
        statistics SB3's VecMonitor logs, without a host copy per step.  episode_stats.EpisodeStats
        reduces them across envs and ranks."""
        self.ep_stats = torch.zeros(3, self.n, dtype=torch.float64, device=self.device) if on else None
        self._b = None                      # rebuild the cached C descriptor

    @property
    def use_storage(self) -> bool:
        """Controller.use_storage (core/controller.py:120-122, 209-228): while on, every step appends the
        Storage columns of each of its DLL steps to `self.storage` (a storage.BatchStorage, kept on the
        device; `self.storage.storage(i)` is env i's reference Storage)."""
        return self._use_storage

    @use_storage.setter
    def use_storage(self, on: bool):
        from .storage import BatchStorage
        on = bool(on)
        if on and self.storage is None:
            self.storage = BatchStorage(self)
        if on != (self.sig is not None):
            self.record_signals(on)
        self._use_storage = on

    def signal(self, name: str) -> torch.Tensor:
        """One recorded signal [n_sub, N] (every DLL step of the last env step) by its model.SIG
        name; [-1] is the value after the env step (record_signals must be on)."""
        from .model import SIG
        assert self.sig is not None, "record_signals() is off"
        return self.sig[:, SIG[name]]

    def set_rew_config(self, rew_config: dict):
        """env/ctrl_env.py:250-252 -- reward constants (reward_config keys of :109-192)."""
        c = self.cfg
        if self.reward_type == RewardType.CLASSIC:
            k1, k2, k3 = rew_config.get("k1", 2), rew_config.get("k2", 2), rew_config.get("k3", 1)
            s = k1 + k2 + k3
            vals = [k1 / s, k2 / s, k3 / s, rew_config.get("kf", 0.1), rew_config.get("kITSE", 0.3),
                    rew_config.get("k0", 2), _calc_exp_k(0.8, 10), _calc_exp_k(0.75, 0.15)]
        elif self.reward_type == RewardType.PID_LIKE:
            vals = [rew_config.get("k", 10)]
        elif self.reward_type == RewardType.MINIMAL:
            vals = [rew_config.get("rmax", 0.2), rew_config.get("k1", 2), rew_config.get("k2", 0.5)]
        elif self.reward_type == RewardType.TF_REFERENCE:
            vals = [rew_config.get("overshoot_ref", 2), rew_config.get("tp_ref", 5), rew_config.get("k", 0.1)]
        else:
            vals = []
        for j, v in enumerate(vals):
            c.rew[j] = float(v)

    def set_state0(self, state0):
        """Per-env (or shared) initial state used by resets when reset_ref_mode is None."""
        v = torch.as_tensor(state0, dtype=torch.float64, device=self.device)
        v = v.expand(self.n, 6) if v.dim() == 1 else v
        self.state0.copy_(v.T)

    def set_reference(self, vartheta=None, oscillating=None, h=None):
        """Per-env reference functions for reset_ref_mode None (Controller.vartheta_func/h_func):
        vartheta: constant pitch [N] or scalar; oscillating: [N, 6] (A1, A2, A3, f1, f2, f3);
        h: altitude command for the CS-PID control types."""
        if vartheta is not None:
            self.ref[0].copy_(torch.as_tensor(vartheta, dtype=torch.float64, device=self.device).expand(self.n))
            self.ref_kind.fill_(0)
        if oscillating is not None:
            # a random reset mode owns the reference: CONST / HYBRID steps read ref[0] only, OSCILLATING
            # resets redraw the waves (core/controller.py:148-179 replace vartheta_func on every reset)
            assert self.reset_ref_mode is None, "oscillating set_reference needs reset_ref_mode=None"
            o = torch.as_tensor(oscillating, dtype=torch.float64, device=self.device)
            o = o.expand(self.n, 6) if o.dim() == 1 else o
            self.ref[1:7].copy_(o.T)
            self.ref_kind.fill_(1)
        if h is not None:
            self.ref[7].copy_(torch.as_tensor(h, dtype=torch.float64, device=self.device).expand(self.n))

    KERNELS = {0: "generic", 1: "defc", 2: "recording", 3: "spec_one_wave", 4: "step_split", 5: "rollout_split"}

    def kernel(self, n_env_steps: int = 1) -> str:
        """Which kernel a step (n_env_steps = 1) or a K-step rollout of this env launches with its current batch and
        configuration (include/b747.h b747_env_kernel): "step_split" / "rollout_split" are the two-wave kernels of the
        bench, "spec_one_wave" / "defc" / "generic" / "recording" the one-wave k_env_steps instantiations."""
        self._batch()
        k = self._L.b747_env_kernel(self._bref, self._cref, self._kref, int(n_env_steps))
        _lib.check(min(k, 0), "b747_env_kernel")
        return self.KERNELS[k]

    # ------------------------------------------------------------------- gym API --
    def reset(self, mask: Optional[torch.Tensor] = None, state0=None, stream=None):
        """ControllerEnv.reset (env/ctrl_env.py:273-278) for all envs or where mask is true."""
        if state0 is not None:
            assert self.reset_ref_mode is None, "explicit state0 with a random reset mode (core/controller.py:142)"
            self.set_state0(state0)
        m = None
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        if mask is not None:
            with torch.cuda.stream(s):              # the converted mask is made (and recycled) on the launch stream
                mask = torch.as_tensor(mask).to(device=self.device, dtype=torch.uint8).contiguous()
            m = ctypes.c_void_p(mask.data_ptr())
        self._batch()
        _lib.check(self._L.b747_env_reset(self._bref, self._cref, self._kref, m, s.cuda_stream), "b747_env_reset")
        if self._use_storage:                       # Controller.reset: backup + clear (core/controller.py:195-199)
            with torch.cuda.stream(s):
                self.storage.episode_reset(mask)
        return self.obs

    def step(self, action, stream=None):
        """ControllerEnv.step (env/ctrl_env.py:260-270) for every env: returns (obs, reward, done, info)
        as device tensors; info = {"terminal_observation", "episode_return", "episode_length"}.

        action None is allowed where the SS PID flies the aircraft (AUTO / FULL_AUTO: the reference's
        Controller ignores the action there, neural/agent.py:232-236 passes None).  The returned tensors
        are the env's own buffers, rewritten by the next step (zero-copy): clone what must outlive it
        (B747VecEnv copies them to the host).  A host or non-contiguous action is staged through the
        env's own action buffer, ordered on `stream`."""
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        b = self._batch()
        if action is None:
            assert self.ctrl_type in (CtrlType.AUTO, CtrlType.FULL_AUTO), \
                "action None needs the SS PID in the loop (core/controller.py:240-250 reads action[-1])"
            with torch.cuda.stream(s):
                self.action.zero_()
            b.action = self.action.data_ptr()
        else:
            with torch.cuda.stream(s):              # conversions / staging on the launch stream: ordered
                a = torch.as_tensor(action, dtype=torch.float32)    # before the kernel, and a temporary's
                if a.device == self.device and a.is_contiguous() and a.numel() == self.n:   # block is
                    b.action = a.data_ptr()         # reused only after it (zero-copy: the caller's buffer)
                else:
                    self.action.copy_(a.reshape(self.n))
                    b.action = self.action.data_ptr()
        _lib.check(self._L.b747_env_step(self._bref, self._cref, self._kref, s.cuda_stream), "b747_env_step")
        if self._use_storage:
            with torch.cuda.stream(s):
                scaled = None
                if action is not None:              # env/ctrl_env.py:262-264: float32(a * action_max) in place
                    av = self.action if b.action == self.action.data_ptr() else a
                    scaled = (av.to(torch.float64) * self.action_max).to(torch.float32) if self.norm_act else av
                self.storage.record_step(scaled)
                if self.cfg.auto_reset:             # SB3's auto-reset at done is a ControllerEnv.reset
                    self.storage.episode_reset(self.done)
        info = {"terminal_observation": self.terminal_obs, "episode_return": self.ep_final_return,
                "episode_length": self.ep_final_len}
        return self.obs, self.reward, self.done, info

    def rollout(self, actions: torch.Tensor, obs_seq=None, reward_seq=None, done_seq=None, stream=None):
        """T env steps with actions [T, N] known in advance, in ONE launch (state stays in VGPRs).
        Fills obs_seq [T, N, obs_dim], reward_seq [T, N], done_seq [T, N] (uint8 or bool) when given."""
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        with torch.cuda.stream(s):                  # the converted actions are made (and recycled) on the launch stream
            actions = torch.as_tensor(actions).to(device=self.device, dtype=torch.float32).contiguous()
        T = actions.shape[0]
        assert actions.shape[1] == self.n
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
        self._batch()
        _lib.check(self._L.b747_env_rollout(self._bref, self._cref, self._kref,
                                            ctypes.c_void_p(actions.data_ptr()), T, ptr(obs_seq), ptr(reward_seq),
                                            ptr(done_seq), s.cuda_stream), "b747_env_rollout")
        return self.obs, self.reward, self.done

    def step_seq(self, actions: torch.Tensor, stream=None):
        """len(actions) consecutive step() calls with actions [T, N] known in advance: T launches of the
        per-step kernel issued by one C call (b747_env_step_seq), so a host loop's per-call Python cost is
        not paid per step.  obs / reward / done hold the last step's afterwards."""
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        with torch.cuda.stream(s):                  # ordered before the launches, recycled only after them
            actions = torch.as_tensor(actions).to(device=self.device, dtype=torch.float32).contiguous()
        assert actions.dim() == 2 and actions.shape[1] == self.n
        assert not self._use_storage, "Storage records per step(): use step()"
        self._batch()
        _lib.check(self._L.b747_env_step_seq(self._bref, self._cref, self._kref, ctypes.c_void_p(actions.data_ptr()),
                                             actions.shape[0], s.cuda_stream), "b747_env_step_seq")
        return self.obs, self.reward, self.done

    def time_steps(self, actions: torch.Tensor, stream=None):
        """Per-launch kernel durations (ms) of len(actions) env steps, HIP events around each launch
        (b747_env_time_steps; synchronous -- a measurement tool, not for graph capture)."""
        import numpy as np
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        with torch.cuda.stream(s):
            actions = torch.as_tensor(actions).to(device=self.device, dtype=torch.float32).contiguous()
        out = np.zeros(actions.shape[0], np.float32)
        self._batch()
        _lib.check(self._L.b747_env_time_steps(self._bref, self._cref, self._kref, ctypes.c_void_p(actions.data_ptr()),
                                               actions.shape[0], out.ctypes.data_as(ctypes.c_void_p),
                                               s.cuda_stream), "b747_env_time_steps")
        return out

    def render(self, mode="human"):
        pass

    # ----------------------------------------------------------- Controller views --
    @property
    def time(self):
        return self.k.to(torch.float64) * self.dt
