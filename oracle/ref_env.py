"""CPU restatement of the reference's Python hot loop (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Mirrors, over the oracle's DLL-ABI library oracle/build/model_simple.so:
  RefModel          core/model.py:87-267   (ctypes binding of the exported globals; one file copy
                                             of the library per instance, core/model.py:99-110)
  RefController     core/controller.py:43-360 (step/reset/quality, action modes, sub-stepping)
  RefControllerEnv  env/ctrl_env.py:61-282  (obs layouts, rewards, done)
Random resets take their draws from an explicit `draws` dict (the GPU path's Philox draws read
back from device) instead of Python's `random`, so both sides see identical episodes.
Only tests/ and bench.py's cpu_baseline leg use this module.
"""
import ctypes
import math
import os
import shutil
import tempfile
import uuid

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "model_simple.so")

_TMP = tempfile.mkdtemp(prefix="b747_ref_models_")


class RefModel:
    """core/model.py Model over model_simple.so (Linux branch of core/model.py:104-113)."""

    SIGNALS = {"time": "sim_time", "vartheta_ref": "vartheta_zh", "deltaz_ref": "U_com_PID", "CXa": "CXa",
               "CYa": "CYa", "mz": "mz", "Kalpha": "K_alpha", "dCm_ddeltaz": "dCm_ddeltaz", "deltaz_com": "U_com",
               "deltaz_real": "deltaz_RP", "dvartheta": "dvartheta", "dvartheta_int": "dvartheta_int",
               "dvartheta_dt": "dvartheta_dt", "dvartheta_dt_dt": "dvartheta_dt_dt", "TAE": "TAE", "ITAE": "ITAE",
               "TSE": "TSE", "ITSE": "ITSE", "AE": "AE", "IAE": "IAE", "SE": "SE", "ISE": "ISE"}
    PARAMS = {"hzh": "h_zh", "use_RP": "use_RP", "use_PID_SS": "use_PID_SS", "use_PID_CS": "use_PID_CS",
              "deltaz": "deltaz", "vartheta_zh": "vartheta", "P": "P"}

    def __init__(self, use_PID_SS=True, use_PID_CS=True, initial_state=None, use_RP=True):
        path = os.path.join(_TMP, f"{uuid.uuid4()}.so")
        shutil.copyfile(SO, path)
        self._dll = ctypes.CDLL(path)
        self._path = path
        self.dt = 0.01
        d = self._dll
        self._sig = {k: ctypes.c_double.in_dll(d, v) for k, v in self.SIGNALS.items()}
        self._par = {k: ctypes.c_double.in_dll(d, v) for k, v in self.PARAMS.items()}
        self._state = (ctypes.c_double * 6).in_dll(d, "state")
        self._state0 = (ctypes.c_double * 6).in_dll(d, "state0")
        self._aero = (ctypes.c_double * 5).in_dll(d, "aero_err")
        self._pid_ss = (ctypes.c_double * 4).in_dll(d, "PID_SS")
        self._pid_cs = (ctypes.c_double * 4).in_dll(d, "PID_CS")
        if initial_state is not None:
            self.state0 = initial_state
        self.use_RP, self.use_PID_CS, self.use_PID_SS = float(use_RP), float(use_PID_CS), float(use_PID_SS)
        self.initialize()

    def __getattr__(self, name):
        if name in RefModel.SIGNALS:
            return float(self._sig[name].value)
        if name in RefModel.PARAMS:
            return float(self._par[name].value)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in RefModel.PARAMS:
            self._par[name].value = float(value)
        else:
            object.__setattr__(self, name, value)

    @property
    def state(self):
        return np.nan_to_num(np.array(list(self._state)))

    @property
    def state_dict(self):
        return dict(zip(["x", "y", "Vx", "Vy", "vartheta", "wz"], self.state))

    @property
    def state0(self):
        return np.array(list(self._state0))

    @state0.setter
    def state0(self, v):
        for i in range(6):
            self._state0[i] = float(v[i])

    @property
    def aero_err(self):
        return np.array(list(self._aero))

    @aero_err.setter
    def aero_err(self, v):
        for i in range(5):
            self._aero[i] = float(v[i])

    def initialize(self):                       # core/model.py:238-244
        self._dll.model_simple_initialize()
        self.step_num = -1
        self.deltaz = 0
        self.vartheta_zh = 0

    def step(self):                              # core/model.py:247-250
        self._dll.model_simple_step()
        self.step_num += 1

    def set_initial(self, state):
        self.state0 = state


class RefController:
    """core/controller.py Controller with explicit reset draws."""

    def __init__(self, ctrl_type, ctrl_mode, reset_ref_mode=None, disturbance_mode=None, tk=60, sample_time=None,
                 action_max=17 * math.pi / 180, vartheta_max=10 * math.pi / 180, use_limiter=False, aero_err=None):
        self.ctrl_type, self.ctrl_mode = ctrl_type, ctrl_mode
        self.reset_ref_mode, self.disturbance_mode, self.aero_err = reset_ref_mode, disturbance_mode, aero_err
        self._init_model()
        self.sample_time = sample_time if sample_time else self.model.dt
        self.tk, self.action_max, self.vartheta_max, self.use_limiter = tk, action_max, vartheta_max, use_limiter
        self.h_func = lambda _: 11000.0
        self.vartheta_func = lambda _: 0.0

    def _init_model(self):                        # core/controller.py:128-131 (ctrl types by value)
        self.use_ctrl = self.ctrl_type in (2, 0)
        self.manual_stab = self.ctrl_type in (3, 2)
        self.model = RefModel(use_PID_CS=self.use_ctrl, use_PID_SS=not self.manual_stab)

    def reset(self, draws):
        """draws: state0 [6], kind ('const'|'osc'), ref (const) or osc (A1..A3, f1..f3), h (altitude),
        hybrid_ctrl (bool, HYBRID only), aero_err [5] or None."""
        if draws.get("hybrid_ctrl") is not None:
            self.ctrl_type = 2 if draws["hybrid_ctrl"] else 3
            self._init_model()
        if draws["kind"] == "osc":
            A1, A2, A3, f1, f2, f3 = draws["osc"]
            self.vartheta_func = lambda t: A1 * math.sin(2 * math.pi * f1 * t) + A2 * math.sin(2 * math.pi * f2 * t) \
                + A3 * math.sin(2 * math.pi * f3 * t)
        else:
            ref = draws["ref"]
            self.vartheta_func = lambda _: ref
        h1 = draws.get("h", 11000.0)
        self.h_func = lambda _: h1
        self.model.set_initial(draws["state0"])
        if draws.get("aero_err") is not None:
            self.model.aero_err = draws["aero_err"]
        self.model.initialize()

    def step(self, action, record=None):          # core/controller.py:231-264
        """record(model) is called after every DLL step (Controller._post_step's Storage hook)."""
        if not self.use_ctrl:
            self.model.vartheta_zh = self.vartheta_func(self.model.time)
        else:
            self.model.hzh = self.h_func(self.model.time)
        if not self.model.use_PID_SS:
            lim = 17 * math.pi / 180
            if self.ctrl_mode is None or self.ctrl_mode == 0:
                self.model.deltaz = action[-1]
            elif self.ctrl_mode == 1:
                self.model.deltaz = float(np.clip([(1 + action[-1]) * self.model.deltaz_ref], [-lim], [lim])[0])
            elif self.ctrl_mode == 3:
                self.model.deltaz = float(np.clip([action[-1] + self.model.deltaz_ref], [-lim], [lim])[0])
            elif self.ctrl_mode == 2:
                self.model.deltaz = float(np.clip([self.model.deltaz + action[-1] * self.sample_time], [-lim], [lim])[0])
        self.model.step()
        if record:
            record(self.model)
        while round(round(self.model.time / self.model.dt) % round(self.sample_time / self.model.dt)) != 0:
            self.model.step()
            if record:
                record(self.model)

    @property
    def vartheta_ref(self):
        return self.model.vartheta_ref if self.model.use_PID_CS else self.model.vartheta_zh

    @property
    def is_limit_err(self):
        return self.use_limiter and (abs(self.model.state_dict["vartheta"]) > 5 * math.pi / 180 + self.vartheta_max
                                     or self.model.deltaz > self.action_max)

    @property
    def is_done(self):
        return self.model.time >= self.tk

    def quality(self):
        return math.exp(-60 * 0.1 * self.model.ITSE / (self.tk * self.vartheta_ref ** 2))


OBS_MAX = {0: [60 * math.pi, math.pi, math.pi], 1: [60 * math.pi, math.pi, math.pi, 500, 100],
           3: [60 * math.pi, math.pi, math.pi, 500, 100, 0.5, 2, 0.6, 0.05, 1.],
           2: [60 * math.pi, math.pi, math.pi, 0.5, 2, 0.6, 0.05, 1.],
           4: [10 * math.pi / 180, 12000, 15000, 500, 100, math.pi, math.pi]}


class RefControllerEnv:
    """env/ctrl_env.py ControllerEnv (no gym): obs/reward/done semantics, float64 like the reference."""

    def __init__(self, obs_type, rew_type, norm_obs, norm_act, ctrl, rew_config=None):
        self.obs_type, self.rew_type, self.norm_obs, self.norm_act, self.ctrl = obs_type, rew_type, norm_obs, norm_act, ctrl
        c = rew_config or {}
        self.c = c
        self.tp = 0

    def _obs_raw(self):
        m = self.ctrl.model
        sd = m.state_dict
        if self.obs_type == 0:
            return np.array([m.dvartheta_int, m.dvartheta, m.dvartheta_dt])
        if self.obs_type == 1:
            return np.array([m.dvartheta_int, m.dvartheta, m.dvartheta_dt, sd["Vx"], sd["Vy"]])
        if self.obs_type == 3:
            return np.array([m.dvartheta_int, m.dvartheta, m.dvartheta_dt, sd["Vx"], sd["Vy"], m.CXa, m.CYa, m.mz,
                             m.dCm_ddeltaz, m.Kalpha])
        if self.obs_type == 2:
            return np.array([m.dvartheta_int, m.dvartheta, m.dvartheta_dt, m.CXa, m.CYa, m.mz, m.dCm_ddeltaz,
                             m.Kalpha])
        return np.array([self.ctrl.vartheta_ref, *m.state])

    def obs(self):
        o = self._obs_raw()
        if self.norm_obs:
            o = o / np.array(OBS_MAX[self.obs_type])
        return o

    def reward(self):
        ctrl, m, c = self.ctrl, self.ctrl.model, self.c
        vf = ctrl.vartheta_ref if ctrl.vartheta_ref else ctrl.vartheta_max
        if self.rew_type == 0:
            k1, k2, k3 = c.get("k1", 2), c.get("k2", 2), c.get("k3", 1)
            kf, kITSE, k0 = c.get("kf", 0.1), c.get("kITSE", 0.3), c.get("k0", 2)
            kt, ko = -math.log(0.8) / 10, -math.log(0.75) / 0.15
            s = k1 + k2 + k3
            k1, k2, k3 = k1 / s, k2 / s, k3 / s
            r1 = 0.50 * math.exp(-k0 * (k1 * abs(m.dvartheta) + k2 * 1 * abs(m.dvartheta_dt) + k3 * abs(m.dvartheta_dt_dt)) / abs(vf))
            r2 = 0.20 * math.exp(-ko * abs(m.dvartheta / vf)) if ctrl.vartheta_ref * m.dvartheta < 0 else 0.20
            r3 = 0.20 * math.exp(-kt * m.time) if abs(m.dvartheta / vf) > 0.05 else 0.20
            r4 = 0.1 * math.exp(-kITSE * m.ITSE / (vf ** 2))
            rf = -kf * abs(m.dvartheta / (2 * vf)) * (abs(m.deltaz - m.deltaz_ref)) / (34 * math.pi / 180) \
                if ctrl.ctrl_mode == 0 else 0
            return r1 + r2 + r3 + r4 + rf
        if self.rew_type == 1:
            return math.exp(-c.get("k", 10) * abs(m.deltaz_com - m.deltaz_ref) / (34 * math.pi / 180))
        if self.rew_type in (2, 3):
            return ctrl.quality()
        overshoot = abs(m.dvartheta / vf) * 100
        if overshoot > 5:
            self.tp = m.time
        return math.exp(-c.get("k", 0.1) * abs(overshoot - c.get("overshoot_ref", 2)) * abs(c.get("tp_ref", 5) - self.tp))

    def step(self, action, record=None):
        """action: float32 scalar as the policy produced it; returns (obs, reward, done)."""
        a = np.array([action], dtype=np.float32)
        if self.norm_act:
            a *= np.array([self.ctrl.action_max])          # in place on float32 (env/ctrl_env.py:262-264)
        self.ctrl.step([float(a[-1])], record)
        return self.obs(), self.reward(), bool(self.ctrl.is_done or self.ctrl.is_limit_err)

    def reset(self, draws):
        self.ctrl.reset(draws)
        return self.obs()
