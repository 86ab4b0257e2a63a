"""BatchModel -- N copies of the reference's `core.model.Model`, resident on one MI355X.

Mirrors core/model.py:87-267 (the ctypes wrapper around model_simple_win64.dll): the same
property names for every exported signal and parameter, the same `initialize()` side effects
(core/model.py:238-244: DLL init, step_num = -1, deltaz = 0, vartheta_zh = 0) and the same
`state` NaN scrubbing (core/model.py:167-168,200).  Every property is a torch tensor with a
leading env dimension [N] (or [N, k] for vectors) living in HBM; nothing is copied to the host.

Differences from the reference, by design:
  * one object = N models (the reference copies the DLL file once per model, core/model.py:99-110);
  * Iz, P, S, c_, g, m0 and the PID gains are batch-wide (`consts`), not per env;
  * `step(n)` can advance n major steps in one launch (state stays in registers).
The numerics run only in libb747.so (HIP, gfx950).  There is no CPU fallback.
"""
import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import F_PID_CS, F_PID_SS, F_RL, F_RP, NAERO, NDISC, NSIG, NX

# column of each exported signal in `sig` (include/b747.h B747_SIG_*)
SIG = {name: i for i, name in enumerate(
    ["sim_time", "dvartheta", "U_com", "alpha", "V", "state_x", "state_y", "state_Vx", "state_Vy",
     "state_vartheta", "state_wz", "Mach", "dvartheta_dt", "dvartheta_dt_dt", "dvartheta_int", "AE",
     "ITAE", "IAE", "ISE", "ITSE", "SE", "TAE", "TSE", "K_alpha", "mz", "dCm_ddeltaz", "CXa", "CYa",
     "deltaz_RP", "U_com_PID", "vartheta_zh"])}
STATE_LABELS = ["x", "y", "Vx", "Vy", "vartheta", "wz"]  # core/model.py:226

DEFAULT_STATE0 = (0.0, 11000.0, 259.1667, 0.0, 0.0, 0.0)  # dll .data


def _stream_handle(stream: Optional[torch.cuda.Stream]):
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class BatchModel:
    """N independent `model_simple` instances (SoA, device resident)."""

    def __init__(self, n: int, device="cuda", x_f64: bool = True, use_PID_SS=True, use_PID_CS=True,
                 initial_state=None, use_RP=True, variant: str = "fast"):
        if not torch.cuda.is_available():
            raise _lib.B747Error("BatchModel needs a ROCm GPU (torch.cuda.is_available() is False)")
        self._L = _lib.lib()
        self.n = int(n)
        self.device = _lib.resolve_device(device)
        self.x_f64 = bool(x_f64)
        assert variant in ("fast", "faithful")
        self.variant = _lib.VARIANT_FAST if variant == "fast" else _lib.VARIANT_FAITHFUL
        self.dt = 0.01  # core/model.py:121
        dev, f64 = self.device, torch.float64
        self.X = torch.zeros(NX, n, dtype=f64 if x_f64 else torch.float32, device=dev)
        self.disc = torch.zeros(NDISC, n, dtype=f64, device=dev)
        self.k = torch.zeros(n, dtype=torch.int32, device=dev)       # read as uint32 by the kernel
        self.mem = torch.zeros(n, dtype=torch.uint8, device=dev)
        self._deltaz = torch.zeros(n, dtype=f64, device=dev)
        self._vartheta = torch.zeros(n, dtype=f64, device=dev)
        self._h_zh = torch.full((n,), 11000.0, dtype=f64, device=dev)
        self.flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        self._aero_err = torch.zeros(NAERO, n, dtype=f64, device=dev)   # double aero_err[5] (core/model.py:164)
        self._state0 = torch.tensor(DEFAULT_STATE0, dtype=f64, device=dev)[:, None].repeat(1, n).contiguous()
        self.sig = torch.zeros(NSIG, n, dtype=f64, device=dev)
        self.consts = _lib.default_consts()
        if initial_state is not None:
            self.state0 = initial_state
        self.use_RP = use_RP
        self.use_PID_CS = use_PID_CS
        self.use_PID_SS = use_PID_SS
        self.Pmax = self.consts.P
        self.step_num = -1
        self.initialize()

    # ------------------------------------------------------------------ C-ABI plumbing --
    def _batch(self) -> _lib.ModelBatch:
        b = _lib.ModelBatch()
        b.n, b.x_f64, b.variant = self.n, int(self.x_f64), self.variant
        b.X, b.disc, b.k, b.mem = (self.X.data_ptr(), self.disc.data_ptr(), self.k.data_ptr(),
                                   self.mem.data_ptr())
        b.deltaz, b.vartheta, b.h_zh = self._deltaz.data_ptr(), self._vartheta.data_ptr(), self._h_zh.data_ptr()
        b.flags, b.aero_err, b.state0 = self.flags.data_ptr(), self._aero_err.data_ptr(), self._state0.data_ptr()
        b.sig = self.sig.data_ptr()
        return b

    def initialize(self, mask: Optional[torch.Tensor] = None, stream=None):
        """core/model.py:238-244 for all envs (or where mask is true)."""
        b = self._batch()
        m = None
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            m = ctypes.c_void_p(mask.data_ptr())
        _lib.check(self._L.b747_model_initialize(ctypes.byref(b), m, _stream_handle(stream)),
                   "b747_model_initialize")
        if mask is None:
            self.step_num = -1
            self._deltaz.zero_()
            self._vartheta.zero_()
        else:
            keep = mask == 0
            self._deltaz.mul_(keep)
            self._vartheta.mul_(keep)

    def step(self, n_steps: int = 1, stream=None):
        """n_steps x model_simple_step on every env (core/model.py:247-250)."""
        b = self._batch()
        _lib.check(self._L.b747_model_step(ctypes.byref(b), ctypes.byref(self.consts), int(n_steps),
                                           _stream_handle(stream)), "b747_model_step")
        self.step_num += n_steps

    def terminate(self):
        """model_simple_terminate is a no-op in the DLL (dll@0x29d0)."""

    def set_initial(self, state):
        self.state0 = state

    # ------------------------------------------------------------------------ helpers --
    def _set_flag(self, bit, value):
        v = torch.as_tensor(value, device=self.device)
        on = (v.to(torch.float64) >= 1.0) if v.dtype != torch.bool else v
        on = on.expand(self.n).to(torch.uint8)
        self.flags.copy_((self.flags & (0xFF ^ bit)) | (on * bit))

    def _get_flag(self, bit):
        return ((self.flags & bit) != 0).to(torch.float64)

    def _sig(self, name):
        return self.sig[SIG[name]]

    # ------------------------------------------------------- signals (read-only, [N]) --
    time = property(lambda self: self._sig("sim_time"))
    vartheta_ref = property(lambda self: self._sig("vartheta_zh"))      # CS PID output (naming trap)
    deltaz_ref = property(lambda self: self._sig("U_com_PID"))
    deltaz_com = property(lambda self: self._sig("U_com"))
    deltaz_real = property(lambda self: self._sig("deltaz_RP"))
    CXa = property(lambda self: self._sig("CXa"))
    CYa = property(lambda self: self._sig("CYa"))
    mz = property(lambda self: self._sig("mz"))
    Kalpha = property(lambda self: self._sig("K_alpha"))
    dCm_ddeltaz = property(lambda self: self._sig("dCm_ddeltaz"))
    dvartheta = property(lambda self: self._sig("dvartheta"))
    dvartheta_int = property(lambda self: self._sig("dvartheta_int"))
    dvartheta_dt = property(lambda self: self._sig("dvartheta_dt"))
    dvartheta_dt_dt = property(lambda self: self._sig("dvartheta_dt_dt"))
    TAE = property(lambda self: self._sig("TAE"))
    ITAE = property(lambda self: self._sig("ITAE"))
    TSE = property(lambda self: self._sig("TSE"))
    ITSE = property(lambda self: self._sig("ITSE"))
    AE = property(lambda self: self._sig("AE"))
    IAE = property(lambda self: self._sig("IAE"))
    SE = property(lambda self: self._sig("SE"))
    ISE = property(lambda self: self._sig("ISE"))
    alpha = property(lambda self: self._sig("alpha"))
    V = property(lambda self: self._sig("V"))
    Mach = property(lambda self: self._sig("Mach"))

    @property
    def state(self):
        """[N, 6] = (x, y, Vx, Vy, vartheta, wz) with NaN scrubbed (core/model.py:200)."""
        return torch.nan_to_num(self.sig[SIG["state_x"]:SIG["state_x"] + 6].T)

    @property
    def state_dict(self):
        st = self.state
        return {lab: st[:, i] for i, lab in enumerate(STATE_LABELS)}

    # ----------------------------------------------------------- parameters (r/w) --
    @property
    def state0(self):
        return self._state0.T

    @state0.setter
    def state0(self, value):
        v = torch.as_tensor(value, dtype=torch.float64, device=self.device)
        v = v.expand(self.n, 6) if v.dim() == 1 else v
        self._state0.copy_(v.T)

    @property
    def hzh(self):
        return self._h_zh

    @hzh.setter
    def hzh(self, value):
        self._h_zh.copy_(torch.as_tensor(value, dtype=torch.float64, device=self.device).expand(self.n))

    @property
    def deltaz(self):
        return self._deltaz

    @deltaz.setter
    def deltaz(self, value):
        self._deltaz.copy_(torch.as_tensor(value, dtype=torch.float64, device=self.device).expand(self.n))

    @property
    def vartheta_zh(self):
        """The DLL *parameter* `vartheta` (commanded pitch) -- core/model.py:162."""
        return self._vartheta

    @vartheta_zh.setter
    def vartheta_zh(self, value):
        self._vartheta.copy_(torch.as_tensor(value, dtype=torch.float64, device=self.device).expand(self.n))

    @property
    def aero_err(self):
        return self._aero_err.T

    @aero_err.setter
    def aero_err(self, value):
        v = torch.as_tensor(value, dtype=torch.float64, device=self.device)
        v = v.expand(self.n, NAERO) if v.dim() == 1 else v
        self._aero_err.copy_(v.T)

    use_RP = property(lambda self: self._get_flag(F_RP), lambda self, v: self._set_flag(F_RP, v))
    use_PID_SS = property(lambda self: self._get_flag(F_PID_SS), lambda self, v: self._set_flag(F_PID_SS, v))
    use_PID_CS = property(lambda self: self._get_flag(F_PID_CS), lambda self, v: self._set_flag(F_PID_CS, v))
    use_RL = property(lambda self: self._get_flag(F_RL), lambda self, v: self._set_flag(F_RL, v))

    @property
    def P(self):
        return self.consts.P

    @P.setter
    def P(self, value):
        self.consts.P = float(value)

    @property
    def PID_SS(self):
        return list(self.consts.PID_SS)

    @PID_SS.setter
    def PID_SS(self, value):
        for i in range(4):
            self.consts.PID_SS[i] = float(value[i])

    @property
    def PID_CS(self):
        return list(self.consts.PID_CS)

    @PID_CS.setter
    def PID_CS(self, value):
        for i in range(4):
            self.consts.PID_CS[i] = float(value[i])
