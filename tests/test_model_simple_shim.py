"""b747_rl_ctrl_amd/model_simple.so: the reference DLL's exported-globals ABI (core/model.py:104-164)
over the HIP model kernels.  CPU: it loads (no GPU call at load), exports every symbol the DLL does and
holds the DLL's parameter defaults.  GPU: driven the way core/model.py drives the DLL (set globals,
model_simple_initialize / model_simple_step, read globals), it follows the CPU oracle's DLL-ABI library
(oracle/build/model_simple.so) to 1e-9 of each signal's range over 600 steps with parameter changes,
a re-initialize and the SS/CS PID loops switched on mid-run."""
import ctypes
import os
import shutil
import tempfile
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "b747_rl_ctrl_amd", "model_simple.so")
ORACLE_SHIM = os.path.join(ROOT, "oracle", "build", "model_simple.so")

PARAMS = ["Iz", "P", "S", "c_", "deltaz", "g", "h_zh", "m0", "use_PID_CS", "use_PID_SS", "use_RL", "use_RP", "vartheta"]
ARRAYS = {"PID_CS": 4, "PID_SS": 4, "aero_err": 5, "state0": 6}
SIGNALS = ["sim_time", "dvartheta", "U_com", "alpha", "V", "Mach", "dvartheta_dt", "dvartheta_dt_dt", "dvartheta_int",
           "AE", "ITAE", "IAE", "ISE", "ITSE", "SE", "TAE", "TSE", "K_alpha", "mz", "dCm_ddeltaz", "CXa", "CYa",
           "deltaz_RP", "U_com_PID", "vartheta_zh"]
DLL_SYMBOLS = ["model_simple_initialize", "model_simple_step", "model_simple_terminate", "state"] + PARAMS + \
    list(ARRAYS) + SIGNALS


def _load(path, install=True):
    """One private copy per model, exactly as core/model.py:99-113 does it: the library sits in a `core`
    folder, and every Model copies it to core/tmp_models/<uuid>.so and loads the copy.  install: the
    user put model_simple.so AND libb747.so in that folder (found from the copy through $ORIGIN/..);
    otherwise only model_simple.so is there and libb747.so comes from the build directory's rpath."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    core = tempfile.mkdtemp(prefix="b747_core_")
    shutil.copyfile(path, os.path.join(core, "model_simple.so"))
    if install and path == SHIM:
        shutil.copyfile(os.path.join(os.path.dirname(SHIM), "libb747.so"), os.path.join(core, "libb747.so"))
    tmp_dir = os.path.join(core, "tmp_models")                              # core/model.py:100-102
    os.makedirs(tmp_dir, exist_ok=True)
    dst = os.path.join(tmp_dir, f"{uuid.uuid4()}.so")                       # core/model.py:103-110
    shutil.copyfile(os.path.join(core, "model_simple.so"), dst)
    return ctypes.CDLL(dst)                                                 # core/model.py:112-113


class Model:
    """The core/model.py access pattern over either library."""

    def __init__(self, path):
        self.d = _load(path)
        self.par = {k: ctypes.c_double.in_dll(self.d, k) for k in PARAMS}
        self.arr = {k: (ctypes.c_double * n).in_dll(self.d, k) for k, n in ARRAYS.items()}
        self.sig = {k: ctypes.c_double.in_dll(self.d, k) for k in SIGNALS}
        self.state = (ctypes.c_double * 6).in_dll(self.d, "state")

    def set(self, **kw):
        for k, v in kw.items():
            if k in ARRAYS:
                for j, x in enumerate(v):
                    self.arr[k][j] = float(x)
            else:
                self.par[k].value = float(v)

    def read(self):
        return np.array([self.sig[k].value for k in SIGNALS] + list(self.state))


@pytest.mark.parametrize("install", [True, False], ids=["beside_core", "build_rpath"])
def test_shim_exports_the_dll_symbol_set_and_defaults(install):
    """Loads as core/model.py loads it (a uuid copy in tmp_models, no symlinks) -- with libb747.so installed
    beside the original or found through the build directory -- and exports the DLL's symbols."""
    shim, ref = _load(SHIM, install), _load(ORACLE_SHIM)
    for name in DLL_SYMBOLS:
        assert hasattr(shim, name), name
    for k in PARAMS:
        assert ctypes.c_double.in_dll(shim, k).value == ctypes.c_double.in_dll(ref, k).value, k
    for k, n in ARRAYS.items():
        assert list((ctypes.c_double * n).in_dll(shim, k)) == list((ctypes.c_double * n).in_dll(ref, k)), k
    for k in SIGNALS:                                   # nothing has run yet: zero, as in the DLL image
        assert ctypes.c_double.in_dll(shim, k).value == 0.0, k


def _close(a, b, span, what):
    err = np.abs(a - b) / np.maximum(span, 1e-12)
    j = int(np.argmax(err))
    names = SIGNALS + [f"state[{i}]" for i in range(6)]
    assert err[j] <= 1e-9, f"{what}: {names[j]} gpu {a[j]!r} oracle {b[j]!r} (rel to range {err[j]:.2e})"


@pytest.mark.gpu
def test_shim_follows_the_oracle_dll_abi_through_a_scripted_session():
    gpu, ref = Model(SHIM), Model(ORACLE_SHIM)
    rows_g, rows_r = [], []

    def both(fn):
        for m, rows in ((gpu, rows_g), (ref, rows_r)):
            fn(m)
            rows.append(m.read())

    # 1) stepping before any initialize: the DLL image is initialised from its defaults
    for _ in range(20):
        both(lambda m: m.d.model_simple_step())
    # 2) core/model.py initialize with a new initial state and aero errors, RP actuator, manual deltaz;
    #    the aero errors are fp64 normal draws as Controller.reset makes them (core/controller.py:181-193),
    #    not exact in float32: the shim must carry the DLL's double aero_err[5] through unrounded
    ae = np.random.default_rng(7).normal([-.1, .1, -.1, -.1, .1], 0.5)
    assert np.all(ae.astype(np.float32).astype(np.float64) != ae)
    both(lambda m: (m.set(state0=[0.0, 9500.0, 240.0, 0.0, 0.03, 0.0], aero_err=ae,
                          use_RP=1.0, use_PID_SS=0.0, use_PID_CS=0.0, deltaz=0.0), m.d.model_simple_initialize()))
    for k in range(200):
        both(lambda m, k=k: (m.set(deltaz=0.05 * np.sin(0.03 * k)), m.d.model_simple_step()))
    # 3) pitch loop (SS PID) on a new reference, then the altitude loop (CS PID) on top, gains changed
    both(lambda m: (m.set(use_PID_SS=1.0, vartheta=0.06), m.d.model_simple_step()))
    for _ in range(200):
        both(lambda m: m.d.model_simple_step())
    both(lambda m: (m.set(use_PID_CS=1.0, h_zh=9700.0, PID_SS=[-6.0, -1.3, -6.5, 55.0]), m.d.model_simple_step()))
    for _ in range(180):
        both(lambda m: m.d.model_simple_step())
    # 4) re-initialize mid-flight (core/model.py:238-241 on every ControllerEnv.reset)
    both(lambda m: (m.set(use_PID_CS=0.0, use_PID_SS=0.0, use_RL=1.0), m.d.model_simple_initialize()))
    for _ in range(20):
        both(lambda m: m.d.model_simple_step())
    g, r = np.array(rows_g), np.array(rows_r)
    assert np.isfinite(r).all()
    span = r.max(axis=0) - r.min(axis=0) + np.abs(r).max(axis=0) * 1e-3
    for t in range(len(g)):
        _close(g[t], r[t], span, f"call {t}")
