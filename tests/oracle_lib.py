"""ctypes bindings of the CPU oracle (oracle/build/*.so) for the test-suite.

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module.  It builds nothing itself; `make -C oracle` (or __graft_entry__.build())
produces the libraries.  Arrays are numpy, in the SoA layout of include/b747.h.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libb747_oracle.so")
DLLABI_SO = os.path.join(ROOT, "oracle", "build", "model_simple.so")
HOSTCHECK_SO = os.path.join(ROOT, "tests", "native", "build", "libb747_hostcheck.so")

NX, NDISC, NSIG, NAERO = 18, 9, 31, 5
F_PID_SS, F_PID_CS, F_RP, F_RL = 1, 2, 4, 8

SIG_NAMES = ["sim_time", "dvartheta", "U_com", "alpha", "V", "x", "y", "Vx", "Vy", "vartheta", "wz",
             "Mach", "dvartheta_dt", "dvartheta_dt_dt", "dvartheta_int", "AE", "ITAE", "IAE", "ISE",
             "ITSE", "SE", "TAE", "TSE", "K_alpha", "mz", "dCm_ddeltaz", "CXa", "CYa", "deltaz_RP",
             "U_com_PID", "vartheta_zh"]

# SURVEY A.7 defaults: Iz, P, S, c_, g, m0, PID_CS[4], PID_SS[4]
DEFAULT_CONSTS = np.array([6.73e7, 275000.0, 511.0, 8.234, 9.80665, 288760.0,
                           0.0069214, 0.00057832, 0.0083279, 1.8385,
                           -5.9151, -1.2404, -6.6927, 58.0826], dtype=np.float64)

_p = ctypes.c_void_p


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_p)


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    return ctypes.CDLL(path)


_libs = {}


def lib(name):
    if name not in _libs:
        path = {"oracle": ORACLE_SO, "hostcheck": HOSTCHECK_SO, "dllabi": DLLABI_SO}[name]
        L = _load(path)
        if name in ("oracle", "hostcheck"):
            fns = [L.b747o_batch_step] if name == "oracle" else [L.b747h_batch_step, L.b747h_batch_step_fast]
            for fn in fns:
                fn.argtypes = [ctypes.c_int64, ctypes.c_int32, _p, ctypes.c_int32] + [_p] * 11
                fn.restype = None
        if name == "oracle":
            L.b747o_batch_initialize.argtypes = [ctypes.c_int64, _p, ctypes.c_int32] + [_p] * 12
            L.b747o_batch_initialize.restype = None
            L.b747o_trajectory.argtypes = [_p, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_uint8, _p, _p, ctypes.c_int32, _p, _p, _p]
            L.b747o_trajectory.restype = None
        _libs[name] = L
    return _libs[name]


class Batch:
    """SoA numpy mirror of include/b747.h's b747_model_batch."""

    def __init__(self, n, x64=True):
        self.n, self.x64 = n, bool(x64)
        self.X = np.zeros((NX, n), np.float64 if x64 else np.float32)
        self.disc = np.zeros((NDISC, n), np.float64)
        self.k = np.zeros(n, np.uint32)
        self.mem = np.zeros(n, np.uint8)
        self.deltaz = np.zeros(n, np.float64)
        self.vartheta = np.zeros(n, np.float64)
        self.h_zh = np.full(n, 11000.0)
        self.flags = np.full(n, F_RP, np.uint8)
        self.aero_err = np.zeros((NAERO, n), np.float64)   # double aero_err[5] (core/model.py:164)
        self.state0 = np.tile(np.array([0.0, 11000.0, 259.1667, 0.0, 0.0, 0.0])[:, None], (1, n))
        self.sig = np.zeros((NSIG, n), np.float64)
        self.consts = DEFAULT_CONSTS.copy()

    def copy(self):
        b = Batch.__new__(Batch)
        for k, v in self.__dict__.items():
            setattr(b, k, v.copy() if isinstance(v, np.ndarray) else v)
        return b

    def state_arrays(self):
        return dict(X=self.X, disc=self.disc, k=self.k, mem=self.mem)

    def _args(self):
        return [_ptr(self.consts), int(self.x64), _ptr(self.X), _ptr(self.disc), _ptr(self.k),
                _ptr(self.mem), _ptr(self.deltaz), _ptr(self.vartheta), _ptr(self.h_zh),
                _ptr(self.flags), _ptr(self.aero_err), _ptr(self.state0), _ptr(self.sig)]


def oracle_initialize(b, mask=None):
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    lib("oracle").b747o_batch_initialize(b.n, *b._args(), _ptr(m))


def oracle_step(b, n_steps=1):
    lib("oracle").b747o_batch_step(b.n, n_steps, *b._args())


def hostcheck_step(b, n_steps=1, fast=False):
    L = lib("hostcheck")
    (L.b747h_batch_step_fast if fast else L.b747h_batch_step)(b.n, n_steps, *b._args())


def trajectory(n_steps, consts=None, deltaz=0.0, vartheta=0.0, h_zh=11000.0, flags=F_RP,
               aero_err=(0, 0, 0, 0, 0), state0=(0.0, 11000.0, 259.1667, 0.0, 0.0, 0.0),
               deltaz_seq=None, vartheta_seq=None):
    """Faithful single-env run (no compact round trip): [n_steps][31] signal read-outs."""
    c = DEFAULT_CONSTS.copy() if consts is None else np.asarray(consts, np.float64)
    out = np.zeros((n_steps, NSIG), np.float64)
    ae = np.asarray(aero_err, np.float64)
    s0 = np.asarray(state0, np.float64)
    dz = None if deltaz_seq is None else np.ascontiguousarray(deltaz_seq, np.float64)
    vt = None if vartheta_seq is None else np.ascontiguousarray(vartheta_seq, np.float64)
    lib("oracle").b747o_trajectory(_ptr(c), deltaz, vartheta, h_zh, flags, _ptr(ae), _ptr(s0),
                                   n_steps, _ptr(dz), _ptr(vt), _ptr(out))
    return out


def random_batch(n, seed=0, x64=True, modes="mixed"):
    """Config-3-like randomized initial conditions (core/controller.py:148-191 distributions)."""
    rng = np.random.default_rng(seed)
    b = Batch(n, x64)
    b.state0 = np.stack([np.zeros(n), rng.uniform(1000, 11000, n), rng.uniform(100, 265, n),
                         rng.uniform(-20, 20, n), np.zeros(n), rng.uniform(-1e-3, 1e-3, n)])
    sign = rng.choice([-1.0, 1.0], n)
    b.vartheta = sign * rng.uniform(np.pi / 180, 10 * np.pi / 180, n)
    b.deltaz = rng.uniform(-17, 17, n) * np.pi / 180
    b.h_zh = b.state0[1] + rng.uniform(-1000, 1000, n)
    b.aero_err = rng.normal([[-0.1], [0.1], [-0.1], [-0.1], [0.1]], 0.5, (NAERO, n))   # fp64, core/controller.py:181-193
    if modes == "mixed":
        b.flags = rng.choice(np.array([F_RP, F_RP | F_PID_SS, F_RP | F_PID_SS | F_PID_CS, F_PID_SS,
                                       F_RP | F_RL, 0], np.uint8), n)
    else:
        b.flags = np.full(n, modes, np.uint8)
    return b


def draw_resets(seed, offset, n, episode=0, mode=0, dist_mode=0, vmax=10 * np.pi / 180):
    """Controller.reset draws (core/controller.py:148-193) of envs offset..offset+n-1 from the host
    build of the GPU's Philox draw (tests/native/hostcheck.cpp b747h_draw_resets):
    state0 [n,6] f64, ref [n,8] f64, aero_err [n,5] f64, flags [n] u8 (ABI v7: float64 as the reference's)."""
    fn = lib("hostcheck").b747h_draw_resets
    fn.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                   ctypes.c_double] + [_p] * 4
    fn.restype = None
    s0, ref = np.zeros((n, 6)), np.zeros((n, 8), np.float64)
    ae, fl = np.zeros((n, 5), np.float64), np.zeros(n, np.uint8)
    fn(seed, offset, n, episode, mode, dist_mode, vmax, _ptr(s0), _ptr(ref), _ptr(ae), _ptr(fl))
    return s0, ref, ae, fl


class EnvCfg(ctypes.Structure):
    """oracle/b747_oracle_env.c b747oe_cfg."""
    _fields_ = [("obs_type", ctypes.c_int32), ("reward_type", ctypes.c_int32), ("ctrl_mode", ctypes.c_int32),
                ("norm_obs", ctypes.c_int32), ("norm_act", ctypes.c_int32), ("use_limiter", ctypes.c_int32),
                ("sample_time", ctypes.c_double), ("tk", ctypes.c_double), ("action_max", ctypes.c_double),
                ("vartheta_max", ctypes.c_double), ("rew", ctypes.c_double * 6)]


OBS_DIM = {0: 3, 1: 5, 2: 8, 3: 10, 4: 7}
REW_DEFAULTS = {0: [2, 2, 1, 0.1, 0.3, 2], 1: [10], 2: [], 3: [], 4: [2, 5, 0.1]}   # env/ctrl_env.py:109-192


class EnvOracle:
    """N ControllerEnvs of the C restatement (b747oe_*): each one DLL-faithful oracle model behind the
    reference's Controller / ControllerEnv step logic, bit-identical to oracle/ref_env.py."""

    def __init__(self, n, obs_type=0, reward_type=0, ctrl_mode=0, flags=F_RP, norm_obs=True, norm_act=True,
                 use_limiter=False, sample_time=0.01, tk=20.0, action_max=17 * np.pi / 180,
                 vartheta_max=10 * np.pi / 180, rew=None):
        L = lib("oracle")
        L.b747oe_sizeof_env.restype = ctypes.c_int64
        for name, args in (("b747oe_create", [ctypes.c_int64, _p, _p]),
                           ("b747oe_reset", [ctypes.c_int64, _p] + [_p] * 6),
                           ("b747oe_step", [ctypes.c_int64, _p, _p, _p, _p, _p, _p]),
                           ("b747oe_export", [ctypes.c_int64, _p, _p, _p]),
                           ("b747oe_export_full", [ctypes.c_int64, _p, _p, _p, _p, _p])):
            getattr(L, name).argtypes = args
            getattr(L, name).restype = None
        self.L, self.n = L, int(n)
        self.od = OBS_DIM[obs_type]
        c = self.cfg = EnvCfg()
        c.obs_type, c.reward_type, c.ctrl_mode = obs_type, reward_type, -1 if ctrl_mode is None else ctrl_mode
        c.norm_obs, c.norm_act, c.use_limiter = int(norm_obs), int(norm_act), int(use_limiter)
        c.sample_time, c.tk, c.action_max, c.vartheta_max = sample_time or 0.01, tk, action_max, vartheta_max
        for j, v in enumerate(REW_DEFAULTS[reward_type] if rew is None else rew):
            c.rew[j] = float(v)
        self.mem = np.zeros(self.n * int(L.b747oe_sizeof_env()), np.uint8)
        fl = np.broadcast_to(np.asarray(flags, np.uint8), (self.n,)).copy()
        L.b747oe_create(self.n, _ptr(self.mem), _ptr(fl))
        self.obs = np.zeros((self.n, self.od), np.float32)
        self.reward = np.zeros(self.n, np.float64)
        self.done = np.zeros(self.n, np.uint8)

    def reset(self, state0, ref, ref_kind, aero_err=None, mask=None, fresh_flags=None):
        """Controller.reset with the device-layout draws: state0 [6, n] f64, ref [8, n] f64,
        ref_kind [n] u8, aero_err [5, n] f64 or None, mask [n] or None, fresh_flags [n] (HYBRID) or None."""
        c = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
        args = [c(mask, np.uint8), c(state0, np.float64), c(ref, np.float64), c(ref_kind, np.uint8),
                c(aero_err, np.float64), c(fresh_flags, np.uint8)]
        self.L.b747oe_reset(self.n, _ptr(self.mem), *[_ptr(a) for a in args])

    def step(self, actions):
        a = np.ascontiguousarray(actions, np.float32)
        self.L.b747oe_step(self.n, _ptr(self.mem), ctypes.byref(self.cfg), _ptr(a), _ptr(self.obs),
                           _ptr(self.reward), _ptr(self.done))
        return self.obs, self.reward, self.done.astype(bool)

    def compact(self):
        X, k = np.zeros((NX, self.n)), np.zeros(self.n, np.uint32)
        self.L.b747oe_export(self.n, _ptr(self.mem), _ptr(X), _ptr(k))
        return X, k

    def compact_full(self):
        """Every env's compact model state in the device layout: X [18, n], disc [9, n], k, mem."""
        X, disc = np.zeros((NX, self.n)), np.zeros((NDISC, self.n))
        k, mem = np.zeros(self.n, np.uint32), np.zeros(self.n, np.uint8)
        self.L.b747oe_export_full(self.n, _ptr(self.mem), _ptr(X), _ptr(disc), _ptr(k), _ptr(mem))
        return X, disc, k, mem


def bench_shard(n, env_offset, seed, tk, actions):
    """Host build of one bench-workload env shard (tests/native/hostcheck.cpp b747h_bench_shard):
    n envs with global ids env_offset.., stepped len(actions) times from their first reset.
    Returns (X [18, n], k, episode, obs [n, 3], reward, done, episode return) after the last step."""
    fn = lib("hostcheck").b747h_bench_shard
    fn.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_int32] + [_p] * 8
    fn.restype = None
    a = np.ascontiguousarray(actions, np.float32)
    X, k, ep = np.zeros((18, n)), np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    obs, rew, done, ret = np.zeros((n, 3), np.float32), np.zeros(n, np.float32), np.zeros(n, np.uint8), np.zeros(n)
    fn(n, env_offset, seed, tk, a.shape[0], _ptr(a), _ptr(X), _ptr(k), _ptr(ep), _ptr(obs), _ptr(rew), _ptr(done),
       _ptr(ret))
    return X, k, ep, obs, rew, done, ret
