"""ctypes binding of libb747.so (include/b747.h).  No fallback: if the HIP library or a GPU is
missing, every entry point raises -- the product path never computes on the CPU."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# B747_LIB_PATH: an A/B build to load instead of the product library (tools/ab_*.sh); the product .so is never
# overwritten by a variant, so an interrupted A/B run cannot leave one in its place
LIB_PATH = os.environ.get("B747_LIB_PATH") or os.path.join(HERE, "libb747.so")
ABI_VERSION = 10         # include/b747.h B747_ABI_VERSION

NX, NDISC, NSIG, NAERO = 18, 9, 31, 5
F_PID_SS, F_PID_CS, F_RP, F_RL = 1, 2, 4, 8
VARIANT_FAST, VARIANT_FAITHFUL, VARIANT_MIXED = 0, 1, 2


class B747Error(RuntimeError):
    pass


class Consts(ctypes.Structure):
    _fields_ = [("Iz", ctypes.c_double), ("P", ctypes.c_double), ("S", ctypes.c_double),
                ("c_", ctypes.c_double), ("g", ctypes.c_double), ("m0", ctypes.c_double),
                ("PID_CS", ctypes.c_double * 4), ("PID_SS", ctypes.c_double * 4)]


class ModelBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("x_f64", ctypes.c_int32), ("variant", ctypes.c_int32),
                ("X", ctypes.c_void_p), ("disc", ctypes.c_void_p), ("k", ctypes.c_void_p),
                ("mem", ctypes.c_void_p), ("deltaz", ctypes.c_void_p), ("vartheta", ctypes.c_void_p),
                ("h_zh", ctypes.c_void_p), ("flags", ctypes.c_void_p), ("aero_err", ctypes.c_void_p),
                ("state0", ctypes.c_void_p), ("sig", ctypes.c_void_p)]


class EnvConfig(ctypes.Structure):
    _fields_ = [("obs_type", ctypes.c_int32), ("reward_type", ctypes.c_int32), ("ctrl_type", ctypes.c_int32),
                ("ctrl_mode", ctypes.c_int32), ("reset_ref_mode", ctypes.c_int32),
                ("disturbance_mode", ctypes.c_int32), ("norm_obs", ctypes.c_int32), ("norm_act", ctypes.c_int32),
                ("use_limiter", ctypes.c_int32), ("auto_reset", ctypes.c_int32), ("n_sub", ctypes.c_int32),
                ("aero_fixed", ctypes.c_int32), ("sample_time", ctypes.c_double), ("tk", ctypes.c_double),
                ("action_max", ctypes.c_double), ("vartheta_max", ctypes.c_double),
                ("rew", ctypes.c_double * 8), ("aero_err_fixed", ctypes.c_double * 5), ("seed", ctypes.c_uint64)]


_ENV_PTRS = ["X", "disc", "k", "mem", "deltaz", "vartheta", "h_zh", "upid", "tp", "flags", "aero_err", "ref",
             "ref_kind", "state0", "episode", "ep_return", "ep_len", "ep_final_return", "ep_final_len",
             "action", "obs", "reward", "done", "terminal_obs", "sig", "rec_params",
             "ep_stats"]


class EnvBatch(ctypes.Structure):
    _fields_ = ([("n", ctypes.c_int64), ("env_offset", ctypes.c_int64), ("x_f64", ctypes.c_int32),
                 ("obs_dim", ctypes.c_int32), ("variant", ctypes.c_int32), ("reserved", ctypes.c_int32)]
                + [(f, ctypes.c_void_p) for f in _ENV_PTRS])


_lib = None

_V, _I32, _I64, _U32, _U64, _F32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                    ctypes.c_uint64, ctypes.c_float)
_PM, _PE, _PC, _PK = (ctypes.POINTER(ModelBatch), ctypes.POINTER(EnvBatch), ctypes.POINTER(EnvConfig),
                      ctypes.POINTER(Consts))

# Every entry point of include/b747.h with its ctypes signature (argtypes, restype).  A library that
# lacks one of them is a stale build of another ABI version: lib() reports it as a version mismatch.
SIGNATURES = {
    "b747_abi_version": ([], _I32),
    "b747_struct_size": ([_I32], _I64),
    "b747_last_error": ([], ctypes.c_char_p),
    "b747_consts_default": ([_PK], _I32),
    "b747_model_initialize": ([_PM, _V, _V], _I32),
    "b747_model_step": ([_PM, _PK, _I32, _V], _I32),
    "b747_env_config_default": ([_PC, _I32, _I32], _I32),
    "b747_env_obs_dim": ([_I32], _I32),
    "b747_env_reset": ([_PE, _PC, _PK, _V, _V], _I32),
    "b747_env_step": ([_PE, _PC, _PK, _V], _I32),
    "b747_env_rollout": ([_PE, _PC, _PK, _V, _I32, _V, _V, _V, _V], _I32),
    "b747_env_time_steps": ([_PE, _PC, _PK, _V, _I32, _V, _V], _I32),
    "b747_env_step_seq": ([_PE, _PC, _PK, _V, _I32, _V], _I32),
    "b747_set_specialization": ([_I32], _I32),
    "b747_env_kernel": ([_PE, _PC, _PK, _I32], _I32),
    "b747_policy_num_params": ([_I32], _I32),
    "b747_policy_pack": ([_V, _I32, _V], _I32),
    "b747_policy_act": ([_V, _I32, _I64, _V, _V, _U64, _V, _U32, _I64, _V, _V, _V, _V, _V, _F32, _F32, _V], _I32),
    "b747_ppo_rollout": ([_PE, _PC, _PK, _V, _U64, _V, _I32] + [_V] * 6 + [_F32, _F32, _V], _I32),
}


def bind(L, version_of_lib):
    """Attach the signatures to a loaded libb747.so; a missing entry point is an ABI mismatch."""
    for name, (argtypes, restype) in SIGNATURES.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            raise B747Error(f"libb747.so ABI version mismatch: it reports version {version_of_lib} but lacks "
                            f"{name} (this binding expects version {ABI_VERSION}); rebuild it with "
                            f"`python -c 'import __graft_entry__ as g; g.build()'`") from None
        fn.argtypes, fn.restype = argtypes, restype
    return L


def lib():
    """Load libb747.so once; raise (never fall back) when it is absent or mismatched."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise B747Error(f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        try:
            L.b747_abi_version.restype = ctypes.c_int32
        except AttributeError:
            raise B747Error("libb747.so ABI version mismatch: no b747_abi_version entry point") from None
        v = int(L.b747_abi_version())
        if v != ABI_VERSION:
            raise B747Error(f"libb747.so ABI version mismatch: library {v}, binding {ABI_VERSION}; rebuild it")
        L = bind(L, v)
        for which, mirror in enumerate((Consts, ModelBatch, EnvConfig, EnvBatch)):   # B747_STRUCT_*
            if int(L.b747_struct_size(which)) != ctypes.sizeof(mirror):
                raise B747Error(f"libb747.so ABI mismatch: sizeof({mirror.__name__}) is {L.b747_struct_size(which)} "
                                f"in the library, {ctypes.sizeof(mirror)} in the binding")
        _lib = L
    return _lib


def resolve_device(device):
    """torch.device with its index filled in ("cuda" -> "cuda:<current>"): tensors report an indexed
    device, so an unindexed one would never compare equal to them (step() would then stage every
    caller's action through a copy kernel instead of reading it in place)."""
    import torch
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def check(rc, what):
    if rc != 0:
        msg = lib().b747_last_error().decode(errors="replace")
        raise B747Error(f"{what} failed ({rc}): {msg}")


def default_consts():
    c = Consts()
    check(lib().b747_consts_default(ctypes.byref(c)), "b747_consts_default")
    return c
