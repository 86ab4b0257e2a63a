"""ctypes binding of libb747.so (include/b747.h).  No fallback: if the HIP library or a GPU is
missing, every entry point raises -- the product path never computes on the CPU."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libb747.so")
ABI_VERSION = 1

NX, NDISC, NSIG, NAERO = 18, 9, 31, 5
F_PID_SS, F_PID_CS, F_RP, F_RL = 1, 2, 4, 8


class B747Error(RuntimeError):
    pass


class Consts(ctypes.Structure):
    _fields_ = [("Iz", ctypes.c_double), ("P", ctypes.c_double), ("S", ctypes.c_double),
                ("c_", ctypes.c_double), ("g", ctypes.c_double), ("m0", ctypes.c_double),
                ("PID_CS", ctypes.c_double * 4), ("PID_SS", ctypes.c_double * 4)]


class ModelBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("x_f64", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("X", ctypes.c_void_p), ("disc", ctypes.c_void_p), ("k", ctypes.c_void_p),
                ("mem", ctypes.c_void_p), ("deltaz", ctypes.c_void_p), ("vartheta", ctypes.c_void_p),
                ("h_zh", ctypes.c_void_p), ("flags", ctypes.c_void_p), ("aero_err", ctypes.c_void_p),
                ("state0", ctypes.c_void_p), ("sig", ctypes.c_void_p)]


_lib = None


def lib():
    """Load libb747.so once; raise (never fall back) when it is absent or mismatched."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise B747Error(f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        L.b747_abi_version.restype = ctypes.c_int32
        if L.b747_abi_version() != ABI_VERSION:
            raise B747Error("libb747.so ABI version mismatch")
        L.b747_last_error.restype = ctypes.c_char_p
        L.b747_consts_default.argtypes = [ctypes.POINTER(Consts)]
        L.b747_consts_default.restype = ctypes.c_int32
        L.b747_model_initialize.argtypes = [ctypes.POINTER(ModelBatch), ctypes.c_void_p, ctypes.c_void_p]
        L.b747_model_initialize.restype = ctypes.c_int32
        L.b747_model_step.argtypes = [ctypes.POINTER(ModelBatch), ctypes.POINTER(Consts), ctypes.c_int32,
                                      ctypes.c_void_p]
        L.b747_model_step.restype = ctypes.c_int32
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().b747_last_error().decode(errors="replace")
        raise B747Error(f"{what} failed ({rc}): {msg}")


def default_consts():
    c = Consts()
    check(lib().b747_consts_default(ctypes.byref(c)), "b747_consts_default")
    return c
