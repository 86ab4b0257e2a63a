"""FAST-variant math kernels (b747_rl_ctrl_amd/csrc/b747_dynamics.h), host build of the same code:
the Chebyshev ISA power against pow (<= 2e-15 relative on the reachable range)."""
import ctypes

import numpy as np

import oracle_lib as O


def _fn(name):
    f = getattr(O.lib("hostcheck"), name)
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_double]
    return f


def test_isa_power_fit():
    f = _fn("b747h_isa_powfit")
    e = 5.255875601466713 - 1
    lo = (288.15 - 11000 * 0.0065) / 288.15
    worst = max(abs(f(t) - t ** e) / t ** e for t in np.linspace(lo, 1.0, 5001))
    assert worst <= 2e-15, worst
