"""FAST-variant math kernels (b747_rl_ctrl_amd/csrc/b747_dynamics.h), host build of the same code:
the ISA power and exponential fits against pow/exp on their reachable ranges and the unit-vector
angle against atan2 over the whole circle (generators: gen/fit_isa_pow.py, gen/fit_unit_atan.py)."""
import ctypes
import math
import os
import re

import numpy as np

import oracle_lib as O


def _fn(name, nargs=1):
    f = getattr(O.lib("hostcheck"), name)
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_double] * nargs
    return f


def test_isa_power_fit():
    f = _fn("b747h_isa_powfit")
    e = 5.255875601466713 - 1
    lo = (288.15 - 11000 * 0.0065) / 288.15
    worst = max(abs(f(t) - t ** e) / t ** e for t in np.linspace(lo, 1.0, 5001))
    assert worst <= 2e-15, worst


def test_isa_exp_fit():
    f = _fn("b747h_isa_expfit")
    k = 0.03416319140953364 / (288.15 - 11000 * 0.0065)
    worst = max(abs(f(d) - math.exp(d * k)) / math.exp(d * k) for d in np.linspace(-9000.0, 0.0, 5001))
    assert worst <= 2e-15, worst


def test_unit_atan2_circle():
    f = _fn("b747h_unit_atan2", 2)
    ang = np.concatenate([np.linspace(-math.pi, math.pi, 20001), np.linspace(-0.5, 0.5, 5001),
                          [0.0, 1e-300, -1e-300, math.pi / 4, math.pi / 2, -math.pi / 2, math.pi]])
    worst = 0.0
    for a in ang:
        s, c = math.sin(a), math.cos(a)
        ref = math.atan2(s, c)
        worst = max(worst, abs(f(s, c) - ref) / max(abs(ref), 1e-300))
    assert worst <= 1e-15, worst
    # the pass's special inputs: (+-0, 1) -> +-0 (atan2(0, 0) = 0 case), NaN propagates
    assert f(0.0, 1.0) == 0.0 and math.copysign(1.0, f(-0.0, 1.0)) == -1.0
    assert math.isnan(f(math.nan, 1.0)) and math.isnan(f(0.5, math.nan))
    # theta from (s2, sqrt(1 - s2^2)), as the pass forms it
    for s2 in np.linspace(-1.0, 1.0, 2001):
        c = math.sqrt((1.0 - s2) * (1.0 + s2))
        assert abs(f(s2, c) - math.asin(s2)) <= 2e-15


def test_cell_grid_index_is_exact():
    """FAST index search on the cell grid == the DLL's interval index (bp_index) everywhere: dense
    grids over and beyond each axis, every breakpoint and its 4 neighbouring doubles on each side,
    cell boundaries, +-inf and NaN."""
    lib = O.lib("hostcheck")
    f = lib.b747h_axis_index
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
    lib.b747h_axis_cells.restype = ctypes.c_int
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "b747_tables.h")).read()
    arrays = dict((m.group(1), [float(x) for x in m.group(2).split(",")])
                  for m in re.finditer(r"double (B747_\w+)\[\d+\] = \{([^}]*)\}", hdr))
    bps = [arrays["B747_CXA_BP1"], arrays["B747_DCM_BP1"], arrays["B747_MZ_BP1"], arrays["B747_KA_BP"]]
    for axis, bp in enumerate(bps):
        assert 3 <= lib.b747h_axis_cells(axis) <= 40
        span = bp[-1] - bp[0]
        us = list(np.linspace(bp[0] - span, bp[-1] + span, 40001))
        for b in bp:
            v = b
            for _ in range(5):
                us.append(v)
                v = np.nextafter(v, -np.inf)
            v = b
            for _ in range(5):
                us.append(v)
                v = np.nextafter(v, np.inf)
        us += [np.inf, -np.inf, 1e300, -1e300, 0.0, -0.0, np.nan]
        for u in us:
            assert f(axis, 1, float(u)) == f(axis, 0, float(u)), (axis, u)
