"""Fit the FAST variant's replacement of rt_powd_snf(thr, 5.2559)/thr = thr^4.2559 (ISA density,
dll@0x1b25 region) on the reachable thr range -- the generator of B747_POWFIT_* in
b747_rl_ctrl_amd/csrc/b747_dynamics.h.  Chebyshev interpolation in x86 long double, converted to
monomials in u = (thr - mid) / half, checked against long-double powl on a dense grid.
Run: python oracle/fit_isa_pow.py   (prints the C table)."""
import numpy as np

LD = np.longdouble
T0, LAPSE, TROPO_UP = LD("288.15"), LD("0.0065"), LD("11000.0")
EXP1 = LD("5.255875601466713") - 1
lo = (T0 - TROPO_UP * LAPSE) / T0          # thr at 11 km
hi = LD(1)
mid, half = (lo + hi) / 2, (hi - lo) / 2
N = 40
k = np.arange(N, dtype=LD)
x = np.cos(np.pi * (k + LD("0.5")) / N).astype(LD)
f = np.power(mid + half * x, EXP1)
c = np.array([(LD(2) / N) * np.sum(f * np.cos(j * np.arccos(x))) for j in range(N)], dtype=LD)
c[0] /= 2
DEG = 11                                   # c_12.. sit at the long-double noise floor (~2e-17)
cd = c[:DEG + 1].astype(np.float64)


def clenshaw(u):
    """double evaluation (the kernel fuses the multiply-adds: at most as large an error)"""
    b1 = b2 = 0.0
    for j in range(DEG, 0, -1):
        b1, b2 = 2 * u * b1 + (cd[j] - b2), b1
    return u * b1 + (cd[0] - b2)


grid = np.linspace(float(lo), 1.0, 100001)
u = (grid - float(mid)) * float(1 / half)
approx = np.array([clenshaw(v) for v in u])
exact = np.power(grid.astype(LD), EXP1)
rel = np.abs((approx.astype(LD) - exact) / exact)
print(f"/* thr^{float(EXP1)!r} on [{float(lo)!r}, 1]: Chebyshev degree {DEG} (Clenshaw), max rel err "
      f"{float(rel.max()):.3e} vs long-double powl */")
print(f"#define B747_POWFIT_MID {float(mid)!r}")
print(f"#define B747_POWFIT_INV_HALF {float(1 / half)!r}")
print("constexpr double kPowFit[%d] = {%s};" % (DEG + 1, ", ".join(repr(float(v)) for v in cd)))
