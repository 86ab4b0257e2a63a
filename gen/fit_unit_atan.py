"""Fit the FAST variant's angle of a unit vector, unit_atan2(s, c) = atan2(s, c) for s^2 + c^2 = 1
(b747_rl_ctrl_amd/csrc/b747_dynamics.h) -- it replaces ocml's general atan2 for the angle of
attack (dll@0x1b25 region: alpha = -rt_atan2d_snf(v, u), with (s, c) = (-v, u) / V) and asin for
the pitch angle (theta = asin(s2), with c = cos(theta) = sqrt((1 - s2)(1 + s2))).

Reduction: lo = min(|s|, |c|), hi = max(|s|, |c|) give psi = atan2(lo, hi) in [0, pi/4]; for a
unit vector sin(psi / 2) = lo / sqrt(2 (1 + hi)) = x in [0, sin(pi/8)], and
psi = 2 asin(x) = 2x (1 + z P(z)), z = x^2.  P is fitted here: Chebyshev interpolation of
g(z) = (asin(sqrt z) - sqrt z) / z^1.5 on [0, sin^2(pi/8)] in x86 long double, converted to
monomials in z (the kernel evaluates them as E(z^2) + z O(z^2) by Horner: depth 6 instead of 10).
Then the octant / quadrant / sign fix-ups.  Checked against long-double arctan2 on a dense grid.
Run: python gen/fit_unit_atan.py   (prints the C table)."""
import numpy as np
from numpy.polynomial import chebyshev as C, polynomial as Pn

LD = np.longdouble
ZMAX = (1 - np.sqrt(LD(2)) / 2) / 2           # sin^2(pi/8)
N = 48
k = np.arange(N, dtype=LD)
t = np.cos(np.pi * (k + LD("0.5")) / N).astype(LD)
z = (t + 1) * ZMAX / 2
x = np.sqrt(z)
g = (np.arcsin(x) - x) / (z * x)
c = np.array([(LD(2) / N) * np.sum(g * np.cos(j * np.arccos(t))) for j in range(N)], dtype=LD)
c[0] /= 2
DEG = 9
mono_t = C.cheb2poly(c[:DEG + 1])             # monomials in t, t = (2 z / ZMAX) - 1
mono_z = np.zeros(DEG + 1, dtype=LD)
lin = np.array([LD(-1), LD(2) / ZMAX], dtype=LD)
powk = np.array([LD(1)], dtype=LD)
for j in range(DEG + 1):
    mono_z[: len(powk)] += mono_t[j] * powk
    powk = Pn.polymul(powk, lin)
cz = mono_z.astype(np.float64)


def estrin(zz):
    """the kernel's poly_even_odd: E(z^2) + z O(z^2), both by Horner"""
    v = zz * zz
    e = 0.0
    for k in reversed(cz[0::2]):
        e = e * v + k
    o = 0.0
    for k in reversed(cz[1::2]):
        o = o * v + k
    return o * zz + e


def unit_atan2(s, cc):
    """double emulation of the kernel (separate roundings: at least as large an error as its FMAs)"""
    a, b = abs(s), abs(cc)
    sw = a > b
    lo, hi = (b, a) if sw else (a, b)
    xx = lo / np.sqrt(2.0 + 2.0 * hi)
    zz = xx * xx
    x2 = xx + xx
    psi = x2 + (x2 * zz) * estrin(zz)
    phi = (np.pi / 2 - psi) if sw else psi
    phi = (np.pi - phi) if cc < 0 else phi
    return -phi if s < 0 else phi


ang = np.concatenate([np.linspace(-np.pi, np.pi, 400001), np.linspace(-0.6, 0.6, 200001),
                      np.array([0.0, 1e-300, 1e-20, np.pi / 4, np.pi / 2, -np.pi / 2])])
s, cc = np.sin(ang), np.cos(ang)
approx = np.array([unit_atan2(a, b) for a, b in zip(s, cc)])
exact = np.arctan2(s.astype(LD), cc.astype(LD))
err = np.abs(approx.astype(LD) - exact)
rel = err / np.maximum(np.abs(exact), LD(1e-300))
ulp = err / np.spacing(np.abs(exact).astype(np.float64)).astype(LD)
zz = np.linspace(0, float(ZMAX), 20001)
xs = np.sqrt(zz)
pol = (xs + xs * zz * np.array([estrin(v) for v in zz])).astype(LD)
prel = np.abs(pol - np.arcsin(xs.astype(LD))) / np.maximum(np.arcsin(xs.astype(LD)), LD(1e-300))
print(f"/* asin(x) = x (1 + z P(z)) on z = x^2 in [0, {float(ZMAX)!r}]: P degree {DEG} (even/odd Horner), max rel "
      f"err {float(prel.max()):.2e}; unit_atan2 over the circle: max {float(ulp.max()):.1f} ulp, "
      f"max rel {float(rel.max()):.2e} vs long-double atan2 */")
print("constexpr double kAsinP[%d] = {%s};" % (DEG + 1, ", ".join(repr(float(v)) for v in cz)))
