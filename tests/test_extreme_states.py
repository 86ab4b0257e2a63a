"""One DLL step from states at the edges of the model's domain, host builds of the product's per-lane code
against the oracle (CPU; tests/test_gpu_extreme_states.py runs the same states through the GPU).

SURVEY 8(c) asks for the reference's edge cases; for this model they are the clamps and extrapolations of
the DLL's own formulas: the ISA atmosphere's clamps at 0, 11,000 and 20,000 m (and beyond them), the
aerodynamic tables' linear extrapolation past their Mach and alpha breakpoints (Mach 2.7, flying
backwards: alpha = 180 deg, steep alpha), the attitude at and near +-90 deg pitch (cos theta = 0), a
standing aircraft (V = 0: atan2(0, 0)), tiny speeds, fast rotation and an unnormalised quaternion.
FAITHFUL (the DLL's operation order) must equal the oracle bit for bit, NaN for NaN; FAST within 1e-10 of
each signal's range over the batch, as the random-state tests (tests/test_gpu_model.py)."""
import itertools
import math

import numpy as np

import oracle_lib as O


def extreme_batch():
    hs = [-500.0, 0.0, 10999.99, 11000.0, 11000.01, 19999.0, 20000.0, 30000.0]
    vs = [(0.0, 0.0), (1e-6, 0.0), (900.0, 0.0), (-200.0, 0.0), (100.0, 100.0), (100.0, -300.0)]
    ths = [0.0, 89.99, 90.0, -90.0, 45.0]
    wzs = [0.0, 5.0]
    cases = list(itertools.product(hs, vs, ths, wzs))
    n = len(cases) + 2
    b = O.random_batch(n, seed=21)
    O.oracle_initialize(b)
    for i, (h, (vx, vy), th, wz) in enumerate(cases):
        t = math.radians(th)
        b.X[1, i], b.X[2, i], b.X[5, i] = h, math.cos(t / 2), math.sin(t / 2)
        b.X[6, i], b.X[7, i], b.X[8, i] = vx, vy, wz
    b.X[2, -2], b.X[5, -2] = 2.0 * math.cos(0.1), 2.0 * math.sin(0.1)   # |q| = 2 (the DLL normalises)
    b.X[6, -1] = 1e-300                                                  # a denormal-range speed
    return b


def _copy(b):
    c = O.Batch(b.n, b.x64)
    for k, v in vars(b).items():
        if isinstance(v, np.ndarray):
            setattr(c, k, v.copy())
    return c


def _rel(got, ref):
    scale = np.nanmax(np.abs(ref), axis=1, keepdims=True)
    scale = np.where(np.isfinite(scale) & (scale > 0), scale, 1.0)
    d = np.abs(got - ref) / scale
    d = np.where((np.isnan(got) & np.isnan(ref)) | (got == ref), 0.0, d)
    return float(np.nanmax(d))


def test_faithful_host_step_is_the_oracle_bit_for_bit_at_the_domain_edges():
    b = extreme_batch()
    h = _copy(b)
    O.oracle_step(b, 1)
    O.hostcheck_step(h, 1, fast=False)
    for name in ("X", "disc", "sig"):
        g, r = getattr(h, name), getattr(b, name)
        assert np.array_equal(g, r, equal_nan=True), f"{name}: {np.argwhere((g != r) & ~(np.isnan(g) & np.isnan(r)))[:5]}"
    assert np.array_equal(h.k, b.k) and np.array_equal(h.mem, b.mem)


def vertical(b):
    """envs at exactly +-90 deg pitch: there the DLL's theta = asin(2 q0n q3n) has an infinite derivative
    (1 ulp of its argument moves theta by ~1.5e-8 rad), while FAST takes theta as the angle of
    (2 q0n q3n, |q0n^2 - q3n^2|) -- FAST's theta is the better conditioned one, and the two
    differ by the asin's own rounding amplification"""
    s2 = 2 * b.X[2] * b.X[5] / (b.X[2] ** 2 + b.X[5] ** 2)
    return np.abs(np.abs(s2) - 1.0) < 1e-12


def test_fast_host_step_is_within_the_fast_gate_at_the_domain_edges():
    b = extreme_batch()
    v = vertical(b)
    h = _copy(b)
    O.oracle_step(b, 1)
    O.hostcheck_step(h, 1, fast=True)
    assert np.array_equal(np.isnan(h.sig), np.isnan(b.sig)), "NaN pattern"
    worst = max(_rel(h.X[:, ~v], b.X[:, ~v]), _rel(h.disc[:, ~v], b.disc[:, ~v]), _rel(h.sig[:, ~v], b.sig[:, ~v]))
    vert = max(_rel(h.X[:, v], b.X[:, v]), _rel(h.disc[:, v], b.disc[:, v]), _rel(h.sig[:, v], b.sig[:, v]))
    print(f"\nFAST vs oracle at the domain edges: {worst:.2e} of each signal's range ({vert:.2e} at +-90 deg pitch)")
    assert worst <= 1e-10
    assert v.sum() >= 64 and vert <= 1e-8
    assert np.array_equal(h.k, b.k) and np.array_equal(h.mem, b.mem)
