"""The FAST ISA cell table (include/b747_isa_cells.h) is what gen/fit_isa_cells.py makes from the DLL's ISA
constants, and its cells reproduce the DLL's atmosphere (oracle/b747_oracle.c isa(), the long-double
reference of gen/fit_isa_pow.py) to a few ulp over the whole clamped range [0, 20000] m."""
import importlib.util
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("fit_isa_cells", os.path.join(ROOT, "gen", "fit_isa_cells.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def test_header_is_the_generators_output_and_uses_the_dlls_constants(tmp_path):
    g = _gen()
    out = tmp_path / "cells.h"
    worst = g.main(str(out))
    assert out.read_text() == open(os.path.join(ROOT, "include", "b747_isa_cells.h")).read()
    assert max(worst) < 1e-15
    hdr = open(os.path.join(ROOT, "include", "b747_tables.h")).read()
    val = lambda name: float(re.search(rf"#define B747_ISA_{name} \(([^)]+)\)", hdr).group(1))
    for name, v in (("T0", g.T0), ("LAPSE", g.LAPSE), ("H_TROPO", g.H_TROPO), ("EXP", g.EXP), ("G_R", g.G_R),
                    ("GAMMA_R", g.GAMMA_R), ("RHO0", g.RHO0), ("STRAT_LO", g.STRAT_LO)):
        assert val(name) == float(v), name


def test_cells_match_the_dll_formula_in_long_double():
    g = _gen()
    hdr = open(os.path.join(ROOT, "include", "b747_isa_cells.h")).read()
    body = hdr[hdr.index("{") + 1:hdr.rindex("}")]
    cells = np.array([float(x) for x in body.replace("\n", " ").split(",") if x.strip()]).reshape(g.NC, 2 * g.STRIDE + g.PAD)[:, :2 * g.STRIDE].reshape(g.NC, 2, g.STRIDE)
    LD = np.longdouble
    h = np.linspace(-500.0, 20500.0, 42001)
    hc = np.clip(h, 0.0, 11000.0).astype(LD)
    T = LD("288.15") - hc * LD("0.0065")
    dhc = np.clip(11000.0 - h, -9000.0, 0.0).astype(LD)
    rho = np.exp(dhc * LD("0.03416319140953364") / T) * (np.power(T / LD("288.15"), LD("5.255875601466713") - 1)
                                                         * LD("1.225"))
    inva = 1 / np.sqrt(T * LD("401.87433999999996"))
    hcl = np.where(h > 20000.0, 20000.0, np.maximum(0.0, h))
    x = hcl * 0.002
    c = np.clip(x.astype(np.int64), 0, g.NC - 1)
    u = x - c
    r, v = cells[c, 0, g.DEG], cells[c, 1, g.DEG]
    for q in range(g.DEG - 1, -1, -1):
        r = r * u + cells[c, 0, q]
        v = v * u + cells[c, 1, q]
    assert float(np.max(np.abs((r - rho) / rho))) < 2e-15
    assert float(np.max(np.abs((v - inva) / inva))) < 1e-15
