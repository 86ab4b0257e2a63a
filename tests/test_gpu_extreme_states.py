"""One DLL step from the domain-edge states of tests/test_extreme_states.py on the GPU, both arithmetic
variants against the oracle (ISA clamps beyond 0 / 11,000 / 20,000 m, table extrapolation past Mach and
alpha, +-90 deg pitch, V = 0, tiny speeds, |q| = 2).  Tolerance as tests/test_gpu_model.py's one-step test,
1e-10 of each signal's range (the GPU's libm differs from the host's by ulps, so FAITHFUL is not
bit-exact here), NaN for NaN, step counters and Memory bits exact; at exactly +-90 deg pitch the DLL's
theta = asin(2 q0n q3n) amplifies one ulp of its argument to ~1e-8 rad, so those envs get 1e-8."""
import numpy as np
import pytest

import oracle_lib as O
from test_extreme_states import _copy, _rel, extreme_batch, vertical
from test_gpu_model import _gpu_model, _load_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_one_step_at_the_domain_edges(variant):
    import torch
    b = extreme_batch()
    v = vertical(b)
    m = _gpu_model(b, variant)
    _load_state(m, b)
    ref = _copy(b)
    O.oracle_step(ref, 1)
    m.step(1)
    torch.cuda.synchronize()
    assert np.array_equal(m.k.cpu().numpy().view(np.uint32), ref.k)
    assert np.array_equal(m.mem.cpu().numpy(), ref.mem)
    got = {"X": m.X.cpu().numpy(), "disc": m.disc.cpu().numpy(), "sig": m.sig.cpu().numpy()}
    assert np.array_equal(np.isnan(got["sig"]), np.isnan(ref.sig)), "NaN pattern"
    worst = max(_rel(got[k][:, ~v], getattr(ref, k)[:, ~v]) for k in got)
    vert = max(_rel(got[k][:, v], getattr(ref, k)[:, v]) for k in got)
    print(f"\n{variant} at the domain edges: {worst:.2e} of range ({vert:.2e} at +-90 deg pitch)")
    assert worst <= 1e-10 and vert <= 1e-8
