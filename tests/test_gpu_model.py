"""GPU parity of the model-level HIP path (b747_model_* through the C ABI) against the CPU
oracle (faithful fp64 restatement of model_simple_win64.dll, oracle/b747_oracle.c).

Tolerances (written here, checked per field as max|gpu-oracle| / max|oracle| over envs):
  * fp64 state, one step from identical state:      <= 1e-10  (libm ulp differences only; the
    double Derivative read-out dvartheta_dt_dt divides them by h twice: ~1e-16 / 1e-4)
  * fp64 state, free-running trajectories:  <= 1e-6 for 1000 steps (chaotic saturated PID envs amplify
    libm ulp differences after that); every 50 steps over all 2000 a shadow batch restarted from the
    oracle's state must match its next step to 1e-10 on every env
Both arithmetic variants (FAST = product default, FAITHFUL = DLL operation order) are held to
the same bars; FAST one-step launches with the default constants run the three-wave kernel
(k_model_step_split), K-step launches the one-wave kernel, and the two agree to a few ulp.
  * fp32 state, one step from identical fp32 state:   <= 1e-5   (north-star per-step gate)
Integer/byte state (k, Memory bits) must match exactly.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _gpu_model(batch, variant="fast"):
    from b747_rl_ctrl_amd import BatchModel
    m = BatchModel(batch.n, x_f64=batch.x64, variant=variant)
    m._state0.copy_(torch.from_numpy(batch.state0))
    m.flags.copy_(torch.from_numpy(batch.flags))
    m._aero_err.copy_(torch.from_numpy(batch.aero_err))
    m._deltaz.copy_(torch.from_numpy(batch.deltaz))
    m._vartheta.copy_(torch.from_numpy(batch.vartheta))
    m._h_zh.copy_(torch.from_numpy(batch.h_zh))
    return m


def _init_both(m, b):
    """Model.initialize() also zeroes the deltaz/vartheta parameters (core/model.py:243-244);
    the raw DLL initialize does not -- restore the batch's parameters on the GPU side."""
    m.initialize()
    m._deltaz.copy_(torch.from_numpy(b.deltaz))
    m._vartheta.copy_(torch.from_numpy(b.vartheta))
    O.oracle_initialize(b)


def _load_state(m, b):
    m.X.copy_(torch.from_numpy(b.X))
    m.disc.copy_(torch.from_numpy(b.disc))
    m.k.copy_(torch.from_numpy(b.k.view(np.int32)))
    m.mem.copy_(torch.from_numpy(b.mem))


def _rel(gpu, ref):
    gpu = np.asarray(gpu, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.max(np.abs(ref), axis=-1, keepdims=True)
    scale = np.where(scale > 0, scale, 1.0)
    d = np.abs(gpu - ref) / scale
    d = np.where(np.isnan(gpu) & np.isnan(ref), 0.0, d)
    return float(np.nanmax(d)) if d.size else 0.0


def _compare(m, b, tol, what, sig_rows=None):
    torch.cuda.synchronize()
    assert np.array_equal(m.k.cpu().numpy().view(np.uint32), b.k), f"{what}: step counters differ"
    assert np.array_equal(m.mem.cpu().numpy(), b.mem), f"{what}: anti-windup memory bits differ"
    ex = _rel(m.X.cpu().numpy(), b.X)
    ed = _rel(m.disc.cpu().numpy(), b.disc)
    rows = slice(None) if sig_rows is None else sig_rows
    es = _rel(m.sig.cpu().numpy()[rows], b.sig[rows])
    if not (ex <= tol and ed <= tol and es <= tol):
        names = [O.SIG_NAMES[j] for j in range(O.NSIG)][rows]
        per = [_rel(m.sig.cpu().numpy()[rows][j], b.sig[rows][j]) for j in range(len(names))]
        worst = names[int(np.argmax(per))]
        raise AssertionError(f"{what}: X {ex:.3e} disc {ed:.3e} sig {es:.3e} (worst {worst}) > {tol}")
    return max(ex, ed, es)


@pytest.mark.parametrize("n", [1, 77, 1000])
def test_initialize_matches_oracle(n):
    b = O.random_batch(n, seed=n)
    m = _gpu_model(b)
    m.initialize()
    O.oracle_initialize(b)
    _compare(m, b, 0.0, "initialize")
    assert float(m.deltaz.abs().max()) == 0.0 and float(m.vartheta_zh.abs().max()) == 0.0


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_single_step_fp64_from_identical_state(variant):
    b = O.random_batch(4096, seed=3)
    O.oracle_initialize(b)
    O.oracle_step(b, 137)           # arrive at a mid-episode state on the CPU
    m = _gpu_model(b, variant)
    _load_state(m, b)
    for _ in range(5):              # then every step starts from the oracle's exact state
        m.step(1)
        O.oracle_step(b, 1)
        _compare(m, b, 1e-10, "one step fp64")
        _load_state(m, b)


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_trajectory_fp64_2000_steps(variant):
    """Free-running 20 s episodes plus a shadow check that constrains EVERY env at every point.
    Free run: all envs agree to 1e-6 for the first 1000 steps.  Beyond that a few closed-loop PID envs
    with a saturated, rate-limited actuator are chaotic (error doubles every ~50 steps from ulp-level
    libm differences -- ocml vs glibc), so a free run cannot be bounded per env over 2000 steps.
    Shadow: every 50 steps over the whole 2000, a second GPU batch is loaded with the ORACLE's state,
    stepped once, and must match the oracle's next step on every env (1e-10 of each signal's range over the
    trajectory -- 1e-9 for the double Derivative dvartheta_dt_dt -- and 1e-9 of its spread at that step)
    with exact step counters and Memory
    bits on every env -- so each env's dynamics are checked along the oracle's own trajectory, late
    episode branches (saturations, rate limits, anti-windup) included."""
    b = O.random_batch(512, seed=5)
    m = _gpu_model(b, variant)
    shadow = _gpu_model(b, variant)
    _init_both(m, b)
    shadow.initialize()
    shadow._deltaz.copy_(torch.from_numpy(b.deltaz))
    shadow._vartheta.copy_(torch.from_numpy(b.vartheta))
    sig_range = np.zeros((O.NSIG, 1))       # each signal's range so far over the whole batch
    for chunk in range(40):
        b1 = b.copy()                        # the oracle's state at step 50 * chunk
        _load_state(shadow, b1)
        shadow.step(1)
        O.oracle_step(b1, 1)
        sig_range = np.maximum(sig_range, np.nanmax(np.abs(b1.sig), axis=1, keepdims=True))
        what = f"shadow step {50 * chunk + 1}"
        # normalised by the signal's spread at this step -- except dvartheta_dt_dt, whose spread at a settled
        # step can be ~1e-4 of its range: the range check below holds it (with fp64 aero_err draws, FAST
        # measured 1.7e-9 of that spread at step 1101 on this batch, 2 ulp of theta x 1/h^2)
        dd = O.SIG_NAMES.index("dvartheta_dt_dt")
        _compare(shadow, b1, 1e-9, what, sig_rows=[j for j in range(O.NSIG) if j != dd])
        # normalised by its range over the trajectory: the double Derivative read-out
        # dvartheta_dt_dt = delta^2 / h^2 magnifies ulps by 1e4, and at settled steps its spread is small
        es = np.nanmax(np.abs(shadow.sig.cpu().numpy() - b1.sig) / np.maximum(sig_range, 1e-300), axis=1)
        tol = np.full(O.NSIG, 1e-10)
        tol[O.SIG_NAMES.index("dvartheta_dt_dt")] = 1e-9      # FAST: ~2 ulp of theta x 1/h^2
        assert np.all(es <= tol), f"{what}: " + ", ".join(f"{O.SIG_NAMES[j]} {es[j]:.2e}"
                                                          for j in np.flatnonzero(es > tol))
        m.step(50)
        O.oracle_step(b, 50)
        if chunk < 20:
            torch.cuda.synchronize()
            g, r = m.sig.cpu().numpy(), b.sig
            scale = np.maximum(np.abs(r).max(axis=1, keepdims=True), 1e-300)
            per_env = np.nanmax(np.abs(g - r) / scale, axis=0)
            assert per_env.max() <= 1e-6, f"free run step {(chunk + 1) * 50}: max {per_env.max():.3e}"
            assert np.array_equal(m.mem.cpu().numpy(), b.mem)
    assert np.all(b.k == 2000)


def _specialization(on):
    from b747_rl_ctrl_amd import _lib
    return _lib.lib().b747_set_specialization(int(on))


def test_multi_step_launch_equals_single_steps():
    """The one-wave kernel: one 50-step launch and 50 one-step launches, bit for bit.  (With the specialised kernels
    on, a one-step launch with the DLL's default constants runs the three-wave kernel instead: next test.)"""
    b = O.random_batch(300, seed=11)
    m1 = _gpu_model(b)
    m2 = _gpu_model(b)
    m1.initialize(); m2.initialize()
    prev = _specialization(0)
    try:
        m1.step(50)
        for _ in range(50):
            m2.step(1)
        torch.cuda.synchronize()
    finally:
        _specialization(prev)
    assert torch.equal(m1.X, m2.X) and torch.equal(m1.disc, m2.disc) and torch.equal(m1.sig, m2.sig)


@pytest.mark.parametrize("n,modes", [(4096, "mixed"), (4096, O.F_RP), (1, O.F_RP), (77, "mixed"), (130, O.F_RP | O.F_PID_CS)])
def test_three_wave_one_step_kernel_matches_the_one_wave_kernel(n, modes):
    """b747_model_step(n_steps = 1) with the DLL's default constants runs k_model_step_split (b747_model_split.h: each
    env over a flight, an ahead and a control wave; BASELINE config 2's per-step calls).  From identical states, every
    step against the one-wave kernel (b747_set_specialization(0)): the same operations, FMA-contracted in a different
    grouping, so X, the discrete state and the 31 signals agree to a few ulp (1e-12 of each field's scale; the double
    Derivative read-out dvartheta_dt_dt, which divides ulps by h^2, to 1e-9) and k and the Memory bits exactly --
    for waves whose delta is posted up front (MANUAL, RP) and lock-step waves (SS PID, dead zone), ragged n."""
    b = O.random_batch(n, seed=21, modes=modes)
    O.oracle_initialize(b)
    O.oracle_step(b, 173)
    split, one = _gpu_model(b), _gpu_model(b)
    dd = O.SIG_NAMES.index("dvartheta_dt_dt")
    for step in range(20):
        _load_state(split, b)
        _load_state(one, b)
        split.step(1)
        prev = _specialization(0)
        try:
            one.step(1)
        finally:
            _specialization(prev)
        torch.cuda.synchronize()
        assert torch.equal(split.k, one.k) and torch.equal(split.mem, one.mem), step
        assert _rel(split.X.cpu().numpy(), one.X.cpu().numpy()) <= 1e-12, step
        assert _rel(split.disc.cpu().numpy(), one.disc.cpu().numpy()) <= 1e-12, step
        gs, go = split.sig.cpu().numpy(), one.sig.cpu().numpy()
        rows = [j for j in range(O.NSIG) if j != dd]
        assert _rel(gs[rows], go[rows]) <= 1e-12, (step, max(rows, key=lambda j: _rel(gs[j], go[j])))
        assert _rel(gs[dd], go[dd]) <= 1e-9, step
        O.oracle_step(b, 1)                              # the next step starts from the oracle's state


@pytest.mark.parametrize("n,modes,k,tol", [(4096, O.F_RP, 100, 1e-10), (77, O.F_RP, 37, 1e-10), (4096, "mixed", 10, 1e-9),
                                            (130, O.F_RP | O.F_PID_CS, 25, 1e-9), (1, O.F_PID_SS, 9, 1e-9)])
def test_three_wave_k_step_kernel_matches_the_one_wave_kernel(n, modes, k, tol):
    """b747_model_step(n_steps = K > 1) with the DLL's default constants on n <= 16,384 envs runs k_model_steps_split
    (b747_model_split.h: the three roles with the state in registers across the K steps, ring hand-offs).  From an
    oracle mid-episode state, one K-step launch against the one-wave kernel's (b747_set_specialization(0)): X, the
    discrete state (U_com history included) and the last step's 31 signals within `tol` of each field's scale --
    ulp-level grouping differences carried over K steps (open loop: 1e-10; closed-loop PID envs, which amplify them:
    1e-9) -- k and the Memory bits exactly; ragged n, lock-step waves, K not a multiple of the rings."""
    b = O.random_batch(n, seed=31, modes=modes)
    O.oracle_initialize(b)
    O.oracle_step(b, 211)
    split, one = _gpu_model(b), _gpu_model(b)
    _load_state(split, b)
    _load_state(one, b)
    split.step(k)
    prev = _specialization(0)
    try:
        one.step(k)
    finally:
        _specialization(prev)
    torch.cuda.synchronize()
    assert torch.equal(split.k, one.k) and torch.equal(split.mem, one.mem)
    assert _rel(split.X.cpu().numpy(), one.X.cpu().numpy()) <= tol
    assert _rel(split.disc.cpu().numpy(), one.disc.cpu().numpy()) <= tol
    dd = O.SIG_NAMES.index("dvartheta_dt_dt")
    gs, go = split.sig.cpu().numpy(), one.sig.cpu().numpy()
    rows = [j for j in range(O.NSIG) if j != dd]
    assert _rel(gs[rows], go[rows]) <= tol, max(rows, key=lambda j: _rel(gs[j], go[j]))
    assert _rel(gs[dd], go[dd]) <= 1e3 * tol
    O.oracle_step(b, k)                                  # and both against the oracle
    _compare(split, b, 1e-8, "k-step three-wave vs oracle", sig_rows=rows)


@pytest.mark.parametrize("variant", ["fast", "faithful"])
def test_single_step_fp32_state_gate(variant):
    b = O.random_batch(4096, seed=7, x64=False)
    O.oracle_initialize(b)
    O.oracle_step(b, 251)
    m = _gpu_model(b, variant)
    for _ in range(3):
        _load_state(m, b)
        m.step(1)
        O.oracle_step(b, 1)
        _compare(m, b, 1e-5, "one step fp32 state")


def test_masked_initialize_and_edge_sizes():
    b = O.random_batch(257, seed=13)
    m = _gpu_model(b)
    m.initialize()
    m.step(30)
    mask = torch.zeros(257, dtype=torch.bool)
    mask[::3] = True
    X_before = m.X.clone()
    m.initialize(mask=mask.cuda())
    torch.cuda.synchronize()
    keep = ~mask.cuda()
    assert torch.equal(m.X[:, keep], X_before[:, keep])
    assert int(m.k[mask.cuda()].abs().max()) == 0
    # zero-size batch is a no-op
    from b747_rl_ctrl_amd import BatchModel
    z = BatchModel(0)
    z.step(3)


def test_config1_scenario_matches_faithful_trajectory():
    """core/model.py:270-279 main(): state0=[100,1000,300,0,0,0], CS PID off, hzh=2000,
    P=300000, vartheta=-0.1 -- 2000 steps, every read-out compared with the faithful oracle."""
    from b747_rl_ctrl_amd import BatchModel
    m = BatchModel(1, use_PID_CS=False, initial_state=[100, 1000, 300, 0, 0, 0])
    m.hzh = 2000
    m.P = 300000
    m.vartheta_zh = -0.1
    consts = O.DEFAULT_CONSTS.copy()
    consts[1] = 300000.0
    ref = O.trajectory(2000, consts=consts, deltaz=0.0, vartheta=-0.1, h_zh=2000.0,
                       flags=O.F_RP | O.F_PID_SS, state0=(100, 1000, 300, 0, 0, 0))
    got = np.zeros_like(ref)
    for s in range(2000):
        m.step(1)
        got[s] = m.sig[:, 0].cpu().numpy()
    assert _rel(got.T, ref.T) <= 1e-6
    assert abs(float(m.time[0]) - 20.0) < 1e-9


def test_nan_state_propagates_and_state_getter_scrubs():
    b = O.random_batch(64, seed=17)
    m = _gpu_model(b)
    m.initialize()
    m.step(3)
    m.X[6, 5] = float("nan")     # Vx of env 5
    m.step(1)
    torch.cuda.synchronize()
    assert torch.isnan(m.sig[:, 5]).any()
    assert not torch.isnan(m.sig[:, 4]).any()
    assert not torch.isnan(m.state).any()        # core/model.py:200 nan_to_num


def test_full_size_invariants_65536():
    """BASELINE config-3 size: size-independent properties (no oracle at this size)."""
    b = O.random_batch(65536, seed=21)
    m = _gpu_model(b)
    m.initialize()
    m.step(200)
    q = m.X[2:6]
    assert float((q.pow(2).sum(0) - 1).abs().max()) < 1e-6      # unit quaternion preserved
    assert torch.all(m.k == 200)
    # determinism + env independence: the second half run alone gives identical bits
    half = 32768
    b2 = O.Batch(half)
    for name in ("state0", "aero_err"):
        setattr(b2, name, np.ascontiguousarray(getattr(b, name)[:, half:]))
    for name in ("flags", "deltaz", "vartheta", "h_zh"):
        setattr(b2, name, np.ascontiguousarray(getattr(b, name)[half:]))
    m2 = _gpu_model(b2)
    m2.initialize()
    m2.step(200)
    torch.cuda.synchronize()
    assert torch.equal(m2.X, m.X[:, half:]) and torch.equal(m2.sig, m.sig[:, half:])


@pytest.mark.parametrize("variant,per_step", [("fast", False), ("faithful", False), ("fast", True)])
def test_config2_4096_envs_step_elevator_2000_steps(variant, per_step):
    """BASELINE configs[1] at full size: 4096 envs, MANUAL (RP on, both PIDs off), default state0,
    held elevator step deltaz = -(1 + i mod 10) deg from t = 0, 2000 steps, against the batched
    oracle on the same inputs (open loop, not chaotic: <= 1e-6 of each signal's range).  per_step: 2000 one-step
    launches (the bench's config-2 line: FAST runs them on the three-wave kernel), else 500 steps per launch."""
    n = 4096
    b = O.Batch(n)
    b.flags[:] = O.F_RP
    dz = -(1 + np.arange(n) % 10) * np.pi / 180
    m = _gpu_model(b, variant)
    _init_both(m, b)
    b.deltaz[:] = dz
    m._deltaz.copy_(torch.from_numpy(dz))
    for chunk in range(4):
        if per_step:
            for _ in range(500):
                m.step(1)
        else:
            m.step(500)
        O.oracle_step(b, 500)
    torch.cuda.synchronize()
    assert torch.all(m.k == 2000) and np.all(b.k == 2000)
    assert _rel(m.sig.cpu().numpy(), b.sig) <= 1e-6
    assert _rel(m.X.cpu().numpy(), b.X) <= 1e-6
