// b747_split.h -- the single-step env kernel with every env split over TWO waves (FAST, kind 3; fp64 or fp32 X storage),
// and the flight / control pieces the two-wave K-step and PPO rollout kernels (b747_ppo_split.h) share with it.
//
// Why two waves: 65,536 envs are exactly one wave per SIMD, and one wave issues at most one instruction per ~4-5
// cycles, pays ~8 cycles for an fp64 op with a scalar operand and ~11 for a dependent one (tools/ubench_valu.hip):
// the RK4 stages of the one-wave kernel keep the VALU only about half busy (profiles/EXPERIMENTS.md).  Here a 512-thread
// workgroup owns 256 envs and each env has a lane in two waves that share a SIMD (waves w and w + 4: measured,
// tools/ubench_simd.hip), so every SIMD runs the flight and the control wave of the same 64 envs.
//
// Round 5: the control wave LEADS (k_env_step_split).  The dependency chain of a step is the flight wave's: stage
// s + 1's air data need stage s's forces.  Everything else reads that chain only two stages late:
//   * the attitude (q0, q3) and altitude h of stage s + 1's input are x_s + c_s dX_s with dq_s = f(w_s, q_s) and
//     dh_s = Vy_s -- stage s's INPUT values, which the flight wave's combine of stage s - 1 produced;
//   * the control stage s reads theta_s and h_s, i.e. the flight wave's stage s - 2;
//   * the read-out (observation, reward, done) reads only the control stage 3's signals.
// So the control wave integrates h, q0 and q3 itself, evaluates the normalised attitude and the ISA atmosphere of
// each flight stage one stage ahead and hands them over (the part of a flight stage that is not its alpha / lookup
// chain), runs its own stages from them, and finishes the read-out while the flight wave is still in its last
// stages.  The flight wave keeps X0, Vx, Vy and w and runs only the chain: air data, alpha, the table lookups, the
// forces and moment, the combine, then posts (Vy, w) of the next stage's input.  Per wave pair the hand-offs are
// LDS progress counters (pair_post / pair_wait), not workgroup barriers:
//   flight:  stage 0 (own attitude / atmosphere) -> [delta_0] -> post (Vy, w)_1 -> [ahead_1] stage 1 -> ... stage 3
//   control: delta table, ahead_1 -> stage 0 -> [(Vy, w)_1] ahead_2 -> stage 1 -> [(Vy, w)_2] ahead_3 -> stage 2
//            -> stage 3 -> read-out, resets -> [(Vy, w)_3] the last combine of h, q0, q3
// The elevator delta the flight wave's moment sees is, for MANUAL control (no SS PID, no dead zone: every env of the
// training configuration), the saturated rate-limiter output -- a function of the stage time and the discrete state
// alone, posted up front (stage 0's first, at issue priority 3, then the other three).  A wave triple holding an env
// whose delta depends on the pitch error of
// the same stage (SS PID, dead zone) posts it per stage instead ("lock step", same code, one more wait per stage).
// Every expression is the one b747::pass / major_step / env_step_lane evaluate for this configuration; the FAST
// unit's FMA contraction may fuse a different product of a sum than in the one-wave kernel (ulp-level;
// tests/test_gpu_split.py).  Lanes past N step a copy of env N-1 and store nothing.
#pragma once

#include "b747_lanes.h"

namespace {

using namespace b747;

constexpr int kSplitEnvs = 256;                 // envs per workgroup
constexpr int kSplitBlock = 2 * kSplitEnvs;     // 4 flight waves + 4 control waves
constexpr int kStepBlock = 3 * kSplitEnvs;      // the per-step kernel: 4 flight, 4 ahead, 4 control waves
constexpr int kNF = 7;                          // flight states (the K-step kernels): X0, X1, X2 (q0), X5 (q3), X6, X7, X8
constexpr int kFX[kNF] = {0, 1, 2, 5, 6, 7, 8};
constexpr int kNC = 9;                          // control states: X9..X17
constexpr uint32_t kSplitSigMask = readout_signal_mask(kSpecObs, kSpecRew, kSpecLimiter);
constexpr int kSplitTbEnd = T_TOTAL;            // the table image part the split kernels stage into LDS (FAST)
constexpr int kSplitTbQ = (kSplitTbEnd - T_FAST_LO + kSplitBlock - 1) / kSplitBlock;   // entries per lane (K-step kernels)

// MIX (B747_VARIANT_MIXED): the flight pass's aerodynamics in fp32 -- ISA on the hardware
// transcendentals, speed and alpha, the table lookups, forces and moment -- while the attitude, the state, the RK4
// combine and the whole control side stay fp64.  Its bilinear records are fp32 {A, B, C, D} (and K_alpha's {A, B}),
// packed two floats per double slot at the start of the image's record region, so that the split kernels' LDS
// staging is the same loop and a record is one ds_read_b128 (the cell grids before them stay fp64: the interval
// index is the FAST one).
constexpr int TF_REC_CYA = 0, TF_REC_DCM = TF_REC_CYA + 4 * B747_CYA_MAX0 * B747_CYA_MAX1,
              TF_REC_MZ = TF_REC_DCM + 4 * B747_DCM_MAX0 * B747_DCM_MAX1,
              TF_REC_CXA = TF_REC_MZ + 4 * B747_MZ_MAX0 * B747_MZ_MAX1,
              TF_REC_KA = TF_REC_CXA + 4 * B747_CXA_MAX0 * B747_CXA_MAX1, TF_TOTAL = TF_REC_KA + 2 * B747_KA_MAX;
static_assert(TF_REC_KA - TF_REC_CYA == T_REC_KA - T_REC_CYA && TF_TOTAL <= 2 * (T_TOTAL - T_REC_CYA),
              "the fp32 records are the fp64 ones, packed");
struct SplitImage {
    double v[T_TOTAL];
};
constexpr SplitImage make_split_image(bool mix)
{
    SplitImage im{};
    for (int j = 0; j < T_TOTAL; ++j) im.v[j] = kTableImage.v[j];
    if (mix) {
        for (int j = T_REC_CYA; j < T_TOTAL; ++j) im.v[j] = 0.0;
        for (int j = 0; j < TF_TOTAL; j += 2) {
            struct P { float a, b; };
            const P pr{(float)kTableImage.v[T_REC_CYA + j], j + 1 < TF_TOTAL ? (float)kTableImage.v[T_REC_CYA + j + 1] : 0.0f};
            im.v[T_REC_CYA + j / 2] = __builtin_bit_cast(double, pr);
        }
    }
    return im;
}
#if defined(__HIPCC__)
__device__
#endif
constexpr SplitImage kSplitImage64 = make_split_image(false);
#if defined(__HIPCC__)
__device__
#endif
constexpr SplitImage kSplitImageMix = make_split_image(true);
template <bool MIX>
__device__ __forceinline__ double split_image(int j) { return MIX ? kSplitImageMix.v[j] : kSplitImage64.v[j]; }

// kfit for kernel bodies (the host pass parses them too; only the device pass runs them)
__host__ __device__ __forceinline__ KPtr split_kfit(int zoff)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return kfit(zoff);
#else
    (void)zoff;
    return nullptr;
#endif
}

// ---------------------------------------------------------------- flight side of one output pass ----
// x: the flight states of the stage input (kFX order).  flight_pre: everything up to the pitching moment's
// elevator term; flight_post / flight_wdot: the moment and the derivatives.
struct FlightPass {
    double q0n, q3n, sth, cth;   // theta = unit_atan2(sth, cth) is the control side's (only it reads theta)
    double ax, ay, mz_aero, mz_gain, mq;
    double M, alpha_deg, qq;
    double alpha, V, CYa, CXa, dCm, Ka;   // exported signals of the pass (the model kernel's read-out; dead elsewhere)
};

// The flight stage's fp64 constants (VALU fp64 instructions on gfx950 take no literal operand: each is an SGPR pair).
struct FlightK {
    double c375, hpi, pi, r2d, tup, t0, lapse, gr, invt0, slo, emid, pmid, rho0, S, P, c_, invm0, g, invIz;
    double dc_w, dc_n, mz_w, mz_n, ka_w, ka_n, cx_w, cx_n;
};
__device__ __forceinline__ FlightK flight_consts()
{
    const Consts &C = kDefaultConsts;
    return FlightK{0.375, 1.5707963267948966, 3.141592653589793, B747_R2D, B747_ISA_TROPO_UP, B747_ISA_T0,
                   B747_ISA_LAPSE, B747_ISA_GAMMA_R, B747_ISA_INV_T0, B747_ISA_STRAT_LO, kExpFitMid, kPowFitMid,
                   B747_ISA_RHO0, C.S, C.P, C.c_, C.inv_m0, C.g, C.inv_Iz,
                   kCellDCm1.invw, kCellDCm1.nlo, kCellMz1.invw, kCellMz1.nlo, kCellKa.invw, kCellKa.nlo,
                   kCellCXa1.invw, kCellCXa1.nlo};
}

// What a stage needs from its input's attitude (q0, q3) and altitude h alone: the normalised quaternion,
// sin / cos theta, and the ISA atmosphere at h (temperature, 1 / speed of sound, density, the dCm table's
// altitude interval).  None of it depends on the stage's velocities.
struct FlightAhead {
    double q0n, q3n, sth, cth, h, T, inva, rho;
    int iDC0;
    float invaf, rhof;   // MIX: 1 / a and rho as computed (fp32)
};
// the attitude (b747::pass, FAST, kPitchPlane: q1 = q2 = 0)
__device__ __forceinline__ void pitch_attitude(double q0, double q3, const FlightK &k, FlightAhead &a)
{
    const double q1 = 0.0, q2 = 0.0;
    const double nn = ((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3;
    const double in = rsqrt_pos(nn, k.c375);
    const double q3n = q3 * in, q0n = q0 * in, q2n = 0.0, q1n = 0.0;
    const double s = q2n * q1n + q3n * q0n;
    const double s2 = s + s;
    // cos(asin(s2)) = sqrt((1 - s2)(1 + s2)) >= 0 is |q0n^2 - q3n^2| for the unit pitch-plane quaternion
    // ((q0n^2 - q3n^2)^2 + (2 q0n q3n)^2 = 1): no second rsqrt, a few ulp either way (and better
    // conditioned at 90 deg); NaN still propagates
    const double cth = fabs(q0n * q0n - q3n * q3n);
    a.q0n = q0n; a.q3n = q3n; a.sth = s2; a.cth = cth;
}
template <bool MIX, bool SKIP_STRAT = true>
__device__ __forceinline__ FlightAhead flight_ahead(double q0, double q3, double h, KPtr kf, const FlightK &k)
{
    FlightAhead a;
    a.invaf = a.rhof = 0.0f;
    pitch_attitude(q0, q3, k, a);
  if constexpr (MIX) {
    // ISA in fp32 on the hardware transcendentals: rho = rho0 thr^(EXP - 1) exp(dhc g / (R T)) as exp2 / log2
    // (<= 6e-7 relative over 0-20 km), 1 / a as v_rsq_f32
    const double hc = h > k.tup ? k.tup : maxsd(B747_ISA_TROPO_LO, h);
    const double T = k.t0 - hc * k.lapse;
    a.h = h;
    a.T = T;
    const float Tf = (float)T;
    a.invaf = __builtin_amdgcn_rsqf(Tf * (float)B747_ISA_GAMMA_R);
    a.inva = (double)a.invaf;
    const float thr = Tf * (float)B747_ISA_INV_T0;
    const double dh = k.tup - h;
    const float dhc = (float)(dh > B747_ISA_STRAT_UP ? B747_ISA_STRAT_UP : maxsd(k.slo, dh));
    const float pw = __builtin_amdgcn_exp2f((float)(B747_ISA_EXP - 1.0) * __builtin_amdgcn_logf(thr));
    const float ex = __builtin_amdgcn_exp2f(dhc * ((float)(B747_ISA_G_R * 1.4426950408889634) / Tf));
    a.rhof = ex * (pw * (float)B747_ISA_RHO0);
    a.rho = (double)a.rhof;
  } else {
    // ISA (branch-free: the polynomial at dhc = 0 is finite and discarded)
    static_assert(B747_ISA_H_TROPO == B747_ISA_TROPO_UP && B747_ISA_STRAT_UP == 0.0, "FlightK.tup");
    const double hc = h > k.tup ? k.tup : maxsd(B747_ISA_TROPO_LO, h);
    const double T = k.t0 - hc * k.lapse;
    a.h = h;
    a.T = T;
    a.inva = rsqrt_pos(T * k.gr, k.c375);
    const double thr = T * k.invt0;
    const double dh = k.tup - h;
    const double dhc = dh > B747_ISA_STRAT_UP ? B747_ISA_STRAT_UP : maxsd(k.slo, dh);
    // the stratosphere's exponential only where a lane of the wave is above the tropopause (or NaN): a
    // wave-uniform branch around the degree-12 fit instead of evaluating and discarding it everywhere
    // (round 4: -0.15 us per launch)
    double ex = 1.0;
    if (!SKIP_STRAT || wave_any(!(dh >= 0.0))) {
        const double exf = isa_expfit(dhc, kf, k.emid);
        ex = B747_UNPRED(dhc == 0.0) ? 1.0 : exf;
    }
    a.rho = ex * (isa_powfit(thr, kf, k.pmid) * k.rho0);
  }
    a.iDC0 = bp_index<B747_DCM_MAX0>(kf + KF_DCM0, h);
    return a;
}
template <bool MIX = false, bool SKIP_STRAT = true>
__device__ __forceinline__ FlightAhead flight_ahead(const double *x, KPtr kf, const FlightK &k)
{
    return flight_ahead<MIX, SKIP_STRAT>(x[2], x[3], x[1], kf, k);
}

// The MIX flight pass (B747_VARIANT_MIXED): flight_pre with the aerodynamics in fp32 -- speed and alpha (v_rsq_f32,
// the unit-vector angle with a degree-5 asin series: <= 4.2e-7 rad), the lookups on the packed fp32 records, the
// forces and the moment -- from the fp64 attitude and state; p carries fp64 values for the fp64 combine.
__device__ __forceinline__ void flight_pre_mix(const double *x, const double *tb, KPtr kf, const double *km, FlightPass &p,
                                               const FlightK &k, const FlightAhead &a)
{
    const double q0n = a.q0n, q3n = a.q3n, sth = a.sth, cth = a.cth;
    p.q0n = q0n; p.q3n = q3n; p.sth = sth; p.cth = cth;
    const double Vx = x[4], Vy = x[5];
    const double u = cth * Vx + sth * Vy;
    const double v = cth * Vy - sth * Vx;
    // speed, alpha in fp32 (MIXED): v_rsq_f32 and the unit-vector angle with a degree-5 asin series
    const float uf = (float)u, vf = (float)v;
    const float V2f = uf * uf + vf * vf;
    const float iVf = __builtin_amdgcn_rsqf(V2f);
    const float Vf = V2f > 0.0f ? V2f * iVf : 0.0f * V2f;
    const bool pos = Vf > 0.0f;
    const float saf = pos ? -vf * iVf : -0.0f * vf;
    const float caf = pos ? uf * iVf : 1.0f + 0.0f * uf;
    float alpha_f;
    {
        const float aa = fabsf(saf), bb = fabsf(caf);
        const bool sw = aa > bb;
        const float lo = sw ? bb : aa, hi = sw ? aa : bb;
        const float xx = lo * __builtin_amdgcn_rsqf(2.0f + 2.0f * hi);
        const float z = xx * xx, x2 = xx + xx;
        float P = 231.0f / 13312.0f;
        P = P * z + 63.0f / 2816.0f; P = P * z + 35.0f / 1152.0f; P = P * z + 5.0f / 112.0f;
        P = P * z + 3.0f / 40.0f; P = P * z + 1.0f / 6.0f;
        const float psi = x2 + (x2 * z) * P;
        float phi = sw ? (1.57079632679f - psi) : psi;
        phi = caf < 0.0f ? (3.14159265359f - phi) : phi;
        alpha_f = copysignf(phi, saf);
    }
    const double h = a.h;
    // lookups, forces and moment in fp32 on the packed fp32 records (interval indices as FAST: fp64 compares
    // against the breakpoints and the fp64 cell grids, so an fp32 rounding never picks a neighbouring interval)
    const float adf = alpha_f * (float)B747_R2D;
    const float Mf = Vf * a.invaf;
    const double M = (double)Mf, alpha_deg = (double)adf;
    const int iM = bp_index<B747_CYA_MAX0>(kf + KF_CYA0, M);
    const int iCY1 = bp_index<B747_CYA_MAX1>(kf + KF_CYA1, alpha_deg);
    const int iCX0 = bp_index<B747_CXA_MAX0>(kf + KF_CXA0, M);
    const int iDC0 = a.iDC0;
    const float qqf = a.rhof * V2f;
    p.M = M; p.alpha_deg = alpha_deg; p.qq = (double)qqf;
    const float *fr = reinterpret_cast<const float *>(tb + T_REC_CYA);
    typedef float f4 __attribute__((ext_vector_type(4)));
    auto rec = [&](int o) __attribute__((always_inline)) { return *reinterpret_cast<const f4 *>(fr + o); };
    auto bil = [](const f4 &r, float u0, float u1) __attribute__((always_inline)) {
        return fmaf(fmaf(r[3], u0, r[2]), u1, fmaf(r[1], u0, r[0]));
    };
    sched_fence();
    const f4 rCY = rec(TF_REC_CYA + 4 * (iCY1 * B747_CYA_MAX0 + iM));
    sched_fence();
    const CellRd cDC = cell_read(tb + T_CELL_DCM1, CellGrid{k.dc_w, k.dc_n, kCellDCm1.nc}, M);
    const CellRd cMZ = cell_read(tb + T_CELL_MZ1, CellGrid{k.mz_w, k.mz_n, kCellMz1.nc}, alpha_deg);
    const CellRd cKa = cell_read(tb + T_CELL_KA, CellGrid{k.ka_w, k.ka_n, kCellKa.nc}, alpha_deg);
    sched_fence();
    const float CYa = bil(rCY, Mf, adf) * (float)km[1];
    const double CYad = (double)CYa;
    const CellRd cCX = cell_read(tb + T_CELL_CXA1, CellGrid{k.cx_w, k.cx_n, kCellCXa1.nc}, CYad);
    sched_fence();
    const f4 rDC = rec(TF_REC_DCM + 4 * (cell_idx(cDC, M) * B747_DCM_MAX0 + iDC0));
    const f4 rMZ = rec(TF_REC_MZ + 4 * (cell_idx(cMZ, alpha_deg) * B747_MZ_MAX0 + iM));
    const int iKa = cell_idx(cKa, alpha_deg);
    const float kaA = fr[TF_REC_KA + 2 * iKa], kaB = fr[TF_REC_KA + 2 * iKa + 1];
    sched_fence();
    const f4 rCX = rec(TF_REC_CXA + 4 * (cell_idx(cCX, CYad) * B747_CXA_MAX0 + iCX0));
    sched_fence();
    const float CXa = bil(rCX, Mf, CYa) * (float)km[0];
    const float qS = qqf * (float)(B747_F_HALF * B747_DEF_S);
    const float D = (float)B747_F_NEG * CXa * qS;
    const float L = qS * CYa;
    const float Fy = (caf * L - D * saf) + 0.0f;
    const float Fx = (D * caf + saf * L) + (float)B747_DEF_P;
    const float cthf = (float)cth, sthf = (float)sth;
    const float im0 = (float)(1.0 / B747_DEF_M0);
    p.ax = (double)((Fx * cthf - sthf * Fy) * im0);
    p.ay = (double)((Fy * cthf + Fx * sthf) * im0 - (float)B747_DEF_G);
    const float dCm = bil(rDC, (float)h, Mf) * (float)km[3];
    const float mzv = bil(rMZ, Mf, adf) * (float)km[2];
    const float Ka = fmaf(kaB, adf, kaA) * (float)km[4];
    p.mq = (double)(qqf * (float)(B747_M_HALF * B747_DEF_S * B747_DEF_C));
    p.mz_gain = (double)((float)B747_R2D * dCm * Ka);
    p.mz_aero = (double)mzv;
    (void)k;
}

// a: flight_ahead of this stage's input x (kFX layout; only Vx = x[4] and Vy = x[5] are read)
template <bool MIX = false>
__device__ __forceinline__ void flight_pre(const double *x, const double *tb, KPtr kf, const double *km, FlightPass &p,
                                           const FlightK &k, const FlightAhead &a)
{
    if constexpr (MIX) {
        flight_pre_mix(x, tb, kf, km, p, k, a);
        return;
    }
    const double q0n = a.q0n, q3n = a.q3n, sth = a.sth, cth = a.cth;
    p.q0n = q0n; p.q3n = q3n; p.sth = sth; p.cth = cth;
    // air data
    const double Vx = x[4], Vy = x[5];
    const double u = cth * Vx + sth * Vy;
    const double v = cth * Vy - sth * Vx;
    const double V2 = u * u + v * v;
    const double iV = rsqrt_pos(V2, k.c375);
    const double V = V2 > 0.0 ? V2 * iV : 0.0 * V2;
    const bool pos = V > 0.0;
    const double sa = pos ? -v * iV : -0.0 * v;
    const double ca = pos ? u * iV : 1.0 + 0.0 * u;
    const double alpha = unit_atan2(sa, ca, kf, k.hpi, k.pi, k.c375);
    const double h = a.h;
    const double alpha_deg = alpha * k.r2d;
    const double M = V * a.inva;
    const double rho = a.rho;
    // Lookups in LDS round trips that do not wait on each other (the critical chain is CYa -> CXa -> forces;
    // the moment's lookups are off it).  Every scalar breakpoint compare comes first, so their scalar loads
    // (lgkmcnt, like LDS) are complete before any LDS read is in flight; then
    //   trip 1: CYa's record + the three cell reads (dCm over M, mz and K_alpha over alpha);
    //   trip 2: CXa's cell (from CYa) + the dCm / mz / K_alpha records;   trip 3: CXa's record.
    const int iM = bp_index<B747_CYA_MAX0>(kf + KF_CYA0, M);
    const int iCY1 = bp_index<B747_CYA_MAX1>(kf + KF_CYA1, alpha_deg);
    const int iCX0 = bp_index<B747_CXA_MAX0>(kf + KF_CXA0, M);
    const int iDC0 = a.iDC0;
    p.M = M; p.alpha_deg = alpha_deg; p.qq = rho * V2;
    sched_fence();
    const BFetch fCY = bilin_fetch<B747_CYA_MAX0>(tb, T_REC_CYA, iM, iCY1);
    sched_fence();
    const CellRd cDC = cell_read(tb + T_CELL_DCM1, CellGrid{k.dc_w, k.dc_n, kCellDCm1.nc}, M);
    const CellRd cMZ = cell_read(tb + T_CELL_MZ1, CellGrid{k.mz_w, k.mz_n, kCellMz1.nc}, alpha_deg);
    const CellRd cKa = cell_read(tb + T_CELL_KA, CellGrid{k.ka_w, k.ka_n, kCellKa.nc}, alpha_deg);
    sched_fence();
    const double CYa = bilin(fCY, M, alpha_deg) * km[1];
    const CellRd cCX = cell_read(tb + T_CELL_CXA1, CellGrid{k.cx_w, k.cx_n, kCellCXa1.nc}, CYa);
    sched_fence();
    const BFetch fDC = bilin_fetch<B747_DCM_MAX0>(tb, T_REC_DCM, iDC0, cell_idx(cDC, M));
    const BFetch fMZ = bilin_fetch<B747_MZ_MAX0>(tb, T_REC_MZ, iM, cell_idx(cMZ, alpha_deg));
    const int iKa = cell_idx(cKa, alpha_deg);
    const double kaA = tb[T_REC_KA + 2 * iKa], kaB = tb[T_REC_KA + 2 * iKa + 1];
    sched_fence();
    const BFetch fCX = bilin_fetch<B747_CXA_MAX0>(tb, T_REC_CXA, iCX0, cell_idx(cCX, CYa));
    sched_fence();
    const double CXa = bilin(fCX, M, CYa) * km[0];
    const double qq = rho * V2;
    const double qS = qq * B747_F_HALF * k.S;
    const double D = B747_F_NEG * CXa * qS;
    const double L = qS * CYa;
    const double Fy = (ca * L - D * sa) + 0.0;
    const double Fx = (D * ca + sa * L) + k.P;
    p.ax = (Fx * cth - sth * Fy) * k.invm0;
    p.ay = (Fy * cth + Fx * sth) * k.invm0 - k.g;
    const double dCm = bilin(fDC, h, M) * km[3];
    const double mzv = bilin(fMZ, M, alpha_deg) * km[2];
    const double Ka = fma(kaB, alpha_deg, kaA) * km[4];
    p.mq = qq * B747_M_HALF * k.S * k.c_;
    static_assert(B747_M_R2D == B747_R2D, "FlightK.r2d");
    p.mz_gain = k.r2d * dCm * Ka;
    p.mz_aero = mzv;
    p.alpha = alpha; p.V = V; p.CYa = CYa; p.CXa = CXa; p.dCm = dCm; p.Ka = Ka;
}

// wdot of the stage for the elevator delta
__device__ __forceinline__ double flight_wdot(double delta, const FlightPass &p, const FlightK &k)
{
    return (p.mz_gain * (delta * B747_GAIN_DELTA) + p.mz_aero) * p.mq * k.invIz;
}
// The attitude's derivatives (q0, q3) from the stage input's w and normalised quaternion
__device__ __forceinline__ double dq0_of(double w, double q3n) { const double nw = -w; return nw * q3n * 0.5; }
__device__ __forceinline__ double dq3_of(double w, double q0n) { return q0n * w * 0.5; }

// dX of the flight states (kFX order) for the elevator delta
__device__ __forceinline__ void flight_post(const double *x, double delta, const FlightPass &p, double *dX, const FlightK &k)
{
    const double wdot = flight_wdot(delta, p, k);
    const double w = x[6];
    dX[0] = x[4];
    dX[1] = x[5];
    dX[2] = dq0_of(w, p.q3n);
    dX[3] = dq3_of(w, p.q0n);
    dX[4] = p.ax;
    dX[5] = p.ay;
    dX[6] = wdot;
}

// --------------------------------------------------------------- control side of one output pass ----
// Rate limiter + saturation (the actuator after the held DSS output), b747::pass "actuator"
__device__ __forceinline__ void actuator(double t, const PassRef &R, double &r, double &dRP)
{
    const double dtl = t - R.t_ref;
    const double du = R.y_dss - R.rl_prevY;
    const double rise = dtl * B747_RATE_RISE, fall = dtl * B747_RATE_FALL;
    const double up = rise + R.rl_prevY, dn = fall + R.rl_prevY;
    const double r_lim = B747_UNPRED(du > rise) ? up : (B747_UNPRED(fall > du) ? dn : R.y_dss);
    r = R.has_ref ? r_lim : R.y_dss;
    dRP = sat(r, B747_SAT4_LO, B747_SAT4_UP);
}

// x: X9..X17 of the stage input; theta, h: the flight side's; returns delta; dX9..dX17 and o
__device__ __forceinline__ double control_pass(const double *x, double t, double theta, double h, const Params &P,
                                               const PassRef &R, double *dX, PassOut &o, double &thPID)
{
    const Consts &C = kDefaultConsts;
    double r, dRP;
    actuator(t, R, r, dRP);
    const double X9 = x[0], X10 = x[1], X11 = x[2], X12 = x[3];
    const double eh = P.h_zh - h;
    const double NpCS = (eh * C.PID_CS[2] - X10) * C.PID_CS[3];
    const double sumCS = eh * C.PID_CS[0] + X9 + NpCS;
    thPID = sat(sumCS, B747_CS_LO, B747_CS_UP);
    const double thref = (P.flags & F_PID_CS) ? thPID : P.vartheta;
    const double e = thref - theta;
    const double NpSS = (e * C.PID_SS[2] - X12) * C.PID_SS[3];
    const double sumSS = e * C.PID_SS[0] + X11 + NpSS;
    const double UPID = sat(sumSS, B747_SS_LO, B747_SS_UP);
    double Ucom;
    if (P.flags & F_RL) Ucom = (B747_RL_DEADZONE > fabs(0.0 - UPID)) ? 0.0 : UPID;
    else if (P.flags & F_PID_SS) Ucom = UPID;
    else Ucom = P.deltaz;
    const double ieSS = C.PID_SS[1] * e;
    const double ieCS = eh * C.PID_CS[1];
    const uint32_t a3 = and3(sumSS * B747_AW_ZEROGAIN, deadzone(sumSS, B747_SS_LO, B747_SS_UP), ieSS) |
                        (and3(sumCS * B747_AW_ZEROGAIN, deadzone(sumCS, B747_CS_LO, B747_CS_UP), ieCS) << 1);
    const double idt = R.has_ref ? (t - R.t_ref > 0.0075 ? 100.0 : 200.0) : 0.0;
    const double ed = R.has_ref ? (e - R.e_ref) * idt : 0.0;
    const double edd = R.has_ref ? (ed - R.ed_ref) * idt : 0.0;
    const double se = e * e;
    const double ae = fabs(e);
    dX[0] = (R.mem & 2u) ? B747_AW_ZERO : ieCS;
    dX[1] = NpCS;
    dX[2] = (R.mem & 1u) ? B747_AW_ZERO : ieSS;
    dX[3] = NpSS;
    dX[4] = e;
    dX[5] = ae * t;
    dX[6] = ae;
    dX[7] = se;
    dX[8] = se * t;
    o.e = e; o.ed = ed; o.edd = edd; o.r = r; o.Ucom = Ucom; o.UPID = UPID; o.and3_bits = a3;
    return (P.flags & F_RP) ? dRP : Ucom;
}

// The part of the delay history a MAJOR step at counter k reads (b747_dynamics.h delay_out: entries k-4, k-3, k-2 of
// the ring, i.e. slots k & 3, (k + 1) & 3, (k + 2) & 3 of disc[5..8]).  Slot (k + 3) & 3, U_com of step k - 1, is
// first read by step k + 1, so the per-step kernel neither loads it nor keeps the four slots' select trees.
struct Hist3 {
    double u4, u3, u2;   // U_com of MAJOR steps k - 4, k - 3, k - 2
};
__device__ __forceinline__ Hist3 load_hist3(const double *disc, int64_t n, int64_t i, uint32_t k)
{
    return Hist3{disc[(int64_t)(5u + (k & 3u)) * n + i], disc[(int64_t)(5u + ((k + 1u) & 3u)) * n + i],
                 disc[(int64_t)(5u + ((k + 2u) & 3u)) * n + i]};
}
// delay_out(k, u_hist) on those three entries: the same operations, hist_get(u_hist, j) and hist_get(u_hist, j - 1)
// being entries k - 3 / k - 4 or k - 2 / k - 3 (bit-identical)
__device__ __forceinline__ double delay_out3(uint32_t k, const Hist3 &u)
{
#pragma clang fp contract(off)
    const double tmd = t_of(k) - B747_DELAY;
    const bool back3 = k >= 3u && t_of(k - 3u) >= tmd;
    const uint32_t j = back3 ? k - 3u : k - 2u;
    const bool j0 = j == 0u;
    const double t2 = t_of(j), u2 = back3 ? u.u3 : u.u2;
    const double t1 = j0 ? 0.0 : t_of(j - 1u);
    const double u1 = j0 ? B747_DELAY_INIT : (back3 ? u.u4 : u.u3);
    const double f1 = (t2 - tmd) / (t2 - t1), f2 = 1.0 - f1;
    const double v = (t2 == t1) ? (tmd >= t2 ? u2 : u1) : u2 * f2 + f1 * u1;
    return (0.0 < tmd) ? v : B747_DELAY_INIT;
}

// delta of the four RK4 stages of the step at counter k from the discrete state at its start, for flags without the
// SS PID or its dead zone (D: x_dss / rl_prevY after the previous step's MAJOR update, y_dss before this step's DSS
// update; ud: the delay output of the step): the actuator at each stage time, stage 0 on the step's start state,
// stages 1-3 after the MAJOR update (PrevY = r of stage 0 at time t_k); stages 1 and 2 share the time t_k + h/2
__device__ __forceinline__ void delta_table(uint32_t k, const Disc &D, double ud, double *d)
{
    const double tk = t_of(k);
    const double tnew = (double)(k + 1u) * H;
    const double temp = 0.5 * H;
    const bool dss_hit = (k % 5u) == 0u;
    PassRef R{};
    R.has_ref = (k != 0u);
    R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
    R.rl_prevY = D.rl_prevY;
    R.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
    double r0, d0, r1, d1, r3, d3;
    actuator(tk, R, r0, d0);
    PassRef R1 = R;
    R1.has_ref = true; R1.t_ref = tk; R1.rl_prevY = r0;
    actuator(temp + tk, R1, r1, d1);
    actuator(tnew, R1, r3, d3);
    d[0] = d0; d[1] = d1; d[2] = d1; d[3] = d3;
}
__device__ __forceinline__ void delta_table(uint32_t k, const Disc &D, double *d)
{
    delta_table(k, D, delay_out(k, D.u_hist), d);
}

// ------------------------------------------------------------- flight/control pair hand-offs ----
// Only flight wave w and control wave w + 4 -- the pair that shares a SIMD and the same 64 envs -- exchange data,
// through a progress counter in LDS per pair instead of workgroup barriers (which would also wait for the other
// three pairs).  A wave's LDS operations are performed in order (AMDGPUUsage, memory model gfx942/gfx950: the LDS
// request queue orders one wave's operations; only different waves' may reorder), so a post is a plain LDS store
// after the data's stores and a wait a polled LDS load before the data's loads; compiler fences keep that order in
// the code, and no s_waitcnt is forced on either side.
__device__ __forceinline__ void pair_post(unsigned *f, unsigned v)
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
template <int SLEEP>
__device__ __forceinline__ void pair_wait(unsigned *f, unsigned v)
{
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < v) {
        if (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// pair_wait remembering the last value read (wave-uniform, in an SGPR): a counter that is already known to be far
// enough costs no LDS round trip (the delta table posts all four stages at once; the ahead wave runs stages ahead)
__device__ __forceinline__ void pair_wait_seen(unsigned *f, unsigned v, unsigned &seen)
{
    while (seen < v) seen = __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ------------------------------------------------------------------------------------ the kernel ----
// One ControllerEnv.step (sample_time = dt: one DLL step) of the reference's training configuration
// (kind 3, DEFC) for every env; the per-step API's K1 case of k_env_steps.  XT: the storage type of the
// continuous state X (double, or float where the batch stores it in fp32: loaded into fp64 registers,
// rounded once by the store, as k_env_steps<float, ...>).
// Three waves per 64 envs, sharing a SIMD (waves w, w + 4, w + 8 of the workgroup):
//   flight  the air data / alpha / table-lookup / force chain of the four RK4 stages and the RK4 of X0..X8;
//   ahead   h, q0, q3 of stage s + 1 from stage s's input (the flight combine of stage s - 1: one stage of slack),
//           and that stage's attitude and atmosphere for the flight wave (round 4 ran it on the control wave, where it
//           competed with the control stages for the same instruction stream: 9.59-9.81 against 9.24-9.33 us);
//   control the controller and X9..X17, the read-out, the resets.
// Diagnostic stamps (-DB747_STAMPS, tools/exp_stamps_split.py --roles 3): 0 start (realtime), 1 tables staged, 2-5
// end of the wave's stage 0-3, 6 control: read-out done / flight: stores issued, 7 end (realtime), 15 the table
// barrier (realtime); flight 8-10 stage 1-3's ahead values arrived, 11-14 stage 0-3's delta arrived; ahead 8-10
// stage 1-3's values posted; control 11 read-out arithmetic done.
constexpr int kAheadF = 7;   // sin, cos theta, h, 1 / a, rho, q0n, q3n of a stage's input (+ the dCm altitude interval)
// The first arguments are what the waves' first loads address (n and six of the batch's pointers, 14 dwords): with
// -mllvm -amdgpu-kernarg-preload-count=14 (build.py) the dispatch places them in SGPRs, so the state loads issue
// without waiting for the argument segment's scalar loads (measured 0.64 us median from wave start, round 5).
constexpr int kStepPreloadDwords = 14;
template <typename XT, bool MIX = false, int ENVS = kSplitEnvs>
__global__ __launch_bounds__(3 * ENVS) B747_NO_FMAC void k_env_step_split(
    int64_t n, const void *xv, const double *aero_err, const uint32_t *kv, const double *disc, const uint8_t *flagsv,
    const float *actions, b747_env_batch b, b747_env_config cfgc, float *obs_seq, float *reward_seq, uint8_t *done_seq)
{
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double xa[3][kAheadF][ENVS];   // ahead -> flight, control: attitude and atmosphere of stages 1-3
    __shared__ int xai[3][ENVS];              // ahead -> flight: the dCm altitude interval of stages 1-3
    __shared__ double xp[2][2][ENVS];         // flight -> ahead: Vy, w of the input of stages 1-2
    __shared__ double xdl[4][ENVS];           // control -> flight: delta per stage
    __shared__ double xa0[3][ENVS];           // ahead -> control: sin, cos theta and h of stage 0's input
    constexpr int kTriples = ENVS / 64;             // wave triples per workgroup
    __shared__ unsigned c_ah[kTriples], c_fl[kTriples], c_dl[kTriples];   // per triple: ahead stages posted, flight
                                                                          // combines, deltas
    __shared__ unsigned c_a0[kTriples];             // per wave triple: stage 0's attitude posted (xa0)
    const int wv = (threadIdx.x >> 6) & (kTriples - 1);   // the triple (waves wv, wv + kTriples, wv + 2 kTriples)
    const int role = (int)threadIdx.x / ENVS;       // 0 flight, 1 ahead, 2 control (wave-uniform)
    // The batch's reads arrive at each XCD's fabric rate (≈2 us for its 2.25 MB, profiles/EXPERIMENTS.md), in the order the
    // waves issue them: the control wave, which ends every workgroup, issues first, the flight wave second, until
    // their state loads are out (measured: -0.15 us per step with the control wave's late loads below)
    if (role == 2) __builtin_amdgcn_s_setprio(3);
    else if (role == 0) __builtin_amdgcn_s_setprio(2);
    B747_STAMP(0, true);
    // the argument segment: n and six pointers (56 B), actions (8), b, cfgc, then three pointers (24); both structs
    // are 8-byte multiples, so no padding lies between
    static_assert(sizeof(b747_env_batch) % 8 == 0 && sizeof(b747_env_config) % 8 == 0, "argument layout");
    unsigned kpd = prefetch_kernargs_issue<64 + sizeof(b747_env_batch) + sizeof(b747_env_config) + 24>();
#if defined(__HIP_DEVICE_COMPILE__)
    prefetch_const_lines<sizeof(FitCoefs)>(split_kfit(0), kpd);
#endif
    const int el = threadIdx.x & (ENVS - 1);
    const int64_t i = (int64_t)blockIdx.x * ENVS + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    EnvCfg cfgk = cfgc;
    spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    if (threadIdx.x < kTriples) { c_ah[threadIdx.x] = 0u; c_fl[threadIdx.x] = 0u; c_dl[threadIdx.x] = 0u; c_a0[threadIdx.x] = 0u; }
    // Only the flight waves read the tables, so only they stage them (this variant's part of the image, <= 3 entries
    // per lane): table loads first, then the state loads, the LDS writes waiting for the table loads alone.  No global
    // load is in flight where the roles' code paths split -- the compiler's wait-count analysis joins the paths, and a
    // load pending there made the role laid out later wait for it before issuing its own (measured: the flight
    // wave's state loads a full memory latency late) -- and the other roles reach the barrier without waiting for
    // any of their loads.
    constexpr int lo = T_FAST_LO, hi = kSplitTbEnd;
    constexpr int kTbQ = (hi - lo + ENVS - 1) / ENVS;   // entries per flight lane
    auto prologue_barrier = [&]() __attribute__((always_inline)) {
        // (a scheduling wall: the compiler would otherwise hoist arithmetic on the first loaded values above the
        // barrier, making every wave wait for its first state load before the workgroup can start)
        prefetch_kernargs_wait(kpd);                            // (the rest of the argument segment)
#ifdef B747_STAMPS
        if (role == 2) B747_STAMP(12, true);                    // (control: the argument segment has arrived)
#endif
        sched_fence();
        wg_barrier();                                           // the tables and the counters before anyone uses them
        sched_fence();
        B747_STAMP(15, true);
        B747_STAMP(1);
    };
    const XT *Xg = (const XT *)xv;
    XT *Xw = (XT *)b.X;
    const double temp = 0.5 * H;
    const double t6 = H / 6.0;

    auto table_loads = [&](double *tv) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < kTbQ; ++q) {
            const int jq = lo + el + q * ENVS;
            tv[q] = (jq < hi) ? split_image<MIX>(jq) : 0.0;
        }
    };
    auto stage_tables = [&](const double *tv) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < kTbQ; ++q) {
            const int jq = lo + el + q * ENVS;
            if (jq < hi) tb[jq] = tv[q];
        }
    };
    if (role == 0) {
        // ---- flight wave
        double tv[kTbQ];
        table_loads(tv);
        double x[kNF], y[kNF], acc[kNF];                        // stage input / base state / accumulator (kFX order)
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        double km[5];                                           // 1 + aero_err
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        __builtin_amdgcn_s_setprio(0);
        stage_tables(tv);
        prologue_barrier();
        // k decides only whether the step ends the episode (the stores at the end): loaded after the barrier, out of
        // the launch's read burst (-0.05 us; the aero multipliers, read mid stage 0, measured slower loaded late)
        const uint32_t k = kv[il];
        const FlightK fk = flight_consts();
#pragma unroll
        for (int j = 0; j < kNF; ++j) { y[j] = x[j]; acc[j] = 0.0; }
        FlightAhead a = flight_ahead<MIX>(x, split_kfit(0), fk);   // stage 0: its own attitude and atmosphere
        unsigned seen_ah = 0u, seen_dl = 0u;
        auto take_ahead = [&](int s1) __attribute__((always_inline)) {   // stage s1's values, from the ahead wave
            pair_wait_seen(&c_ah[wv], (unsigned)s1, seen_ah);
            FlightAhead an;
            an.sth = xa[s1 - 1][0][el]; an.cth = xa[s1 - 1][1][el]; an.h = xa[s1 - 1][2][el];
            an.inva = xa[s1 - 1][3][el]; an.rho = xa[s1 - 1][4][el];
            an.q0n = xa[s1 - 1][5][el]; an.q3n = xa[s1 - 1][6][el];
            an.iDC0 = xai[s1 - 1][el];
            an.invaf = (float)an.inva; an.rhof = (float)an.rho;  // (MIX: exactly the fp32 values)
            return an;
        };
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));                     // as major_step: each stage re-derives its constant pointers
#endif
            if (st > 0) {
                a = take_ahead(st);
                B747_STAMP(7 + st);
            }
            FlightPass fp{};
            flight_pre<MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, a);
            pair_wait_seen(&c_dl[wv], (unsigned)st + 1u, seen_dl);   // delta of this stage (all four at once unless lock step)
            B747_STAMP(11 + st);
            double dX[kNF];
            flight_post(x, xdl[st][el], fp, dX, fk);
            const double c = (st == 2) ? H : temp;              // RK4 combine (b747::major_step, dll@0x2c60)
            const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
            for (int j = 0; j < kNF; ++j) {
                acc[j] = acc[j] + wm * dX[j];
                x[j] = c * dX[j] + y[j];
            }
            if (st < 2) {                                       // the next stage input's Vy and w, to the ahead wave
                xp[st][0][el] = x[5];
                xp[st][1][el] = x[6];
                pair_post(&c_fl[wv], (unsigned)st + 1u);
            }
            B747_STAMP(2 + st);
        }
        // an env that ends its episode in this step is reset by the control wave, which stores its whole state
        const bool rs = cfg.auto_reset && t_of(k + 1u) >= cfg.tk;   // (EnvReadOut's done of the kind-3 read-out)
        if (valid && !rs) {
#pragma unroll
            for (int j = 0; j < kNF; ++j) st_state(&Xw[kFX[j] * n + i], (XT)(acc[j] * t6 + y[j]));
        }
        B747_STAMP(6);
        B747_STAMP(7, true);
        return;
    }

    if (role == 1) {
        // ---- ahead wave: stage st + 1's input h, q0, q3 from stage st's derivatives (flight_post's expressions: the
        // stage input's Vy, w and attitude), then its attitude and atmosphere for the flight wave
        double xq[3] = {(double)Xg[1 * n + il], (double)Xg[2 * n + il], (double)Xg[5 * n + il]};   // h, q0, q3
        double vy = (double)Xg[7 * n + il], w = (double)Xg[8 * n + il];                         // stage 0's Vy, w
        prologue_barrier();
        const FlightK fk = flight_consts();
        const double yq[3] = {xq[0], xq[1], xq[2]};
        FlightAhead at;
        pitch_attitude(xq[1], xq[2], fk, at);
        // stage 0's attitude and h for the control wave, which then neither loads X1, X2, X5 (that the flight wave
        // overwrites at its end) nor evaluates the attitude itself
        xa0[0][el] = at.sth; xa0[1][el] = at.cth; xa0[2][el] = xq[0];
        pair_post(&c_a0[wv], 1u);
        int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(zoff));
#endif
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            if (st > 0) {                                       // stage st's input Vy, w from the flight wave's combine
                pair_wait<0>(&c_fl[wv], (unsigned)st);
                vy = xp[st - 1][0][el];
                w = xp[st - 1][1][el];
            }
            const double dq[3] = {vy, dq0_of(w, at.q3n), dq3_of(w, at.q0n)};
            const double c = (st == 2) ? H : temp;
#pragma unroll
            for (int q = 0; q < 3; ++q) xq[q] = c * dq[q] + yq[q];
            at = flight_ahead<MIX>(xq[1], xq[2], xq[0], split_kfit(zoff), fk);
            xa[st][0][el] = at.sth; xa[st][1][el] = at.cth; xa[st][2][el] = at.h;
            xa[st][3][el] = at.inva; xa[st][4][el] = at.rho; xa[st][5][el] = at.q0n; xa[st][6][el] = at.q3n;
            xai[st][el] = at.iDC0;
            pair_post(&c_ah[wv], (unsigned)st + 1u);
            B747_STAMP(8 + st);
        }
        B747_STAMP(7, true);
        return;
    }

    // ---- control wave: the controller and X9..X17, the read-out, the resets
    // before the barrier only what the delta table needs (k, x_dss, y_dss, rl_prevY, flags, the action)
    const uint32_t k = kv[il];
    Disc D;
    D.x_dss = disc[0 * n + il];                                 // (read on the 0.05 s tick only, but loading it
                                                                //  under that condition measured slower: a branch)
    D.y_dss = disc[1 * n + il];
    D.rl_prevY = disc[2 * n + il];
    const uint32_t flags = flagsv[il];
    const float a = actions[il];
    double x[kNC], y[kNC], acc[kNC];                            // X9..X17: stage input / base state / RK4 accumulator
    __builtin_amdgcn_s_setprio(0);
    prologue_barrier();
    // what the control stages need but the delta table does not -- e_prev, ed_prev and X9..X17, 88 B of every env --
    // issued after the barrier: the launch's read burst then carries the data every wave's first computation waits
    // for (the flight wave's state, the delta table's inputs) ahead of them (measured: -0.11 us per step,
    // profiles/r06/ab_step_kernel.txt)
    D.e_prev = disc[3 * n + il];
    D.ed_prev = disc[4 * n + il];
#pragma unroll
    for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
    // the loads whose pointers are not among the preloaded arguments: issued after the barrier, so that waiting for
    // the argument segment does not hold the control wave's arrival at it
    uint32_t mem = b.mem[il];
    const double ref0 = b.ref[il];
    double h_zh = b.h_zh[il];
    double ep_ret = (double)b.ep_return[il];
    sched_fence();                                              // (nothing k-dependent above these loads: the scheduler
                                                                //  hoisted k & 3 there, whose wait for k's round trip held
                                                                //  their issue by ~1,400 cycles; -0.05 us)
    // the delay history last: its addresses need k (a load issued before the barrier would hold this wave's arrival
    // there for k's round trip), and only the 0.05 s DSS tick reads it, so no wait for the loads above waits for it
    const Hist3 uh = load_hist3(disc, n, il, k);
#ifdef B747_STAMPS
    asm volatile("" ::"v"(k), "v"(D.x_dss), "v"(D.y_dss), "v"(D.rl_prevY), "v"(flags), "v"(a));
    B747_STAMP(14);                                             // (diagnostic: the delta table's inputs have landed)
#endif
    // delta of a stage depends on that stage's pitch error (SS PID, dead zone): then this triple posts it per stage
    const bool lock = wave_any((flags & (F_PID_SS | F_RL)) != 0u);   // wave-uniform
    // controller (core/controller.py:231-264 as env_step_lane; kind 3: MANUAL/DIRECT, CONST refs)
    const bool ctrl0 = (flags & F_PID_CS) != 0u;
    const double tk = t_of(k);
    const double tnew = (double)(k + 1u) * H;
    const bool dss_hit = (k % 5u) == 0u;
    const uint32_t mem_held = mem;
    const bool use_ctrl = (flags & F_PID_CS) != 0u;
    const bool manual = (flags & F_PID_SS) == 0u;
    const double vartheta = use_ctrl ? 0.0 : ref0;             // pitch_ref of a CONST reference
    h_zh = use_ctrl ? (double)0.0f : h_zh;                      // ref[7] is not loaded in kind 3 (as env_load)
    // major_step: delay / DSS
    // the delay output feeds only the DSS, on its 0.05 s tick: a wave without a ticking lane (4 steps of 5 in lock
    // step) neither computes it nor waits for the history's loads, and posts its delta table at once
    double ud = 0.0;
    if (wave_any(dss_hit)) {
        ud = delay_out3(k, uh);
        D.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
    }
    if (!lock) {
        // stage 0's delta first (the flight wave's stage 0 waits for it; stage 1 reads the rest ~2,400 cycles later):
        // delta_table's expressions, posted in two parts
        const bool rp = (flags & F_RP) != 0u;
        const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
        const double dz = manual ? (double)a32 : 0.0;
        PassRef R0{};
        R0.has_ref = (k != 0u);
        R0.t_ref = R0.has_ref ? t_of(k - 1u) : 0.0;
        R0.rl_prevY = D.rl_prevY;
        R0.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
        double r0, d0, r1, d1, r3, d3;
        __builtin_amdgcn_s_setprio(3);                          // (the SIMD's three waves all issue here: the control
                                                                //  wave first until stage 0's delta is out, -0.06 us)
        actuator(tk, R0, r0, d0);
        xdl[0][el] = rp ? d0 : dz;
        pair_post(&c_dl[wv], 1u);
        __builtin_amdgcn_s_setprio(0);
        sched_fence();
        PassRef R1 = R0;
        R1.has_ref = true; R1.t_ref = tk; R1.rl_prevY = r0;
        actuator(0.5 * H + tk, R1, r1, d1);
        actuator(tnew, R1, r3, d3);
        xdl[1][el] = rp ? d1 : dz;
        xdl[2][el] = rp ? d1 : dz;
        xdl[3][el] = rp ? d3 : dz;
        pair_post(&c_dl[wv], 4u);
        B747_STAMP(13);
    }
    FlightAhead att[4];                                         // attitude of each stage's input (the ahead wave's)
    double hst[4];                                              // and its h
    {
        unsigned seen_a0 = 0u;
        pair_wait_seen(&c_a0[wv], 1u, seen_a0);
        att[0].sth = xa0[0][el];
        att[0].cth = xa0[1][el];
        hst[0] = xa0[2][el];
    }
    // controller and the control stages
    const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
    const double deltaz = manual ? (double)a32 : 0.0;
    Params P{};
    P.deltaz = deltaz; P.vartheta = vartheta; P.h_zh = h_zh; P.flags = flags;
    PassRef R{};
    R.has_ref = (k != 0u);
    R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
    R.e_ref = D.e_prev; R.ed_ref = D.ed_prev; R.rl_prevY = D.rl_prevY;
    R.y_dss = D.y_dss; R.mem = mem;
#pragma unroll
    for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
    PassOut o{};
    double thPID = 0.0;
    SigVals sv{};
    auto cstage = [&](int st, int zoff) __attribute__((always_inline)) {
        const double t = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
        double dX[kNC];
        const double delta = control_pass(x, t, unit_atan2(att[st].sth, att[st].cth, split_kfit(zoff)), hst[st], P, R, dX,
                                          o, thPID);
        if (lock) {
            xdl[st][el] = delta;
            pair_post(&c_dl[wv], (unsigned)st + 1u);
        }
        if (st == 3) {   // the read-out's stage-4 signals (kSplitSigMask)
            sv.v[S_SIM_TIME] = t;
            sv.v[S_DVARTHETA] = o.e;
            sv.v[S_VARTHETA_ZH] = thPID;
            sv.v[S_U_COM_PID] = o.UPID;
            sv.v[S_DVARTHETA_DT] = o.ed;
            sv.v[S_DVARTHETA_DT_DT] = o.edd;
            sv.v[S_ITSE] = x[8];
            sv.v[S_DVARTHETA_INT] = x[4];
        }
        if (st == 0) {   // MAJOR-only updates (dll@0x271a), then only what the step changed is written back
            D.x_dss = dss_hit ? B747_DSS_A * D.x_dss + B747_DSS_B * ud : D.x_dss;
            D.rl_prevY = o.r;
            D.e_prev = o.e;
            D.ed_prev = o.ed;
            mem = o.and3_bits;
            R.has_ref = true; R.t_ref = tk; R.e_ref = o.e; R.ed_ref = o.ed; R.rl_prevY = o.r;
            R.mem = mem_held;
            if (valid) {
                if (dss_hit) {
                    st_state(&b.disc[0 * n + i], D.x_dss);
                    st_state(&b.disc[1 * n + i], D.y_dss);
                }
                st_state(&b.disc[2 * n + i], D.rl_prevY);
                st_state(&b.disc[3 * n + i], D.e_prev);
                st_state(&b.disc[4 * n + i], D.ed_prev);
                st_state(&b.disc[(int64_t)(5u + (k & 3u)) * n + i], o.Ucom);   // (the slot of entry k - 4)
                b.k[i] = k + 1u;
                b.mem[i] = (uint8_t)mem;
            }
        }
        const double c = (st == 2) ? H : temp;                  // RK4 combine of X9..X17
        const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
            acc[j] = acc[j] + wm * dX[j];
            x[j] = c * dX[j] + y[j];
        }
        B747_STAMP(2 + st);
    };
    int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(zoff));
#endif
    // the episode return is read only by the read-out; waiting for its load there would also wait for every store
    // issued before it (one vmcnt for loads and stores): take it where the stage-0 pass waits for X9..X17 (the
    // loads before it) anyway, before the stage's discrete-state stores
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(ep_ret));
#endif
    cstage(0, zoff);
    unsigned seen_ah = 0u;
#pragma unroll
    for (int st = 1; st < 4; ++st) {                            // each stage's attitude from the ahead wave
        pair_wait_seen(&c_ah[wv], (unsigned)st, seen_ah);
        att[st].sth = xa[st - 1][0][el];
        att[st].cth = xa[st - 1][1][el];
        hst[st] = xa[st - 1][2][el];
        cstage(st, zoff);
    }
    // ---- read-out (EnvReadOut of the kind-3 configuration) and episode bookkeeping, from the signals in registers.
    // The arguments from here on are fresh copies of the kernel's: the compiler then loads the fields where they are
    // used instead of keeping the early copies' wide SGPR tuples live through the stages (spilled to VGPR lanes and
    // restored whole at every later use: 177 against 38 v_readlane in this kernel)
    const b747_env_batch bl = b;
    EnvCfg cfgl = cfgc;
    spec_config(cfgl);
    double sgr[sig_rows(kSplitSigMask)];
    SigStash<kSplitSigMask>{sgr, 1}(sv);
    const bool done = sgr[sig_row(kSplitSigMask, S_SIM_TIME)] >= cfgl.tk;
    const bool rs = done && cfgl.auto_reset;                     // (the flight wave decides the same from k)
    if (valid) {
        const int od = bl.obs_dim;
        float *orow = bl.obs + i * od;
        float *orow2 = obs_seq ? obs_seq + i * od : nullptr;
        float *trow = bl.terminal_obs ? bl.terminal_obs + i * od : nullptr;
        EnvReadOut<true, kSplitSigMask> ro{cfgl, flags, deltaz, vartheta, orow, trow, orow2, 0.0, 0.0, 0.0, false};
        ro(sgr, 1);
        const float r32 = (float)ro.reward;
        ep_ret = vecmonitor_add(ep_ret, ro.reward);
        B747_STAMP(11);
        const int32_t ep_len = (int32_t)(k + 1u);               // ceil(k / n_sub) before the step, + 1
        bl.reward[i] = r32;
        bl.done[i] = done ? 1 : 0;
        if (reward_seq) reward_seq[i] = r32;
        if (done_seq) done_seq[i] = done ? 1 : 0;
        if (done) {   // record_episode_end
            if (bl.ep_final_return) bl.ep_final_return[i] = ep_ret;
            if (bl.ep_final_len) bl.ep_final_len[i] = ep_len;
            if (bl.ep_stats) {
                bl.ep_stats[i] += 1.0;
                bl.ep_stats[n + i] += ep_ret;
                bl.ep_stats[2 * n + i] += (double)ep_len;
            }
        }
        bl.ep_return[i] = rs ? 0.0f : (float)ep_ret;   // (exact: VecMonitor's float32 sums)
    }
    B747_STAMP(6);
    if (valid && rs) {
        // env_reset_lane (Controller.reset + Model.initialize) and env_store(slot_params): the env's whole state,
        // the flight wave's X0..X8 included (it stores nothing for a resetting env)
        EnvSlot s{};
        s.episode = bl.episode[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) s.ref[j] = bl.ref[j * n + i];
        s.flags = flags;
        s.ref_kind = REF_CONST;
        double aero[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) aero[j] = bl.aero_err[j * n + i];
        double s0[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) s0[j] = bl.state0 ? bl.state0[j * n + i] : (j == 1 ? 11000.0 : (j == 2 ? 259.1667 : 0.0));
        draw_reset(cfgl, (uint64_t)(bl.env_offset + i), s, s0, aero);
        if (bl.state0 && cfgl.reset_ref_mode != RM_NONE) {
#pragma unroll
            for (int j = 0; j < 6; ++j) bl.state0[j * n + i] = s0[j];
        }
        s.episode += 1u;
        double xi[NX];
        Disc Di;
        uint32_t k0, m0;
        initialize(xi, Di, k0, m0, s0);
#pragma unroll
        for (int j = 0; j < NX; ++j) st_state(&((XT *)bl.X)[j * n + i], (XT)xi[j]);
        store_disc(bl.disc, n, i, Di);
        bl.k[i] = k0;
        bl.mem[i] = (uint8_t)m0;
        bl.deltaz[i] = 0.0;
        bl.upid[i] = 0.0;
        bl.tp[i] = 0.0;
        bl.ep_len[i] = 0;
        bl.vartheta[i] = 0.0;
        bl.h_zh[i] = h_zh;
        bl.flags[i] = (uint8_t)s.flags;
        bl.episode[i] = s.episode;
#pragma unroll
        for (int j = 0; j < 8; ++j) bl.ref[j * n + i] = s.ref[j];
        bl.ref_kind[i] = (uint8_t)s.ref_kind;
#pragma unroll
        for (int j = 0; j < 5; ++j) bl.aero_err[j * n + i] = aero[j];
    } else if (valid) {
#pragma unroll
        for (int j = 0; j < kNC; ++j) st_state(&((XT *)bl.X)[(9 + j) * n + i], (XT)(acc[j] * t6 + y[j]));
        if (ctrl0 || (flags & F_PID_CS)) bl.h_zh[i] = h_zh;
    }
    B747_STAMP(7, true);
}

}  // namespace
