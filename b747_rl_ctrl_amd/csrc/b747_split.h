// b747_split.h -- the single-step env kernel with every env split over TWO waves (FAST, kind 3; fp64 or fp32 X storage).
//
// Why: 65,536 envs are exactly one wave per SIMD, and one wave issues at most one instruction per ~4-5
// cycles, pays ~8 cycles for an fp64 op with a scalar operand and ~11 for a dependent one
// (tools/ubench_valu.hip): the RK4 stages of the one-wave kernel keep the VALU only about half busy
// (DESIGN.md 4).  Here a 512-thread workgroup owns 256 envs and each env has a lane in two waves:
//   flight wave  (waves 0-3) -- attitude, air data, ISA atmosphere, the aerodynamic table lookups, forces
//                               and moment, and the states X0, X1, q0 (X2), q3 (X5), Vx, Vy, wz
//                               (q1 = q2 = 0: kPitchPlane);
//   control wave (waves 4-7) -- actuator (delay, DSS, rate limiter, saturation), both PID loops with
//                               anti-windup, the Derivative blocks, the states X9..X17, the discrete
//                               state, the controller, the read-out and the resets.
// Waves w and w + 4 of a workgroup share a SIMD (measured, tools/ubench_simd.hip), so every SIMD runs the
// flight and the control wave of the same 64 envs.
//
// The flight states never read a control state: the one input the flight side needs, the elevator
// deflection delta the moment equation sees, is for MANUAL control (flags without the SS PID or its
// dead zone, i.e. every env of the training configuration) the saturated rate-limiter output -- a
// function of the stage time and the discrete state alone, known for all four RK4 stages before the
// first one.  So the flight wave runs its four stages back to back and the control wave follows one
// stage behind, fed through LDS with (theta, h) of each stage:
//   iteration j = 0..3:  flight: stage j -> LDS theta[j], h[j]      control: stage j - 1
//   barrier
//   iteration 4:                                                    control: stage 3, read-out
// A workgroup holding an env whose flags put the SS PID (or its dead zone) in the loop -- delta then
// depends on the pitch error of the same stage -- runs the stages in lock step instead: flight
// (everything up to the moment), barrier, control (delta), barrier, flight (moment, combine).
// Every expression is the one b747::pass / major_step / env_step_lane evaluate for this configuration;
// the FAST unit's FMA contraction may fuse a different product of a sum than in the one-wave kernel
// (ulp-level; tests/test_gpu_split.py).  Both roles execute the same barrier sequence; lanes past N step
// a copy of env N-1 and store nothing.
#pragma once

#include "b747_lanes.h"

namespace {

using namespace b747;

constexpr int kSplitEnvs = 256;                 // envs per workgroup
constexpr int kSplitBlock = 2 * kSplitEnvs;     // 4 flight waves + 4 control waves
constexpr int kNF = 7;                          // flight states: X0, X1, X2 (q0), X5 (q3), X6, X7, X8
constexpr int kFX[kNF] = {0, 1, 2, 5, 6, 7, 8};
constexpr int kNC = 9;                          // control states: X9..X17
constexpr uint32_t kSplitSigMask = readout_signal_mask(kSpecObs, kSpecRew, kSpecLimiter);
// the table image part the split kernels stage into LDS (FAST cell grids and records, + the ISA cells)
#ifdef B747_ISA_CELLS
constexpr int kSplitTbEnd = T_TOTAL_ISA;
#else
constexpr int kSplitTbEnd = T_TOTAL;
#endif
constexpr int kSplitTbQ = (kSplitTbEnd - T_FAST_LO + kSplitBlock - 1) / kSplitBlock;   // entries per lane

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
    double v[T_TOTAL_ISA];
};
constexpr SplitImage make_split_image(bool mix)
{
    SplitImage im{};
    for (int j = 0; j < T_TOTAL_ISA; ++j) im.v[j] = kTableImage.v[j];
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
// elevator term; flight_post: the moment and the derivatives.
struct FlightPass {
    double q0n, q3n, sth, cth;   // theta = unit_atan2(sth, cth) is the control side's (only it reads theta)
    double ax, ay, mz_aero, mz_gain, mq;
    double M, alpha_deg, qq;     // the moment's inputs (B747_MOMENT_CTRL: evaluated by the control wave)
};

// The flight stage's fp64 constants.  VALU fp64 instructions on gfx950 take no literal operand, so every
// non-inline constant costs two s_mov_b32 per use site per stage (plus a v_mov where an instruction already
// reads one SGPR): ~35 constants, ~75 SALU + ~40 v_mov issue slots per flight stage.  With B747_FLIGHT_VK
// they are made opaque VGPR values once per launch (registers the flight role has spare) and every stage
// reads them from there; the values and the order of every operation are unchanged (bit-identical).
#ifndef B747_FLIGHT_VK
#define B747_FLIGHT_VK 0
#endif
struct FlightK {
    double c375, hpi, pi, r2d, tup, t0, lapse, gr, invt0, slo, emid, pmid, rho0, S, P, c_, invm0, g, invIz;
    double dc_w, dc_n, mz_w, mz_n, ka_w, ka_n, cx_w, cx_n;
};
template <bool OPAQUE = (B747_FLIGHT_VK != 0)>
__device__ __forceinline__ FlightK flight_consts()
{
    const Consts &C = kDefaultConsts;
    FlightK k{0.375, 1.5707963267948966, 3.141592653589793, B747_R2D, B747_ISA_TROPO_UP, B747_ISA_T0,
              B747_ISA_LAPSE, B747_ISA_GAMMA_R, B747_ISA_INV_T0, B747_ISA_STRAT_LO, kExpFitMid, kPowFitMid,
              B747_ISA_RHO0, C.S, C.P, C.c_, C.inv_m0, C.g, C.inv_Iz,
              kCellDCm1.invw, kCellDCm1.nlo, kCellMz1.invw, kCellMz1.nlo, kCellKa.invw, kCellKa.nlo,
              kCellCXa1.invw, kCellCXa1.nlo};
#if defined(__HIP_DEVICE_COMPILE__)
#define B747_VK_OPAQUE(f) if (OPAQUE) asm volatile("" : "+v"(k.f))
    B747_VK_OPAQUE(c375); B747_VK_OPAQUE(hpi); B747_VK_OPAQUE(pi); B747_VK_OPAQUE(r2d); B747_VK_OPAQUE(tup);
    B747_VK_OPAQUE(t0); B747_VK_OPAQUE(lapse); B747_VK_OPAQUE(gr); B747_VK_OPAQUE(invt0); B747_VK_OPAQUE(slo);
    B747_VK_OPAQUE(emid); B747_VK_OPAQUE(pmid); B747_VK_OPAQUE(rho0); B747_VK_OPAQUE(S); B747_VK_OPAQUE(P);
    B747_VK_OPAQUE(c_); B747_VK_OPAQUE(invm0); B747_VK_OPAQUE(g); B747_VK_OPAQUE(invIz);
    B747_VK_OPAQUE(dc_w); B747_VK_OPAQUE(dc_n); B747_VK_OPAQUE(mz_w); B747_VK_OPAQUE(mz_n);
    B747_VK_OPAQUE(ka_w); B747_VK_OPAQUE(ka_n); B747_VK_OPAQUE(cx_w); B747_VK_OPAQUE(cx_n);
#undef B747_VK_OPAQUE
#endif
    return k;
}

// B747_STAMPS_FLIGHT (diagnostic builds, tools/exp_stamps_split.py --flight): phase stamps inside the stage
// whose call passes stamp_on = true -- 7 start, 13 alpha, 14 the four lookups fetched, 15 end
#ifdef B747_STAMPS_FLIGHT
#define B747_FSTAMP(slot) do { if (stamp_on) B747_STAMP(slot); } while (0)
#else
#define B747_FSTAMP(slot) ((void)0)
#endif
// B747_STAMPS_CHAIN (diagnostic builds, tools/exp_stamps_split.py --chain): readiness probes along the flight
// stage's dependency chain in stage 2 -- a v_mov that reads the value (the in-order wave stalls until it is
// written), then s_memtime into slots 4-15; the kernel's other stamps keep only slot 3 (iteration 2 start).
#if defined(B747_STAMPS) && defined(B747_STAMPS_CHAIN)
__device__ __forceinline__ void probe_ready(double v)
{
    unsigned d;
    asm volatile("v_mov_b32 %0, %1" : "=v"(d) : "v"(__double2hiint(v)));
    asm volatile("" ::"v"(d));
}
#define B747_PROBE(slot, v) do { if (stamp_on) { probe_ready(v); B747_STAMP(slot); } } while (0)
#define B747_MSTAMP(slot, ...) do { if ((slot) == 3) B747_STAMP(slot, ##__VA_ARGS__); } while (0)
#else
#define B747_PROBE(slot, v) ((void)0)
#define B747_MSTAMP(...) B747_STAMP(__VA_ARGS__)
#endif
// What a stage needs from its input's attitude (q0, q3) and altitude h alone: the normalised quaternion,
// sin / cos theta, and the ISA atmosphere at h (temperature, 1 / speed of sound, density, the dCm table's
// altitude interval).  None of it depends on the stage's velocities, so with -DB747_FLIGHT_AHEAD the
// pipelined loop of k_env_step_split evaluates stage j + 1's inside stage j, from the stage-j derivatives
// the combine will use (dq = f(w, q0n, q3n), dh = Vy: all stage-j INPUTS), beside stage j's alpha / lookup
// chain, so that the quaternion rsqrt and the density fits leave the stage's dependency chain.  Same
// expressions, same values.  Measured: a stage that no longer evaluates its own is ~700
// cycles shorter, one that evaluates the next stage's instead is as long as before, and the launch is
// 0.1 us slower -- the flight stage pays for its work like an issue-bound wave, not for its chain depth;
// off by default.
#ifndef B747_ISA_SKIP_STRAT
#define B747_ISA_SKIP_STRAT 1   // skip the stratosphere fit in waves entirely below the tropopause (round 4: -0.15 us)
#endif
struct FlightAhead {
    double q0n, q3n, sth, cth, h, T, inva, rho;
    int iDC0;
    float invaf, rhof;   // MIX: 1 / a and rho as computed (fp32)
};
template <bool MIX>
__device__ __forceinline__ FlightAhead flight_ahead(double q0, double q3, double h, KPtr kf, const FlightK &k,
                                                 const double *tb_isa)
{
    FlightAhead a;
    a.invaf = a.rhof = 0.0f;
    // attitude (b747::pass, FAST, kPitchPlane)
    const double q1 = 0.0, q2 = 0.0;
    const double nn = ((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3;
    const double in = rsqrt_pos(nn, k.c375);
    const double q3n = q3 * in, q0n = q0 * in, q2n = 0.0, q1n = 0.0;
    const double s = q2n * q1n + q3n * q0n;
    const double s2 = s + s;
    // cos(asin(s2)) = sqrt((1 - s2)(1 + s2)) >= 0 is |q0n^2 - q3n^2| for the unit pitch-plane quaternion
    // ((q0n^2 - q3n^2)^2 + (2 q0n q3n)^2 = 1): no second rsqrt, a few ulp either way (and better
    // conditioned at 90 deg); NaN still propagates
#ifndef B747_SPLIT_SQRT_COS
    const double cth = fabs(q0n * q0n - q3n * q3n);
#else
    const double wq = (1.0 - s2) * (1.0 + s2);
    const double cth = wq > 0.0 ? wq * rsqrt_pos(wq) : (wq <= 0.0 ? 0.0 : wq);
#endif
    a.q0n = q0n; a.q3n = q3n; a.sth = s2; a.cth = cth;
#ifdef B747_ISA_CELLS
    // ISA from the cell table (gen/fit_isa_cells.py: rho and 1/a as degree-6 polynomials in the cell
    // coordinate, <= 6.5e-16 relative): the clamp keeps the DLL's select semantics (NaN h stays NaN: the cell
    // index of NaN converts to 0 and u is NaN), four ds_read_b128 per quantity, two Horner chains
    (void)kf;
    const double hcl = h > B747_ISA_CELL_HMAX ? B747_ISA_CELL_HMAX : maxsd(0.0, h);
    const double xc = hcl * B747_ISA_CELL_INVW;
    int ci = (int)xc;
    ci = ci < B747_ISA_NCELL - 1 ? ci : B747_ISA_NCELL - 1;
    ci = ci > 0 ? ci : 0;
    const double u = xc - (double)ci;
    const double *rec = tb_isa + ci * B747_ISA_CELL_REC;
    double cr[B747_ISA_CELL_STRIDE], cv[B747_ISA_CELL_STRIDE];
#pragma unroll
    for (int q = 0; q < B747_ISA_CELL_STRIDE; ++q) { cr[q] = rec[q]; cv[q] = rec[B747_ISA_CELL_STRIDE + q]; }
    double rho = cr[B747_ISA_CELL_DEG], inva = cv[B747_ISA_CELL_DEG];
#pragma unroll
    for (int q = B747_ISA_CELL_DEG - 1; q >= 0; --q) { rho = rho * u + cr[q]; inva = inva * u + cv[q]; }
    a.h = h;
    a.T = 0.0;
    a.inva = inva;
    a.rho = rho;
#else
  if constexpr (MIX) {
    // ISA in fp32 on the hardware transcendentals: rho = rho0 thr^(EXP - 1) exp(dhc g / (R T)) as exp2 / log2
    // (<= 6e-7 relative over 0-20 km), 1 / a as v_rsq_f32
    (void)tb_isa; (void)kf;
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
    (void)tb_isa;
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
#if B747_ISA_SKIP_STRAT
    // the stratosphere's exponential only where a lane of the wave is above the tropopause (or NaN): a
    // wave-uniform branch around the degree-12 fit instead of evaluating and discarding it everywhere
    double ex = 1.0;
    if (__ballot(!(dh >= 0.0)) != 0) {
        const double exf = isa_expfit(dhc, kf, k.emid);
        ex = B747_UNPRED(dhc == 0.0) ? 1.0 : exf;
    }
#else
    const double exf = isa_expfit(dhc, kf, k.emid);
    const double ex = B747_UNPRED(dhc == 0.0) ? 1.0 : exf;
#endif
    a.rho = ex * (isa_powfit(thr, kf, k.pmid) * k.rho0);
  }
#endif
    a.iDC0 = bp_index<B747_DCM_MAX0>(kf + KF_DCM0, h);
    return a;
}
template <bool MIX = false>
__device__ __forceinline__ FlightAhead flight_ahead(const double *x, KPtr kf, const FlightK &k, const double *tb)
{
    return flight_ahead<MIX>(x[2], x[3], x[1], kf, k, tb + T_ISA);
}

// The MIX flight pass (B747_VARIANT_MIXED): flight_pre with the aerodynamics in fp32 -- speed and alpha (v_rsq_f32,
// the unit-vector angle with a degree-5 asin series: <= 4.2e-7 rad), the lookups on the packed fp32 records, the
// forces and the moment -- from the fp64 attitude and state; p carries fp64 values for the fp64 combine.
template <bool MOMENT>
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
    if (MOMENT) {
        const float dCm = bil(rDC, (float)h, Mf) * (float)km[3];
        const float mzv = bil(rMZ, Mf, adf) * (float)km[2];
        const float Ka = fmaf(kaB, adf, kaA) * (float)km[4];
        p.mq = (double)(qqf * (float)(B747_M_HALF * B747_DEF_S * B747_DEF_C));
        p.mz_gain = (double)((float)B747_R2D * dCm * Ka);
        p.mz_aero = (double)mzv;
    } else {
        p.mq = p.mz_gain = p.mz_aero = 0.0;
    }
    (void)k;
}

// a: flight_ahead of this stage's input x.  With next != nullptr, also stage j + 1's: cn is stage j's
// combine factor (h/2, h/2, h for j = 0, 1, 2) and yb the step's base state (the combine's y).
template <bool MOMENT = true, bool MIX = false>
__device__ __forceinline__ void flight_pre(const double *x, const double *tb, KPtr kf, const double *km, FlightPass &p,
                                           const FlightK &k, const FlightAhead &a, FlightAhead *next = nullptr,
                                           double cn = 0.0, const double *yb = nullptr, bool stamp_on = false)
{
    if constexpr (MIX) {   // (no look-ahead, stamps or probes in the MIX pass)
        (void)next; (void)cn; (void)yb; (void)stamp_on;
        flight_pre_mix<MOMENT>(x, tb, kf, km, p, k, a);
        return;
    }
    (void)stamp_on;
    B747_FSTAMP(7);
    B747_PROBE(4, x[4]);
    const double q0n = a.q0n, q3n = a.q3n, sth = a.sth, cth = a.cth;
    p.q0n = q0n; p.q3n = q3n; p.sth = sth; p.cth = cth;
    // air data
    const double Vx = x[4], Vy = x[5];
    const double u = cth * Vx + sth * Vy;
    const double v = cth * Vy - sth * Vx;
    const double V2 = u * u + v * v;
    B747_PROBE(7, V2);
    const double iV = rsqrt_pos(V2, k.c375);
    B747_PROBE(8, iV);
    const double V = V2 > 0.0 ? V2 * iV : 0.0 * V2;
    const bool pos = V > 0.0;
    const double sa = pos ? -v * iV : -0.0 * v;
    const double ca = pos ? u * iV : 1.0 + 0.0 * u;
    B747_PROBE(9, sa);
    const double alpha = unit_atan2(sa, ca, kf, k.hpi, k.pi, k.c375);
    B747_PROBE(10, alpha);
    B747_FSTAMP(13);
    if (next) {
        // stage j + 1's attitude and atmosphere (the combine's x = c dX + y of q0, q3 and h, with flight_post's
        // dX[2], dX[3] and dX[1] = Vy), in this basic block so that they fill the alpha chain's latency
        const double w = x[6];
        const double nw = -w;
        const double f2 = nw * q3n * 0.5, f3 = q0n * w * 0.5;
        *next = flight_ahead<false>(cn * f2 + yb[2], cn * f3 + yb[3], cn * Vy + yb[1], kf, k, tb + T_ISA);
    }
    const double h = a.h;
    const double alpha_deg = alpha * k.r2d;
    const double M = V * a.inva;
    B747_PROBE(11, M);
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
    CellRd cDC{}, cMZ{}, cKa{};
    if (MOMENT) {
        cDC = cell_read(tb + T_CELL_DCM1, CellGrid{k.dc_w, k.dc_n, kCellDCm1.nc}, M);
        cMZ = cell_read(tb + T_CELL_MZ1, CellGrid{k.mz_w, k.mz_n, kCellMz1.nc}, alpha_deg);
        cKa = cell_read(tb + T_CELL_KA, CellGrid{k.ka_w, k.ka_n, kCellKa.nc}, alpha_deg);
    }
    sched_fence();
    B747_FSTAMP(14);
    B747_PROBE(12, fCY.d);
    const double CYa = bilin(fCY, M, alpha_deg) * km[1];
    B747_PROBE(13, CYa);
    const CellRd cCX = cell_read(tb + T_CELL_CXA1, CellGrid{k.cx_w, k.cx_n, kCellCXa1.nc}, CYa);
    sched_fence();
    BFetch fDC{}, fMZ{};
    double kaA = 0.0, kaB = 0.0;
    if (MOMENT) {
        fDC = bilin_fetch<B747_DCM_MAX0>(tb, T_REC_DCM, iDC0, cell_idx(cDC, M));
        fMZ = bilin_fetch<B747_MZ_MAX0>(tb, T_REC_MZ, iM, cell_idx(cMZ, alpha_deg));
        const int iKa = cell_idx(cKa, alpha_deg);
        kaA = tb[T_REC_KA + 2 * iKa]; kaB = tb[T_REC_KA + 2 * iKa + 1];
    }
    sched_fence();
    const BFetch fCX = bilin_fetch<B747_CXA_MAX0>(tb, T_REC_CXA, iCX0, cell_idx(cCX, CYa));
    sched_fence();
    B747_PROBE(14, fCX.d);
    const double CXa = bilin(fCX, M, CYa) * km[0];
    const double qq = rho * V2;
    const double qS = qq * B747_F_HALF * k.S;
    const double D = B747_F_NEG * CXa * qS;
    const double L = qS * CYa;
    const double Fy = (ca * L - D * sa) + 0.0;
    const double Fx = (D * ca + sa * L) + k.P;
    p.ax = (Fx * cth - sth * Fy) * k.invm0;
    p.ay = (Fy * cth + Fx * sth) * k.invm0 - k.g;
    if (MOMENT) {
        const double dCm = bilin(fDC, h, M) * km[3];
        const double mzv = bilin(fMZ, M, alpha_deg) * km[2];
        const double Ka = fma(kaB, alpha_deg, kaA) * km[4];
        p.mq = qq * B747_M_HALF * k.S * k.c_;
        static_assert(B747_M_R2D == B747_R2D, "FlightK.r2d");
        p.mz_gain = k.r2d * dCm * Ka;
        p.mz_aero = mzv;
    } else {
        p.mq = p.mz_gain = p.mz_aero = 0.0;
    }
    B747_PROBE(15, p.ay);
    B747_FSTAMP(15);
}

// dX of the flight states (kFX order) for the elevator delta
__device__ __forceinline__ void flight_post(const double *x, double delta, const FlightPass &p, double *dX, const FlightK &k)
{
    const double wdot = (p.mz_gain * (delta * B747_GAIN_DELTA) + p.mz_aero) * p.mq * k.invIz;
    const double w = x[6];
    const double nw = -w;
    dX[0] = x[4];
    dX[1] = x[5];
    dX[2] = nw * p.q3n * 0.5;
    dX[3] = p.q0n * w * 0.5;
    dX[4] = p.ax;
    dX[5] = p.ay;
    dX[6] = wdot;
}

// The pitching moment's derivative wdot from the flight side's (M, alpha, h, rho V^2) of a stage and its delta:
// flight_pre's moment lookups and flight_post's wdot, the same expressions (B747_MOMENT_CTRL: on the control wave).
// km3 = 1 + aero_err[2..4] (mz, dCm, K_alpha).
__device__ __forceinline__ double moment_wdot(const double *tb, KPtr kf, const FlightK &k, double M, double alpha_deg,
                                              double h, double qq, const double *km3, double delta)
{
    const int iM = bp_index<B747_CYA_MAX0>(kf + KF_CYA0, M);
    const int iDC0 = bp_index<B747_DCM_MAX0>(kf + KF_DCM0, h);
    sched_fence();
    const CellRd cDC = cell_read(tb + T_CELL_DCM1, CellGrid{k.dc_w, k.dc_n, kCellDCm1.nc}, M);
    const CellRd cMZ = cell_read(tb + T_CELL_MZ1, CellGrid{k.mz_w, k.mz_n, kCellMz1.nc}, alpha_deg);
    const CellRd cKa = cell_read(tb + T_CELL_KA, CellGrid{k.ka_w, k.ka_n, kCellKa.nc}, alpha_deg);
    sched_fence();
    const BFetch fDC = bilin_fetch<B747_DCM_MAX0>(tb, T_REC_DCM, iDC0, cell_idx(cDC, M));
    const BFetch fMZ = bilin_fetch<B747_MZ_MAX0>(tb, T_REC_MZ, iM, cell_idx(cMZ, alpha_deg));
    const int iKa = cell_idx(cKa, alpha_deg);
    const double kaA = tb[T_REC_KA + 2 * iKa], kaB = tb[T_REC_KA + 2 * iKa + 1];
    sched_fence();
    const double dCm = bilin(fDC, h, M) * km3[1];
    const double mzv = bilin(fMZ, M, alpha_deg) * km3[0];
    const double Ka = fma(kaB, alpha_deg, kaA) * km3[2];
    const double mq = qq * B747_M_HALF * k.S * k.c_;
    const double mz_gain = k.r2d * dCm * Ka;
    return (mz_gain * (delta * B747_GAIN_DELTA) + mzv) * mq * k.invIz;
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

// ------------------------------------------------------------- flight/control pair hand-offs ----
// B747_PAIR_SYNC: in the pipelined (non-lock-step) stage loop only flight wave w and control wave w + 4 -- the
// pair that shares a SIMD and the same 64 envs -- exchange data, so the per-stage workgroup barriers (which
// also wait for the other three pairs) become a progress counter in LDS per pair.  And the control wave runs
// stage j BESIDE the flight wave's stage j instead of one stage behind it: the only flight values a control
// stage reads, (sin theta, cos theta, h) of the stage input, are known as soon as the flight wave has combined
// the previous stage and normalised the attitude, so the flight wave publishes them before its long alpha /
// table-lookup chain and posts the stage; the control wave waits for that post.  The control wave's stage 3
// (and with it the read-out's stash, posted to the flight wave) is then done while the flight wave is still in
// its own stage 3, which takes it off the end of the step.  The flight wave never waits inside the loop (its
// delta table was complete at the barrier after the prologue).
// A wave's LDS operations are performed in order (AMDGPUUsage, memory model gfx942/gfx950: the LDS request
// queue orders one wave's operations; only different waves' may reorder), so a post is a plain LDS store
// after the data's stores and a wait a polled LDS load before the data's loads; compiler fences keep that
// order in the code, and no s_waitcnt is forced on either side.
#ifndef B747_PAIR_SYNC
#define B747_PAIR_SYNC 0
#endif
#ifndef B747_RO_SPLIT
#define B747_RO_SPLIT 0   // A/B: per-step kernel read-out split (control: reward / done / episode, flight: obs rows)
#endif
#ifndef B747_DIAG_MEM
#define B747_DIAG_MEM 0   // diagnostic builds only (wrong results): 1 the launch alone, 2 + the loads and stores
#endif
// B747_MOMENT_CTRL: the pitching moment (dCm, mz and K_alpha lookups, wdot) of every stage on the control wave,
// which has slack, instead of the flight wave (pipelined, non-pair path; see the kernel)
#ifndef B747_MOMENT_CTRL
#define B747_MOMENT_CTRL 0
#endif
#if B747_MOMENT_CTRL && B747_PAIR_SYNC
#error "B747_MOMENT_CTRL is implemented for the barrier path only"
#endif
#ifdef B747_PAIR_ACQ   // A/B: release / acquire orderings (s_waitcnt vmcnt(0) lgkmcnt(0) at every post / after every wait)
constexpr int kPairPost = __ATOMIC_RELEASE, kPairWait = __ATOMIC_ACQUIRE;
#else
constexpr int kPairPost = __ATOMIC_RELAXED, kPairWait = __ATOMIC_RELAXED;
#endif
__device__ __forceinline__ void pair_post(unsigned *f, unsigned v)
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(f, v, kPairPost, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
template <int SLEEP>
__device__ __forceinline__ void pair_wait(unsigned *f, unsigned v)
{
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, kPairWait, __HIP_MEMORY_SCOPE_WORKGROUP)) < v) {
        if (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ------------------------------------------------------------------------------------ the kernel ----
// One ControllerEnv.step (sample_time = dt: one DLL step) of the reference's training configuration
// (kind 3, DEFC) for every env; the per-step API's K1 case of k_env_steps.  XT: the storage type of the
// continuous state X (double, or float where the batch stores it in fp32: loaded into fp64 registers,
// rounded once by the store, as k_env_steps<float, ...>).
template <typename XT, bool MIX = false>
__global__ __launch_bounds__(kSplitBlock) B747_NO_FMAC void k_env_step_split(b747_env_batch b, b747_env_config cfgc,
                                                                            const float *actions, float *obs_seq,
                                                                            float *reward_seq, uint8_t *done_seq)
{
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double sg[sig_rows(kSplitSigMask)][kSplitEnvs];   // stage-4 read-out stash (control wave)
    __shared__ double xth[4][kSplitEnvs], xct[4][kSplitEnvs];    // flight -> control: sin, cos theta per stage
    __shared__ double xh[4][kSplitEnvs];                         // flight -> control: h per stage
    __shared__ double xdl[4][kSplitEnvs];                        // control -> flight: delta per stage
    __shared__ double xr[6][kSplitEnvs];                         // control -> flight: state0 of a reset
    __shared__ double xcv[2][kSplitEnvs];                        // control -> flight: deltaz, vartheta
#if B747_MOMENT_CTRL
    __shared__ double xmo[3][4][kSplitEnvs];                     // flight -> control: M, alpha (deg), rho V^2 per stage
    __shared__ double xwd[4][kSplitEnvs];                        // control -> flight: wdot per stage
#endif
    __shared__ uint32_t xcu[2][kSplitEnvs];                      // control -> flight: flags, k
    __shared__ uint8_t xdone[kSplitEnvs];                        // flight -> control: reset this env
    __shared__ unsigned lockstep;                                // some env of the block has delta(e)
    __shared__ unsigned any_reset;                               // some env of the block resets
    __shared__ unsigned pf2c[4], pc2f[4];                        // B747_PAIR_SYNC progress per wave pair
    const int wv = (threadIdx.x >> 6) & 3;                       // the pair (flight wave wv, control wave wv + 4)
    (void)wv;
#if defined(B747_FLIGHT_AHEAD) || B747_MOMENT_CTRL
    static_assert(!MIX, "the MIX flight pass has no look-ahead / moment-on-control form");
#endif
#if B747_DIAG_MEM == 1   // speed-of-light budget (diagnostic build, tools/exp_budget.sh): the launch alone
    return;
#endif
    B747_MSTAMP(0, true);
    unsigned kpd = prefetch_kernargs_issue<sizeof(b747_env_batch) + sizeof(b747_env_config) + 40>();
#if defined(__HIP_DEVICE_COMPILE__)
    prefetch_const_lines<sizeof(FitCoefs)>(split_kfit(0), kpd);
#endif
    const int64_t n = b.n;
    const int el = threadIdx.x & (kSplitEnvs - 1);
    const bool flight = threadIdx.x < kSplitEnvs;                // waves 0-3 (wave-uniform)
    const int64_t i = (int64_t)blockIdx.x * kSplitEnvs + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    EnvCfg cfgk = cfgc;
    spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    // table image (this variant's part, <= 2 entries per lane), issued before the state loads
    constexpr int lo = T_FAST_LO, hi = kSplitTbEnd;
    double tv[kSplitTbQ];
    #pragma unroll
    for (int q = 0; q < kSplitTbQ; ++q) {
        const int jq = lo + (int)threadIdx.x + q * kSplitBlock;
        tv[q] = (jq < hi) ? split_image<MIX>(jq) : 0.0;
    }
    prefetch_kernargs_wait(kpd);
    if (threadIdx.x == 0) { lockstep = 0u; any_reset = 0u; }
    if (B747_PAIR_SYNC && threadIdx.x < 4) { pf2c[threadIdx.x] = 0u; pc2f[threadIdx.x] = 0u; }

    const XT *Xg = (const XT *)b.X;
    double x[kNC], y[kNC], acc[kNC];   // stage input / base state / RK4 accumulator of this role's states
    double km[5];                      // flight: 1 + aero_err
    Disc D;                            // control side from here
    uint32_t k = 0u, mem = 0u, flags = 0u;
    double ref0 = 0.0;
    float a = 0.0f;
    double ep_ret = 0.0, h_zh = 0.0;
    if (flight) {
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        x[7] = x[8] = 0.0;
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = b.aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        if (!B747_RO_SPLIT) ep_ret = b.ep_return[il];
    } else {
        k = b.k[il];                     // first-use order: k and the delay history start the MAJOR step
        load_disc(b.disc, n, il, D);
        flags = b.flags[il];
        a = actions[il];
#pragma unroll
        for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
        mem = b.mem[il];
        ref0 = b.ref[il];
        h_zh = b.h_zh[il];
        if (B747_RO_SPLIT) ep_ret = b.ep_return[il];
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = (B747_MOMENT_CTRL && j >= 2) ? b.aero_err[j * n + il] + B747_M_ONE : 0.0;
    }
    #pragma unroll

    for (int q = 0; q < kSplitTbQ; ++q) {

        const int jq = lo + (int)threadIdx.x + q * kSplitBlock;

        if (jq < hi) tb[jq] = tv[q];

    }
    wg_barrier();                      // lockstep = 0 and the tables before anyone uses them
    B747_MSTAMP(1);
#if B747_DIAG_MEM == 2   // speed-of-light budget (diagnostic build): the launch + this kernel's loads and stores only
    if (valid) {
        XT *Xd = (XT *)b.X;
        if (flight) {
#pragma unroll
            for (int j = 0; j < kNF; ++j) st_state(&Xd[kFX[j] * n + i], (XT)(x[j] + km[j % 5]));
            b.ep_return[i] = ep_ret;
            b.reward[i] = (float)ep_ret;
            b.done[i] = ep_ret > 1e300 ? 1 : 0;
#pragma unroll
            for (int q = 0; q < 3; ++q) b.obs[i * 3 + q] = (float)x[q];
        } else {
#pragma unroll
            for (int j = 0; j < kNC; ++j) st_state(&Xd[(9 + j) * n + i], (XT)(x[j] + (double)a));
            st_state(&b.disc[2 * n + i], D.rl_prevY + ref0);
            st_state(&b.disc[3 * n + i], D.e_prev + h_zh);
            st_state(&b.disc[4 * n + i], D.ed_prev);
            st_state(&b.disc[(int64_t)(5u + (k & 3u)) * n + i], D.u_hist[k & 3u] + (double)flags);
            if (k % 5u == 0u) {
                st_state(&b.disc[0 * n + i], D.x_dss);
                st_state(&b.disc[1 * n + i], D.y_dss);
            }
            b.k[i] = k + 1u;
            b.mem[i] = (uint8_t)mem;
        }
    }
    return;
#endif

    // ---- controller (core/controller.py:231-264 as env_step_lane; kind 3: MANUAL/DIRECT, CONST refs)
    Params P{};
    const bool ctrl0 = (flags & F_PID_CS) != 0u;
    double deltaz = 0.0, vartheta = 0.0;
    const double tk = t_of(k);
    const double tnew = (double)(k + 1u) * H;
    const double temp = 0.5 * H;
    const bool dss_hit = (k % 5u) == 0u;
    double ud = 0.0;
    PassRef R{};
    const uint32_t mem_held = mem;
    if (!flight) {
        const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
        const double act = (double)a32;
        const bool use_ctrl = (flags & F_PID_CS) != 0u;
        const bool manual = (flags & F_PID_SS) == 0u;
        vartheta = use_ctrl ? 0.0 : ref0;    // pitch_ref of a CONST reference
        h_zh = use_ctrl ? (double)0.0f : h_zh;        // ref[7] is not loaded in kind 3 (as env_load)
        deltaz = manual ? act : 0.0;
        P.deltaz = deltaz; P.vartheta = vartheta; P.h_zh = h_zh; P.flags = flags;
        xcv[0][el] = deltaz; xcv[1][el] = vartheta;   // for the read-out, which the flight side runs
        xcu[0][el] = flags; xcu[1][el] = k;
        // major_step: delay / DSS
        ud = delay_out(k, D.u_hist);
        D.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
        R.has_ref = (k != 0u);
        R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
        R.e_ref = D.e_prev; R.ed_ref = D.ed_prev; R.rl_prevY = D.rl_prevY;
        R.y_dss = D.y_dss; R.mem = mem;
        // delta of the four stages where it does not depend on the pitch error (no SS PID, no dead zone):
        // the actuator at each stage time, stage 0 on the step's start state, stages 1-3 after the MAJOR
        // update (PrevY = r of stage 0 at time t_k)
        if (flags & (F_PID_SS | F_RL)) {
            __hip_atomic_fetch_or(&lockstep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            double r0, d0, r1, d1, r3, d3;
            actuator(tk, R, r0, d0);
            PassRef R1 = R;
            R1.has_ref = true; R1.t_ref = tk; R1.rl_prevY = r0;
            actuator(temp + tk, R1, r1, d1);
            actuator(tnew, R1, r3, d3);
            const bool rp = (flags & F_RP) != 0u;
            xdl[0][el] = rp ? d0 : P.deltaz;
            xdl[1][el] = rp ? d1 : P.deltaz;
            xdl[2][el] = rp ? d1 : P.deltaz;        // stages 1 and 2 share the time t_k + h/2
            xdl[3][el] = rp ? d3 : P.deltaz;
        }
    }
#pragma unroll
    for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
    // the flight side's stage 0 up to the moment needs nothing from the control side: it overlaps the
    // control side's prologue (its state loads, the controller and the delta table)
    FlightPass fp{};
    const FlightK fk = flight_consts();
#ifdef B747_FLIGHT_AHEAD
    FlightAhead fa{};                  // flight: flight_ahead of the next stage's input (the pipelined loop)
#endif
#if B747_PAIR_SYNC && defined(B747_FLIGHT_AHEAD)
#error "B747_PAIR_SYNC and B747_FLIGHT_AHEAD are exclusive"
#endif
    if (flight) {
        const FlightAhead a0 = flight_ahead<MIX>(x, split_kfit(0), fk, tb);
#if B747_PAIR_SYNC
        xth[0][el] = a0.sth; xct[0][el] = a0.cth;   // before the long part of the stage (read after the barrier)
        xh[0][el] = x[1];
#endif
#ifdef B747_FLIGHT_AHEAD
        flight_pre<true, MIX>(x, tb, split_kfit(0), km, fp, fk, a0, &fa, temp, y);
#elif B747_MOMENT_CTRL
        flight_pre<false>(x, tb, split_kfit(0), km, fp, fk, a0);   // (lock step recomputes it with the moment)
        xmo[0][0][el] = fp.M; xmo[1][0][el] = fp.alpha_deg; xmo[2][0][el] = fp.qq;
#else
        flight_pre<true, MIX>(x, tb, split_kfit(0), km, fp, fk, a0);
#endif
#if !B747_PAIR_SYNC
        xth[0][el] = fp.sth; xct[0][el] = fp.cth;
        xh[0][el] = x[1];
#endif
    }
    wg_barrier();
    B747_MSTAMP(2);
    const bool lock = lockstep != 0u;               // workgroup-uniform
    XT *Xw = (XT *)b.X;
    PassOut o{};
    double thPID = 0.0;

    // RK4 combine of this role's states after stage st (b747::major_step, dll@0x2c60)
    auto combine = [&](int st, const double *dX, int ns) __attribute__((always_inline)) {
        const double c = (st == 2) ? H : temp;
        const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
        for (int j = 0; j < ns; ++j) {
            const double fj = dX[j];
            acc[j] = acc[j] + wm * fj;
            x[j] = c * fj + y[j];
        }
    };
    // control stage st on the flight side's (theta, h) of that stage; returns delta
    auto control_stage = [&](int st, double theta, double h, double *dX) __attribute__((always_inline)) -> double {
        const double t = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
        const double delta = control_pass(x, t, theta, h, P, R, dX, o, thPID);
        if (st == 3) {   // the read-out's stage-4 signals (kSplitSigMask)
            SigVals sv;
            sv.v[S_SIM_TIME] = t;
            sv.v[S_DVARTHETA] = o.e;
            sv.v[S_VARTHETA_ZH] = thPID;
            sv.v[S_U_COM_PID] = o.UPID;
            sv.v[S_DVARTHETA_DT] = o.ed;
            sv.v[S_DVARTHETA_DT_DT] = o.edd;
            sv.v[S_ITSE] = x[8];
            sv.v[S_DVARTHETA_INT] = x[4];
            SigStash<kSplitSigMask>{&sg[0][el], kSplitEnvs}(sv);
        }
        if (st == 0) {   // MAJOR-only updates (dll@0x271a), then only what the step changed is written back
            D.x_dss = dss_hit ? B747_DSS_A * D.x_dss + B747_DSS_B * ud : D.x_dss;
            hist_put(D.u_hist, k, o.Ucom);
            D.rl_prevY = o.r;
            D.e_prev = o.e;
            D.ed_prev = o.ed;
            mem = o.and3_bits;
            R.has_ref = true; R.t_ref = tk; R.e_ref = o.e; R.ed_ref = o.ed; R.rl_prevY = o.r;
            R.mem = mem_held;
            if (valid) {
                if (k % 5u == 0u) {
                    st_state(&b.disc[0 * n + i], D.x_dss);
                    st_state(&b.disc[1 * n + i], D.y_dss);
                }
                st_state(&b.disc[2 * n + i], D.rl_prevY);
                st_state(&b.disc[3 * n + i], D.e_prev);
                st_state(&b.disc[4 * n + i], D.ed_prev);
                st_state(&b.disc[(int64_t)(5u + (k & 3u)) * n + i], hist_get(D.u_hist, k));
                b.k[i] = k + 1u;
                b.mem[i] = (uint8_t)mem;
            }
        }
        return delta;
    };

    if (!lock) {
#if B747_PAIR_SYNC
        // iteration j: flight finishes stage j - 1 (moment, combine), publishes stage j's (theta, h) and runs
        // stage j up to the moment; control runs stage j as soon as that (theta, h) is posted
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));   // as major_step: each stage re-derives its constant pointers
#endif
            double dX[kNC];
            if (flight) {
                if (j > 0) {   // (stage 0 up to the moment ran before the barrier, beside the control prologue)
                    flight_post(x, xdl[j - 1][el], fp, dX, fk);
                    combine(j - 1, dX, kNF);
                    const FlightAhead aj = flight_ahead<MIX>(x, split_kfit(zoff), fk, tb + zoff);
                    xth[j][el] = aj.sth; xct[j][el] = aj.cth;
                    xh[j][el] = x[1];
#ifndef B747_PAIR_LATE
                    pair_post(&pf2c[wv], (unsigned)j);
#endif
                    flight_pre<true, MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, aj, nullptr, 0.0, nullptr, j == 2);
#ifdef B747_PAIR_LATE   // A/B: post only after the stage's long part (the control wave one stage behind)
                    pair_post(&pf2c[wv], (unsigned)j);
#endif
                }
            } else {
                if (j > 0) pair_wait<B747_PAIR_SYNC>(&pf2c[wv], (unsigned)j);
                control_stage(j, unit_atan2(xth[j][el], xct[j][el], split_kfit(zoff)), xh[j][el], dX);
                if (j == 3) pair_post(&pc2f[wv], 1u);   // the read-out's stash is written
                combine(j, dX, kNC);
            }
            B747_MSTAMP(3 + j);
        }
        if (flight) {
            double dX[kNF];
            flight_post(x, xdl[3][el], fp, dX, fk);
            combine(3, dX, kNF);
        }
#else
        // iteration j: flight finishes stage j - 1 (moment, combine) and runs stage j up to the moment;
        // control runs stage j - 1 on the (theta, h) flight wrote for it one iteration earlier
#ifdef B747_SPLIT_ROLLED
#pragma unroll 1
#else
#pragma unroll
#endif
        for (int j = 1; j <= 4; ++j) {
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));   // as major_step: each stage re-derives its constant pointers
#endif
            double dX[kNC];
#if B747_MOMENT_CTRL
            // the pitching moment of stage st is the control wave's (iteration st + 1); its wdot reaches the flight
            // wave one iteration later, in time: w = X8 of stage st + 1's input is first read by flight_post(st + 1)
            if (flight) {
                if (j >= 2) {   // X8 of stage j - 1's input from stage j - 2's wdot (combine's expressions)
                    const int sw = j - 2;
                    const double wd = xwd[sw][el];
                    const double cw = (sw == 2) ? H : temp;
                    const double ww = (sw == 1 || sw == 2) ? 2.0 : 1.0;
                    acc[kNF - 1] = acc[kNF - 1] + ww * wd;
                    x[kNF - 1] = cw * wd + y[kNF - 1];
                }
                flight_post(x, xdl[j - 1][el], fp, dX, fk);   // (its dX[6] is not used)
                combine(j - 1, dX, kNF - 1);
                if (j < 4) {
                    flight_pre<false>(x, tb + zoff, split_kfit(zoff), km, fp, fk, flight_ahead<MIX>(x, split_kfit(zoff), fk, tb + zoff),
                                      nullptr, 0.0, nullptr, j == 2);
                    xth[j][el] = fp.sth; xct[j][el] = fp.cth;
                    xh[j][el] = x[1];
                    xmo[0][j][el] = fp.M; xmo[1][j][el] = fp.alpha_deg; xmo[2][j][el] = fp.qq;
                }
            } else {
                control_stage(j - 1, unit_atan2(xth[j - 1][el], xct[j - 1][el], split_kfit(zoff)), xh[j - 1][el], dX);
                combine(j - 1, dX, kNC);
                xwd[j - 1][el] = moment_wdot(tb + zoff, split_kfit(zoff), fk, xmo[0][j - 1][el], xmo[1][j - 1][el],
                                             xh[j - 1][el], xmo[2][j - 1][el], km + 2, xdl[j - 1][el]);
            }
#else
            if (flight) {
                flight_post(x, xdl[j - 1][el], fp, dX, fk);
                combine(j - 1, dX, kNF);
                if (j < 4) {
#ifdef B747_FLIGHT_AHEAD
                    const FlightAhead aj = fa;
                    if (j < 3) flight_pre<true, MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, aj, &fa, j == 2 ? H : temp, y, j == 2);
                    else flight_pre<true, MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, aj, nullptr, 0.0, nullptr, false);
#else
                    flight_pre<true, MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, flight_ahead<MIX>(x, split_kfit(zoff), fk, tb + zoff),
                               nullptr, 0.0, nullptr, j == 2);
#endif
                    xth[j][el] = fp.sth; xct[j][el] = fp.cth;
                    xh[j][el] = x[1];
                }
            } else {
#ifdef B747_DIAG_IDLE_CONTROL   // diagnostic timing build only (wrong results): the control wave idles in iterations 1-3
                if (j < 4) {
#pragma unroll
                    for (int q = 0; q < kNC; ++q) dX[q] = 0.0;
                } else
#endif
                control_stage(j - 1, unit_atan2(xth[j - 1][el], xct[j - 1][el], split_kfit(zoff)), xh[j - 1][el], dX);
                combine(j - 1, dX, kNC);
            }
#endif
            if (j < 4) {
#ifndef B747_STAMPS_FLIGHT
                B747_MSTAMP(12 + j);   // diagnostic: this role's work of iteration j done (13-15)
#endif
                wg_barrier();
            }
            B747_MSTAMP(2 + j);
        }
#endif
    } else {
        // lock step: delta of stage st needs the pitch error of stage st (flight's stage 0 up to the moment
        // ran before the barrier above)
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));
#endif
            double dX[kNC];
#if B747_MOMENT_CTRL && !B747_PAIR_SYNC
            if (st == 0 && flight)   // stage 0 ran before the barrier without the moment
                flight_pre<true, MIX>(x, tb, split_kfit(zoff), km, fp, fk, flight_ahead<MIX>(x, split_kfit(zoff), fk, tb));
#endif
            if (st > 0) {
                if (flight) {
                    flight_pre<true, MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, flight_ahead<MIX>(x, split_kfit(zoff), fk, tb + zoff));
                    xth[st][el] = fp.sth; xct[st][el] = fp.cth;
                    xh[st][el] = x[1];
                }
                wg_barrier();
            }
            if (!flight) {
                xdl[st][el] = control_stage(st, unit_atan2(xth[st][el], xct[st][el], split_kfit(zoff)), xh[st][el], dX);
                combine(st, dX, kNC);
            }
            wg_barrier();
            if (flight) {
                flight_post(x, xdl[st][el], fp, dX, fk);
                combine(st, dX, kNF);
            }
        }
    }
    // ---- end of the step.  Flight: last combine, X0..X8, then the read-out of the control side's stage-4
    // signals; control meanwhile: last combine, X9..X17.  Then the resets: control draws (Controller.reset)
    // and stores its part, flight initialises X0..X8 from the drawn state0.
    const double t6 = H / 6.0;
    const bool wlate = B747_MOMENT_CTRL && !B747_PAIR_SYNC && !lock;   // X8 waits for the control's stage-3 wdot
    if (flight) {
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = acc[j] * t6 + y[j];
        if (valid) {
#pragma unroll
            for (int j = 0; j < kNF; ++j)
                if (!(wlate && j == kNF - 1)) st_state(&Xw[kFX[j] * n + i], (XT)x[j]);
        }
    }
    B747_MSTAMP(11);
    if (B747_PAIR_SYNC && !lock) {                  // the stage-4 stash of this pair's envs is complete
        if (flight) pair_wait<0>(&pc2f[wv], 1u);    // (posted by the control wave in its stage 3)
    } else {
        wg_barrier();                               // the stage-4 stash is complete
    }
#if B747_MOMENT_CTRL
    if (wlate && flight) {   // X8 with stage 3's wdot (combine's expressions, weight 1)
        const double wd = xwd[3][el];
        acc[kNF - 1] = acc[kNF - 1] + 1.0 * wd;
        x[kNF - 1] = acc[kNF - 1] * t6 + y[kNF - 1];
        if (valid) st_state(&Xw[kFX[kNF - 1] * n + i], (XT)x[kNF - 1]);
    }
#endif
    B747_MSTAMP(12);
    if (!flight) {
#pragma unroll
        for (int j = 0; j < kNC; ++j) x[j] = acc[j] * t6 + y[j];
        if (valid) {
#pragma unroll
            for (int j = 0; j < kNC; ++j) st_state(&Xw[(9 + j) * n + i], (XT)x[j]);
            if (ctrl0 || (flags & F_PID_CS)) b.h_zh[i] = h_zh;
        }
    }
#if B747_RO_SPLIT
    // the read-out split over both waves once the stash is complete: the control wave the reward, done and episode
    // bookkeeping (EnvReadOut over its own stash, its deltaz / vartheta / flags / k in registers), the flight wave
    // the observation rows (the kind-3 read-out's PID_LIKE rows, the same expressions as the PPO kernel's early obs)
    if (!flight && valid) {
        float odummy[OBS_MAX_DIM];
        EnvReadOut<true, kSplitSigMask> ro{cfg, flags, deltaz, vartheta, odummy, nullptr, nullptr, 0.0, 0.0, 0.0, false};
        ro(&sg[0][el], kSplitEnvs);
        const float r32 = (float)ro.reward;
        ep_ret += (double)r32;
        const int32_t ep_len = (int32_t)(k + 1u);
        const bool done = ro.done;
        b.reward[i] = r32;
        b.done[i] = done ? 1 : 0;
        if (reward_seq) reward_seq[i] = r32;
        if (done_seq) done_seq[i] = done ? 1 : 0;
        if (done) {   // record_episode_end
            if (b.ep_final_return) b.ep_final_return[i] = ep_ret;
            if (b.ep_final_len) b.ep_final_len[i] = ep_len;
            if (b.ep_stats) {
                b.ep_stats[i] += 1.0;
                b.ep_stats[n + i] += ep_ret;
                b.ep_stats[2 * n + i] += (double)ep_len;
            }
        }
        const bool reset = done && cfg.auto_reset;
        b.ep_return[i] = reset ? 0.0 : ep_ret;
        xdone[el] = reset ? 1 : 0;
        if (reset) __hip_atomic_fetch_or(&any_reset, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (!flight) {
        xdone[el] = 0;
    }
    if (flight && valid) {
        static_assert(kSpecObs == OBS_PID_LIKE && kSpecLimiter == 0, "the kind-3 read-out's observation and done");
        constexpr uint32_t M = kSplitSigMask;
        const double tr = sg[sig_row(M, S_SIM_TIME)][el];
        const bool d = tr >= cfg.tk;
        const bool rs = d && cfg.auto_reset;
        const float o0 = (float)(sg[sig_row(M, S_DVARTHETA_INT)][el] * inv_obs_max(OBS_PID_LIKE, 0));
        const float o1 = (float)(sg[sig_row(M, S_DVARTHETA)][el] * inv_obs_max(OBS_PID_LIKE, 1));
        const float o2 = (float)(sg[sig_row(M, S_DVARTHETA_DT)][el] * inv_obs_max(OBS_PID_LIKE, 2));
        float *orow = b.obs + i * 3;
        orow[0] = rs ? 0.0f : o0; orow[1] = rs ? 0.0f : o1; orow[2] = rs ? 0.0f : o2;
        if (obs_seq) { float *q = obs_seq + i * 3; q[0] = orow[0]; q[1] = orow[1]; q[2] = orow[2]; }
        if (d && b.terminal_obs) { float *q = b.terminal_obs + i * 3; q[0] = o0; q[1] = o1; q[2] = o2; }
    }
#else
    if (flight && valid) {   // read-out (EnvReadOut of the kind-3 configuration) and episode bookkeeping
        const uint32_t fl = xcu[0][el], k1 = xcu[1][el] + 1u;
        const int od = b.obs_dim;
        float *orow = b.obs + i * od;
        float *orow2 = obs_seq ? obs_seq + i * od : nullptr;
        float *trow = b.terminal_obs ? b.terminal_obs + i * od : nullptr;
        EnvReadOut<true, kSplitSigMask> ro{cfg, fl, xcv[0][el], xcv[1][el], orow, trow, orow2, 0.0, 0.0, 0.0, false};
        ro(&sg[0][el], kSplitEnvs);
        const float r32 = (float)ro.reward;
        ep_ret += (double)r32;
        const int32_t ep_len = (int32_t)k1;          // ceil(k / n_sub) before the step, + 1
        const bool done = ro.done;
        b.reward[i] = r32;
        b.done[i] = done ? 1 : 0;
        if (reward_seq) reward_seq[i] = r32;
        if (done_seq) done_seq[i] = done ? 1 : 0;
        if (done) {   // record_episode_end
            if (b.ep_final_return) b.ep_final_return[i] = ep_ret;
            if (b.ep_final_len) b.ep_final_len[i] = ep_len;
            if (b.ep_stats) {
                b.ep_stats[i] += 1.0;
                b.ep_stats[n + i] += ep_ret;
                b.ep_stats[2 * n + i] += (double)ep_len;
            }
        }
        const bool reset = done && cfg.auto_reset;
        b.ep_return[i] = reset ? 0.0 : ep_ret;
        xdone[el] = reset ? 1 : 0;
        if (reset) __hip_atomic_fetch_or(&any_reset, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (flight) {
        xdone[el] = 0;
    }
#endif
    B747_MSTAMP(8);
    wg_barrier();
    B747_MSTAMP(9);
    if (any_reset != 0u) {                          // workgroup-uniform
        if (!flight && valid && xdone[el]) {   // env_reset_lane (reload) + env_store(slot_params), control side
            EnvSlot s{};
            s.episode = b.episode[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) s.ref[j] = b.ref[j * n + i];
            s.flags = flags;
            s.ref_kind = REF_CONST;
            double aero[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) aero[j] = b.aero_err[j * n + i];
            double s0[6];
#pragma unroll
            for (int j = 0; j < 6; ++j)
                s0[j] = b.state0 ? b.state0[j * n + i] : (j == 1 ? 11000.0 : (j == 2 ? 259.1667 : 0.0));
            draw_reset(cfg, (uint64_t)(b.env_offset + i), s, s0, aero);
            if (b.state0 && cfg.reset_ref_mode != RM_NONE) {
#pragma unroll
                for (int j = 0; j < 6; ++j) b.state0[j * n + i] = s0[j];
            }
            s.episode += 1u;
            double xi[NX];
            uint32_t k0, m0;
            initialize(xi, D, k0, m0, s0);
#pragma unroll
            for (int j = 0; j < kNC; ++j) st_state(&Xw[(9 + j) * n + i], (XT)xi[9 + j]);
            store_disc(b.disc, n, i, D);
            b.k[i] = k0;
            b.mem[i] = (uint8_t)m0;
            b.deltaz[i] = 0.0;
            b.upid[i] = 0.0;
            b.tp[i] = 0.0;
            b.ep_len[i] = 0;
            b.vartheta[i] = 0.0;
            b.h_zh[i] = h_zh;
            b.flags[i] = (uint8_t)s.flags;
            b.episode[i] = s.episode;
#pragma unroll
            for (int j = 0; j < 8; ++j) b.ref[j * n + i] = s.ref[j];
            b.ref_kind[i] = (uint8_t)s.ref_kind;
#pragma unroll
            for (int j = 0; j < 5; ++j) b.aero_err[j * n + i] = aero[j];
#pragma unroll
            for (int j = 0; j < 6; ++j) xr[j][el] = s0[j];
        }
        wg_barrier();
        if (flight && valid && xdone[el]) {   // the reset's initialize(), flight side: X0..X8 (q1 = q2 = 0)
            double sf[6], xi[NX];
#pragma unroll
            for (int j = 0; j < 6; ++j) sf[j] = xr[j][el];
            Disc Dd;
            uint32_t k0, m0;
            initialize(xi, Dd, k0, m0, sf);
#pragma unroll
            for (int j = 0; j < 9; ++j) st_state(&Xw[j * n + i], (XT)xi[j]);
        }
    }
    B747_MSTAMP(10, true);
}

}  // namespace
