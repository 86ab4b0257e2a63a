/* b747_oracle.c -- fp64 CPU restatement of core/model_simple_win64.dll (TEST INFRASTRUCTURE).
 *
 * Block-for-block restatement of the Simulink-ERT code in the reference DLL, written from its
 * disassembly (read as text).  Every expression keeps the DLL's
 * operand order so that, with -ffp-contract=off and a correctly rounded libm, the arithmetic
 * is the DLL's up to the last-ulp behaviour of the transcendental functions (the DLL links
 * the MSVC UCRT libm statically; glibc is used here).  Addresses are RVAs in that DLL.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this file.
 */
#include "b747_oracle.h"

#include <math.h>
#include <string.h>

#include "../include/b747_tables.h"

/* rtwCAPI / rt_nonfinite constants (dll.data@0x27110..0x27120, set by rt_InitInfAndNaN) */
#define RT_INF (INFINITY)
#define RT_MINF (-INFINITY)
/* rt_hypotd / norm scaling constants in .rdata, used at dll@0x18fa and dll@0x193e */
#define NORM_SCALE (3.312168642111238e-170)
#define NORM_INV_SCALE (3.019169939857233e+169)

/* ---------------------------------------------------------------- helpers ------------- */

/* x86 MAXSD semantics: returns a if a > b else b (so NaN in either operand yields b). */
static inline double maxsd(double a, double b) { return a > b ? a : b; }

/* Saturation as emitted at dll@0x1ed4 and friends: u > up ? up : maxsd(lo, u). */
static inline double sat(double u, double lo, double up) { return u > up ? up : maxsd(lo, u); }

/* look2_binlx, dll@0x1000-0x119d: binary search on both axes, linear interpolation with
 * linear extrapolation at both ends; table index = i0 + stride*i1. */
static double look2_binlx(double u0, double u1, const double *bp0, const double *bp1,
                          const double *table, const uint32_t *maxIndex, uint32_t stride)
{
    double frac0, frac1;
    uint32_t bpIdx0, bpIdx1, iLeft, iRght, bpIdx;
    if (bp0[0] >= u0) {                                        /* dll@0x1015 */
        bpIdx0 = 0;
        frac0 = (u0 - bp0[0]) / (bp0[1] - bp0[0]);
    } else if (u0 < bp0[maxIndex[0]]) {                       /* dll@0x1041 */
        bpIdx = maxIndex[0] >> 1;
        iLeft = 0;
        iRght = maxIndex[0];
        while (iRght - iLeft > 1) {
            if (bp0[bpIdx] <= u0) iLeft = bpIdx; else iRght = bpIdx;
            bpIdx = (iRght + iLeft) >> 1;
        }
        bpIdx0 = iLeft;
        frac0 = (u0 - bp0[iLeft]) / (bp0[iLeft + 1] - bp0[iLeft]);
    } else {                                                   /* dll@0x10a1 */
        bpIdx0 = maxIndex[0] - 1;
        frac0 = (u0 - bp0[maxIndex[0] - 1]) / (bp0[maxIndex[0]] - bp0[maxIndex[0] - 1]);
    }
    if (bp1[0] >= u1) {                                        /* dll@0x10b5 */
        bpIdx1 = 0;
        frac1 = (u1 - bp1[0]) / (bp1[1] - bp1[0]);
    } else if (u1 < bp1[maxIndex[1]]) {
        bpIdx = maxIndex[1] >> 1;
        iLeft = 0;
        iRght = maxIndex[1];
        while (iRght - iLeft > 1) {
            if (bp1[bpIdx] <= u1) iLeft = bpIdx; else iRght = bpIdx;
            bpIdx = (iRght + iLeft) >> 1;
        }
        bpIdx1 = iLeft;
        frac1 = (u1 - bp1[iLeft]) / (bp1[iLeft + 1] - bp1[iLeft]);
    } else {
        bpIdx1 = maxIndex[1] - 1;
        frac1 = (u1 - bp1[maxIndex[1] - 1]) / (bp1[maxIndex[1]] - bp1[maxIndex[1] - 1]);
    }
    uint32_t base = bpIdx1 * stride + bpIdx0;                  /* dll@0x1145 */
    double yL = table[base] + (table[base + 1] - table[base]) * frac0;
    base += stride;
    double yH = table[base] + (table[base + 1] - table[base]) * frac0;
    return yL + (yH - yL) * frac1;
}

/* inline look1_binlx for K_alpha, dll@0x2083-0x21b0 */
static double look1_Ka(double u)
{
    const double *bp = B747_KA_BP, *tb = B747_KA_TBL;
    uint32_t idx;
    double frac;
    if (bp[0] >= u) {
        idx = 0;
        frac = (u - bp[0]) / (bp[1] - bp[0]);
    } else if (bp[B747_KA_MAX] > u) {
        uint32_t bpIdx = B747_KA_MAX >> 1, iLeft = 0, iRght = B747_KA_MAX;
        while (iRght - iLeft > 1) {
            if (bp[bpIdx] <= u) iLeft = bpIdx; else iRght = bpIdx;
            bpIdx = (iRght + iLeft) >> 1;
        }
        idx = iLeft;
        frac = (u - bp[iLeft]) / (bp[iLeft + 1] - bp[iLeft]);
    } else {
        idx = B747_KA_MAX - 1;
        frac = (u - bp[B747_KA_MAX - 1]) / (bp[B747_KA_MAX] - bp[B747_KA_MAX - 1]);
    }
    return (tb[idx + 1] - tb[idx]) * frac + tb[idx];           /* dll@0x21a1 */
}

/* rt_powd_snf, dll@0x3530 */
static double rt_powd_snf(double u0, double u1)
{
    if (isnan(u0) || isnan(u1)) return NAN;
    double a0 = fabs(u0), a1 = fabs(u1);
    if (isinf(u1)) {
        if (a0 == 1.0) return 1.0;
        if (a0 > 1.0) return u1 > 0.0 ? RT_INF : 0.0;
        return u1 > 0.0 ? 0.0 : RT_INF;
    }
    if (a1 == 0.0) return 1.0;
    if (a1 == 1.0) return u1 > 0.0 ? u0 : 1.0 / u0;
    if (u1 == 2.0) return u0 * u0;
    if (u1 == 0.5 && u0 >= 0.0) return sqrt(u0);
    if (u0 < 0.0 && u1 > floor(u1)) return NAN;
    return pow(u0, u1);
}

/* inline rt_atan2d_snf, dll@0x19a0-0x1a5a */
static double rt_atan2d_snf(double u0, double u1)
{
    if (isnan(u0) || isnan(u1)) return NAN;
    if (isinf(u0) && isinf(u1)) {
        return atan2(u0 > 0.0 ? 1.0 : -1.0, u1 > 0.0 ? 1.0 : -1.0);
    }
    if (u1 == 0.0) {
        if (u0 > 0.0) return M_PI / 2.0;
        if (u0 < 0.0) return -M_PI / 2.0;
        return 0.0;
    }
    return atan2(u0, u1);
}

/* sign as used by the anti-windup AND3 blocks (dll@0x23aa-0x2419): NaN passes through */
static inline double sgn_nan(double x)
{
    if (isnan(x)) return x;
    if (0.0 > x) return -1.0;
    return x > 0.0 ? 1.0 : 0.0;
}
/* cvttsd2si to int32 then compare the low byte (dll@0x2422-0x2432) */
static inline int8_t i8_of(double x)
{
    if (isnan(x)) return 0;  /* 0x80000000 -> low byte 0 */
    return (int8_t)(int32_t)x;
}
static inline uint8_t and3(double zero_sum, double dz, double ie)
{
    if (zero_sum == dz) return 0;                             /* ucomisd ordered-equal */
    return i8_of(sgn_nan(dz)) == i8_of(sgn_nan(ie)) ? 1 : 0;
}
static inline double deadzone(double s, double lo, double up)
{
    if (s > up) return s - up;
    if (!(s >= lo)) return s - lo;                            /* jb: below or unordered */
    return 0.0;
}

/* rt_TDelayInterpolate, dll@0x29e0 (discrete = 0, minorStepAndTAtLastMajorOutput = 0) */
static double rt_TDelayInterpolate(double tMinusDelay, double tStart, const double *uBuf, int bufSz,
                                   int *lastIdx, int oldestIdx, int newIdx, double initOutput)
{
    const double *tBuf = uBuf + bufSz;
    if (newIdx == 0 && oldestIdx == 0 && tMinusDelay > tStart) return initOutput;
    if (!(tStart < tMinusDelay)) return initOutput;           /* dll@0x2a07: <= or NaN */
    if (tMinusDelay <= tBuf[oldestIdx]) {
        int tempIdx = oldestIdx + 1;
        if (oldestIdx == bufSz - 1) tempIdx = 0;
        double t1 = tBuf[oldestIdx], t2 = tBuf[tempIdx], u1 = uBuf[oldestIdx], u2 = uBuf[tempIdx];
        if (t2 == t1) return tMinusDelay >= t2 ? u2 : u1;
        double f1 = (t2 - tMinusDelay) / (t2 - t1), f2 = 1.0 - f1;
        return u2 * f2 + f1 * u1;
    }
    int i = *lastIdx;
    if (tBuf[i] < tMinusDelay) {
        while (tBuf[i] < tMinusDelay) {
            if (i == newIdx) break;
            i = (i < bufSz - 1) ? i + 1 : 0;
        }
    } else {
        while (tBuf[i] >= tMinusDelay) i = (i > 0) ? i - 1 : bufSz - 1;
        i = (i < bufSz - 1) ? i + 1 : 0;
    }
    *lastIdx = i;
    double t1, u1;
    if (i == 0) { t1 = tBuf[bufSz - 1]; u1 = uBuf[bufSz - 1]; }
    else        { t1 = tBuf[i - 1];     u1 = uBuf[i - 1]; }
    double t2 = tBuf[i], u2 = uBuf[i];
    if (t2 == t1) return tMinusDelay >= t2 ? u2 : u1;
    double f1 = (t2 - tMinusDelay) / (t2 - t1), f2 = 1.0 - f1;
    return u2 * f2 + f1 * u1;                                  /* dll@0x2c2d */
}

/* Simulink Derivative block output, dll@0x24b2 (D1) / dll@0x250a (D2) */
static double derivative_out(double u, double t, double TA, double uA, double TB, double uB)
{
    if (TA >= t && TB >= t) return 0.0;
    double lastT = TA, lastU = uA;
    if (TA < TB) {
        if (TB < t) { lastT = TB; lastU = uB; }
    } else if (TA >= t) {
        lastT = TB; lastU = uB;
    }
    return (u - lastU) / (t - lastT);
}
/* Derivative block update, dll@0x281c (D1) / dll@0x2881 (D2) */
static void derivative_update(double u, double t, double *TA, double *uA, double *TB, double *uB)
{
    if (*TA == RT_INF)      { *TA = t; *uA = u; }
    else if (*TB == RT_INF) { *TB = t; *uB = u; }
    else if (*TB > *TA)     { *TA = t; *uA = u; }
    else                    { *TB = t; *uB = u; }
}

/* ------------------------------------------------------------ the model ------------- */

void b747o_defaults(b747o_model *m)
{
    memset(m, 0, sizeof(*m));
    m->Iz = B747_DEF_IZ;
    m->P = B747_DEF_P;
    for (int i = 0; i < 4; ++i) { m->PID_CS[i] = B747_DEF_PID_CS[i]; m->PID_SS[i] = B747_DEF_PID_SS[i]; }
    m->S = B747_DEF_S;
    for (int i = 0; i < 5; ++i) m->aero_err[i] = B747_DEF_AERO_ERR[i];
    m->c_ = B747_DEF_C;
    m->deltaz = B747_DEF_DELTAZ;
    m->g = B747_DEF_G;
    m->h_zh = B747_DEF_H_ZH;
    m->m0 = B747_DEF_M0;
    for (int i = 0; i < 6; ++i) m->state0[i] = B747_DEF_STATE0[i];
    m->use_PID_CS = B747_DEF_USE_PID_CS;
    m->use_PID_SS = B747_DEF_USE_PID_SS;
    m->use_RL = B747_DEF_USE_RL;
    m->use_RP = B747_DEF_USE_RP;
    m->vartheta = B747_DEF_VARTHETA;
    b747o_initialize(m);
}

void b747o_initialize(b747o_model *m)
{
    /* dll@0x12a0: timing */
    m->t = 0.0;
    m->stop_time = 0.0;
    m->clock_tick0 = m->clock_tick1 = 0;
    m->major = 1;
    m->tid2 = 0;
    /* zero exported signals, B and DW (dll@0x13e6-0x14c5, memset dll@0x1528) */
    m->sim_time = m->dvartheta = m->U_com = m->alpha = m->V = m->Mach = 0.0;
    for (int i = 0; i < 6; ++i) m->state[i] = 0.0;
    m->dvartheta_dt = m->dvartheta_dt_dt = m->dvartheta_int = m->AE = m->ITAE = m->IAE = 0.0;
    m->ISE = m->ITSE = m->SE = m->TAE = m->TSE = 0.0;
    m->K_alpha = m->mz = m->dCm_ddeltaz = m->CXa = m->CYa = m->deltaz_RP = 0.0;
    m->U_com_PID = m->vartheta_zh = 0.0;
    m->rdot[0] = m->rdot[1] = m->acc[0] = m->acc[1] = m->wdot = 0.0;
    for (int i = 0; i < 4; ++i) m->qdot[i] = 0.0;
    m->in_CS = m->Np_CS = m->in_SS = m->Np_SS = 0.0;
    m->k_CX = m->k_CY = m->k_mz = m->k_dCm = m->k_Ka = 0.0;
    m->ud = m->y_dss = m->rl_out = 0.0;
    m->and3_SS = m->and3_CS = m->mem_SS = m->mem_CS = 0;
    /* DWork initial values (dll@0x1532-0x167c) */
    m->ic_firstT = RT_MINF;
    m->x_dss = B747_DSS_X0;
    m->rl_prevY = 0.0;
    m->rl_lastT = RT_INF;
    m->d1_TA = m->d1_TB = m->d2_TA = m->d2_TB = RT_INF;
    m->d1_uA = m->d1_uB = m->d2_uA = m->d2_uB = 0.0;
    m->dw_mem_SS = m->dw_mem_CS = 0;
    m->dl_tail = m->dl_head = m->dl_last = 0;
    m->dl_bufsz = B747_DELAY_BUFSZ;
    memset(m->dl_buf, 0, sizeof(m->dl_buf));
    m->dl_buf[0] = B747_DELAY_INIT;          /* uBuf[0] */
    m->dl_buf[B747_DELAY_BUFSZ] = m->t;      /* tBuf[0] */
    /* continuous states from state0 (dll@0x1579-0x16a7) */
    m->X[0] = m->state0[0];
    m->X[1] = m->state0[1];
    m->X[6] = m->state0[2];
    m->X[7] = m->state0[3];
    m->X[8] = m->state0[5];
    m->X[9] = m->X[10] = m->X[11] = m->X[12] = 0.0;
    m->X[13] = m->X[14] = m->X[15] = m->X[16] = m->X[17] = 0.0;
    double half = m->state0[4] * 0.5;
    m->X[2] = cos(half);
    m->X[3] = m->X[4] = 0.0;
    m->X[5] = sin(half);
    m->first_step = 1;
}

/* Output pass: model_simple_step body dll@0x176c-0x2711 (MAJOR or MINOR per m->major). */
static void output_pass(b747o_model *m)
{
    const int major = m->major;
    const double t = m->t;
    double *X = m->X;
    /* quaternion normalisation and pitch angle */
    double q0 = X[2], q1 = X[3], q2 = X[4], q3 = X[5];
    double n = sqrt(((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3);
    double q3n = q3 / n, q0n = q0 / n, q2n = q2 / n, q1n = q1 / n;
    double s = q2n * q1n + q3n * q0n;
    double theta = asin(s + s);
    /* IC block (dll@0x1828) */
    if (m->ic_firstT == RT_MINF || m->ic_firstT == t) {
        m->ic_firstT = t;
        for (int i = 0; i < 6; ++i) m->state[i] = m->state0[i];
    } else {
        m->state[0] = X[0]; m->state[1] = X[1]; m->state[2] = X[6];
        m->state[3] = X[7]; m->state[4] = theta; m->state[5] = X[8];
    }
    double sth = sin(theta), cth = cos(theta);
    double Vx = X[6], Vy = X[7];
    double u = cth * Vx + sth * Vy;
    double v = cth * Vy - sth * Vx;
    /* airspeed: scaled 2-norm (dll@0x18fa-0x1aae) */
    double scale = NORM_SCALE, y;
    double au = fabs(u);
    if (au > scale) { y = 1.0; scale = au; }
    else { double tt = au * NORM_INV_SCALE; y = tt * tt; }
    double av = fabs(v);
    if (av > scale) { double tt = scale / av; y = y * tt * tt + 1.0; scale = av; }
    else { double tt = av / scale; y = y + tt * tt; }
    double V = sqrt(y) * scale;
    m->V = V;
    double alpha = -rt_atan2d_snf(v, u);
    m->alpha = alpha;
    /* ISA atmosphere (dll@0x1a93-0x1cb7) */
    double h = X[1];
    double hc = h > B747_ISA_TROPO_UP ? B747_ISA_TROPO_UP : maxsd(B747_ISA_TROPO_LO, h);
    double T = B747_ISA_T0 - hc * B747_ISA_LAPSE;
    double a = sqrt(T * B747_ISA_GAMMA_R);
    double alpha_deg = alpha * B747_R2D;
    double M = V / a;
    m->Mach = M;
    m->T_isa = T;
    m->a_isa = a;
    if (major) {                                               /* dll@0x1b1a */
        m->k_CY = m->aero_err[1] + B747_F_ONE;
        m->k_CX = m->aero_err[0] + B747_F_ONE;
    }
    double CYa = look2_binlx(M, alpha_deg, B747_CYA_BP0, B747_CYA_BP1, B747_CYA_TBL,
                             (const uint32_t[]){B747_CYA_MAX0, B747_CYA_MAX1}, 4) * m->k_CY;
    m->CYa = CYa;
    double CXa = look2_binlx(M, CYa, B747_CXA_BP0, B747_CXA_BP1, B747_CXA_TBL,
                             (const uint32_t[]){B747_CXA_MAX0, B747_CXA_MAX1}, 4) * m->k_CX;
    m->CXa = CXa;
    double thr = T * B747_ISA_INV_T0;
    double pr;
    if (0.0 > thr && B747_ISA_EXP > floor(B747_ISA_EXP)) pr = -rt_powd_snf(-thr, B747_ISA_EXP);
    else pr = rt_powd_snf(thr, B747_ISA_EXP);
    double dh = B747_ISA_H_TROPO - h;
    double dhc = dh > B747_ISA_STRAT_UP ? B747_ISA_STRAT_UP : maxsd(B747_ISA_STRAT_LO, dh);
    double ex = exp(dhc * B747_ISA_G_R * (1.0 / T));
    double rho = ex * (pr / thr * B747_ISA_RHO0);
    double qq = rho * (V * V);
    double qS = qq * B747_F_HALF * m->S;
    m->rho = rho;
    m->qq = qq;
    /* aerodynamic forces in the velocity frame (dll@0x1cc0-0x1d59) */
    double sa = sin(alpha), ca = cos(alpha);
    double D = B747_F_NEG * CXa * qS;
    double L = qS * CYa;
    double Fy = (ca * L - D * sa) + 0.0;
    double Fx = (D * ca + sa * L) + m->P;
    /* actuator: transport delay -> DSS -> rate limiter -> saturation (dll@0x1d43-0x1e8c) */
    double ud = rt_TDelayInterpolate(t - B747_DELAY, 0.0, m->dl_buf, m->dl_bufsz, &m->dl_last,
                                     m->dl_tail, m->dl_head, B747_DELAY_INIT);
    m->ud = ud;
    if (major && m->tid2 == 0) m->y_dss = m->x_dss * B747_DSS_C + B747_DSS_D * ud;
    double ydss = m->y_dss;
    double r;
    if (m->rl_lastT == RT_INF) {
        r = ydss;
    } else {
        double dtl = t - m->rl_lastT;
        double du = ydss - m->rl_prevY;
        double rise = dtl * B747_RATE_RISE;
        if (du > rise) {
            r = rise + m->rl_prevY;
        } else {
            double fall = dtl * B747_RATE_FALL;
            r = (fall > du) ? fall + m->rl_prevY : ydss;
        }
    }
    m->rl_out = r;
    double dRP = sat(r, B747_SAT4_LO, B747_SAT4_UP);
    m->deltaz_RP = dRP;
    /* altitude-hold PID (CS loop), dll@0x1e6f */
    double eh = m->h_zh - h;
    double NpCS = (eh * m->PID_CS[2] - X[10]) * m->PID_CS[3];
    double sumCS = eh * m->PID_CS[0] + X[9] + NpCS;
    m->Np_CS = NpCS;
    double thPID = sat(sumCS, B747_CS_LO, B747_CS_UP);
    m->vartheta_zh = thPID;
    double thref = (m->use_PID_CS >= B747_SWITCH_THR) ? thPID : m->vartheta;
    double e = thref - theta;
    m->dvartheta = e;
    /* pitch-stabilisation PID (SS loop), dll@0x1f1f */
    double NpSS = (e * m->PID_SS[2] - X[12]) * m->PID_SS[3];
    double sumSS = e * m->PID_SS[0] + X[11] + NpSS;
    m->Np_SS = NpSS;
    double UPID = sat(sumSS, B747_SS_LO, B747_SS_UP);
    m->U_com_PID = UPID;
    double Ucom;
    if (m->use_RL >= B747_SWITCH_THR) Ucom = (B747_RL_DEADZONE > fabs(0.0 - UPID)) ? 0.0 : UPID;
    else if (m->use_PID_SS >= B747_SWITCH_THR) Ucom = UPID;
    else Ucom = m->deltaz;
    m->U_com = Ucom;
    /* aerodynamic moments (dll@0x1fe4-0x2213) */
    if (major) {
        m->k_dCm = m->aero_err[3] + B747_M_ONE;
        m->k_Ka = m->aero_err[4] + B747_M_ONE;
    }
    double dCm = look2_binlx(h, M, B747_DCM_BP0, B747_DCM_BP1, B747_DCM_TBL,
                             (const uint32_t[]){B747_DCM_MAX0, B747_DCM_MAX1}, 5) * m->k_dCm;
    m->dCm_ddeltaz = dCm;
    double Ka = look1_Ka(alpha_deg) * m->k_Ka;
    m->K_alpha = Ka;
    double mzv = look2_binlx(M, alpha_deg, B747_MZ_BP0, B747_MZ_BP1, B747_MZ_TBL,
                             (const uint32_t[]){B747_MZ_MAX0, B747_MZ_MAX1}, 4);
    if (major) m->k_mz = m->aero_err[2] + B747_M_ONE;
    mzv = mzv * m->k_mz;
    m->mz = mzv;
    /* translational dynamics (dll@0x21ee-0x2285) */
    double sth2 = sin(theta);
    double ax = (Fx * cth - sth2 * Fy) / m->m0;
    double ay = (Fy * cth + Fx * sth) / m->m0 - m->g;
    m->rdot[0] = Vx; m->rdot[1] = Vy;
    m->acc[0] = ax; m->acc[1] = ay;
    /* pitch dynamics (dll@0x2265-0x2320): no pitch-damping term in this model */
    double delta = (m->use_RP >= B747_SWITCH_THR) ? dRP : Ucom;
    double mq = qq * B747_M_HALF * m->S * m->c_;
    m->wdot = (B747_M_R2D * dCm * Ka * (delta * B747_GAIN_DELTA) + mzv) * mq / m->Iz;
    /* quaternion kinematics (dll@0x22bc-0x2360) */
    double w = X[8], nw = -w;
    m->qdot[1] = q2n * w * 0.5;
    m->qdot[0] = nw * q3n * 0.5;
    m->qdot[2] = nw * q1n * 0.5;
    m->qdot[3] = q0n * w * 0.5;
    /* clamping anti-windup, SS loop (dll@0x2368-0x2479) */
    double zeroSS = sumSS * B747_AW_ZEROGAIN;
    double dzSS = deadzone(sumSS, B747_SS_LO, B747_SS_UP);
    double ieSS = m->PID_SS[1] * e;
    m->in_SS = ieSS;
    m->and3_SS = and3(zeroSS, dzSS, ieSS);
    if (major) m->mem_SS = m->dw_mem_SS;
    if (m->mem_SS) m->in_SS = B747_AW_ZERO;
    /* error characteristics (dll@0x2481-0x25ae) */
    m->sim_time = t;
    double ed = derivative_out(e, t, m->d1_TA, m->d1_uA, m->d1_TB, m->d1_uB);
    m->dvartheta_dt = ed;
    double edd = derivative_out(ed, t, m->d2_TA, m->d2_uA, m->d2_TB, m->d2_uB);
    m->dvartheta_dt_dt = edd;
    double se = e * e;
    m->SE = se;
    m->AE = fabs(e);
    m->TSE = se * t;
    m->TAE = fabs(e) * t;
    /* clamping anti-windup, CS loop (dll@0x25a2-0x26b9) */
    double zeroCS = sumCS * B747_AW_ZEROGAIN;
    double dzCS = deadzone(sumCS, B747_CS_LO, B747_CS_UP);
    double ieCS = eh * m->PID_CS[1];
    m->in_CS = ieCS;
    m->and3_CS = and3(zeroCS, dzCS, ieCS);
    if (major) m->mem_CS = m->dw_mem_CS;
    if (m->mem_CS) m->in_CS = B747_AW_ZERO;
    m->dvartheta_int = X[13];
    m->ITAE = X[14];
    m->IAE = X[15];
    m->ITSE = X[17];
    m->ISE = X[16];
}

/* MAJOR-only updates, dll@0x271a-0x28fb */
static void update_pass(b747o_model *m)
{
    const double t = m->t;
    int last = m->dl_bufsz - 1;
    m->dl_head = (m->dl_head < last) ? m->dl_head + 1 : 0;
    if (m->dl_head == m->dl_tail) m->dl_tail = (m->dl_tail < last) ? m->dl_tail + 1 : 0;
    m->dl_buf[m->dl_head + m->dl_bufsz] = t;
    m->dl_buf[m->dl_head] = m->U_com;
    if (m->tid2 == 0) m->x_dss = B747_DSS_A * m->x_dss + B747_DSS_B * m->ud;
    m->rl_prevY = m->rl_out;
    m->rl_lastT = t;
    m->dw_mem_SS = m->and3_SS;
    derivative_update(m->dvartheta, t, &m->d1_TA, &m->d1_uA, &m->d1_TB, &m->d1_uB);
    derivative_update(m->dvartheta_dt, t, &m->d2_TA, &m->d2_uA, &m->d2_TB, &m->d2_uB);
    m->dw_mem_CS = m->and3_CS;
}

/* model_simple_derivatives, dll@0x11a0 */
static void derivatives(const b747o_model *m, double *dX)
{
    dX[0] = m->rdot[0]; dX[1] = m->rdot[1];
    dX[2] = m->qdot[0]; dX[3] = m->qdot[1]; dX[4] = m->qdot[2]; dX[5] = m->qdot[3];
    dX[6] = m->acc[0]; dX[7] = m->acc[1];
    dX[8] = m->wdot;
    dX[9] = m->in_CS; dX[10] = m->Np_CS; dX[11] = m->in_SS; dX[12] = m->Np_SS;
    dX[13] = m->dvartheta; dX[14] = m->TAE; dX[15] = m->AE; dX[16] = m->SE; dX[17] = m->TSE;
}

/* rt_ertODEUpdateContinuousStates (ode4), dll@0x2c60 */
static void ode4(b747o_model *m)
{
    double y[B747O_NX], f0[B747O_NX], f1[B747O_NX], f2[B747O_NX], f3[B747O_NX];
    const double t0 = m->t, tnew = m->stop_time, h = B747_STEP_SIZE;
    m->major = 0;
    memcpy(y, m->X, sizeof(y));
    derivatives(m, f0);
    double temp = 0.5 * h;
    for (int i = 0; i < B747O_NX; ++i) m->X[i] = temp * f0[i] + y[i];
    m->t = temp + t0;
    output_pass(m);
    derivatives(m, f1);
    for (int i = 0; i < B747O_NX; ++i) m->X[i] = temp * f1[i] + y[i];
    output_pass(m);
    derivatives(m, f2);
    for (int i = 0; i < B747O_NX; ++i) m->X[i] = h * f2[i] + y[i];
    m->t = tnew;
    output_pass(m);
    derivatives(m, f3);
    temp = h / 6.0;
    for (int i = 0; i < B747O_NX; ++i)
        m->X[i] = ((((f1[i] + f1[i]) + f0[i]) + (f2[i] + f2[i])) + f3[i]) * temp + y[i];
    m->major = 1;
}

void b747o_step(b747o_model *m)
{
    /* dll@0x1724: stop time = (clockTick0 + 1) * stepSize */
    m->stop_time = (double)(m->clock_tick0 + 1u) * B747_STEP_SIZE;
    output_pass(m);
    update_pass(m);
    if (m->first_step) {                                       /* dll@0x28fb */
        m->major = 0;
        m->first_step = 0;
        output_pass(m);
        m->major = 1;
    }
    ode4(m);
    m->clock_tick0++;
    m->t = m->stop_time;
    m->clock_tick1++;
    m->tid2 = (uint8_t)((m->tid2 + 1 > 4) ? 0 : m->tid2 + 1);
}

/* ------------------------------------------------------ compact import / export ----- */

static inline double t_of(uint32_t j) { return (double)j * B747_STEP_SIZE; }

void b747o_export_compact(const b747o_model *m, b747o_compact *c)
{
    memset(c, 0, sizeof(*c));
    uint32_t k = m->clock_tick0;
    c->k = k;
    c->mem = (m->dw_mem_SS ? 1u : 0u) | (m->dw_mem_CS ? 2u : 0u);
    memcpy(c->X, m->X, sizeof(c->X));
    c->x_dss = m->x_dss;
    c->y_dss = m->y_dss;
    c->rl_prevY = m->rl_prevY;
    if (k >= 1) {
        /* the Derivative slot holding t_{k-1} is the one with the larger time stamp */
        int d1B = (m->d1_TB != RT_INF) && (m->d1_TB > m->d1_TA);
        int d2B = (m->d2_TB != RT_INF) && (m->d2_TB > m->d2_TA);
        c->e_prev = d1B ? m->d1_uB : m->d1_uA;
        c->ed_prev = d2B ? m->d2_uB : m->d2_uA;
    }
    for (uint32_t d = 1; d <= 4 && d <= k; ++d) {
        uint32_t j = k - d;
        int idx = (int)((j + 1) % (uint32_t)m->dl_bufsz);
        c->u_hist[j & 3] = m->dl_buf[idx];
    }
}

void b747o_import_compact(b747o_model *m, const b747o_compact *c)
{
    uint32_t k = c->k;
    int B = B747_DELAY_BUFSZ;
    m->clock_tick0 = m->clock_tick1 = k;
    m->t = t_of(k);
    m->stop_time = m->t;
    m->major = 1;
    m->tid2 = (uint8_t)(k % 5u);
    m->first_step = (k == 0);
    memcpy(m->X, c->X, sizeof(m->X));
    m->x_dss = c->x_dss;
    m->y_dss = c->y_dss;
    m->ic_firstT = (k == 0) ? RT_MINF : 0.0;
    m->rl_prevY = (k == 0) ? 0.0 : c->rl_prevY;
    m->rl_lastT = (k == 0) ? RT_INF : t_of(k - 1);
    m->dw_mem_SS = (c->mem & 1u) ? 1 : 0;
    m->dw_mem_CS = (c->mem & 2u) ? 1 : 0;
    /* Derivative slots: A = older (t_{k-2}, value never read again), B = t_{k-1} */
    m->d1_TA = m->d1_TB = m->d2_TA = m->d2_TB = RT_INF;
    m->d1_uA = m->d1_uB = m->d2_uA = m->d2_uB = 0.0;
    if (k == 1) {
        m->d1_TA = 0.0; m->d1_uA = c->e_prev;
        m->d2_TA = 0.0; m->d2_uA = c->ed_prev;
    } else if (k >= 2) {
        m->d1_TA = t_of(k - 2); m->d1_uA = NAN; m->d1_TB = t_of(k - 1); m->d1_uB = c->e_prev;
        m->d2_TA = t_of(k - 2); m->d2_uA = NAN; m->d2_TB = t_of(k - 1); m->d2_uB = c->ed_prev;
    }
    /* transport-delay ring: entry 0 = (0, init), entry j+1 = (t_j, U_com_j) */
    m->dl_bufsz = B;
    for (int i = 0; i < 2 * B; ++i) m->dl_buf[i] = NAN;
    m->dl_head = (int)(k % (uint32_t)B);
    m->dl_tail = (k < (uint32_t)B) ? 0 : (int)((k + 1) % (uint32_t)B);
    if (k < (uint32_t)B) { m->dl_buf[0] = B747_DELAY_INIT; m->dl_buf[B] = 0.0; }
    uint32_t jlo = (k + 1 > (uint32_t)B) ? k + 1 - (uint32_t)B : 0;
    for (uint32_t j = jlo; j < k; ++j) m->dl_buf[B + (int)((j + 1) % (uint32_t)B)] = t_of(j);
    for (uint32_t d = 1; d <= 4 && d <= k; ++d) {
        uint32_t j = k - d;
        m->dl_buf[(int)((j + 1) % (uint32_t)B)] = c->u_hist[j & 3];
    }
    m->dl_last = (k >= 4) ? (int)((k - 3) % (uint32_t)B) : 0;
}

/* ------------------------------------------------------------------- test hooks ----- */

double b747o_test_lookup(int which, double u0, double u1)
{
    switch (which) {
    case 0: return look2_binlx(u0, u1, B747_CYA_BP0, B747_CYA_BP1, B747_CYA_TBL,
                               (const uint32_t[]){B747_CYA_MAX0, B747_CYA_MAX1}, 4);
    case 1: return look2_binlx(u0, u1, B747_CXA_BP0, B747_CXA_BP1, B747_CXA_TBL,
                               (const uint32_t[]){B747_CXA_MAX0, B747_CXA_MAX1}, 4);
    case 2: return look2_binlx(u0, u1, B747_DCM_BP0, B747_DCM_BP1, B747_DCM_TBL,
                               (const uint32_t[]){B747_DCM_MAX0, B747_DCM_MAX1}, 5);
    case 3: return look2_binlx(u0, u1, B747_MZ_BP0, B747_MZ_BP1, B747_MZ_TBL,
                               (const uint32_t[]){B747_MZ_MAX0, B747_MZ_MAX1}, 4);
    default: return look1_Ka(u0);
    }
}

void b747o_test_pass(const double *X, uint32_t k, double deltaz, double vartheta, double use_pid_ss,
                     double *sig31, double *isa4)
{
    static b747o_model m;
    b747o_defaults(&m);
    b747o_compact c;
    memset(&c, 0, sizeof(c));
    c.k = k;
    memcpy(c.X, X, sizeof(c.X));
    c.x_dss = B747_DSS_X0;
    b747o_import_compact(&m, &c);
    m.deltaz = deltaz;
    m.vartheta = vartheta;
    m.use_PID_SS = use_pid_ss;
    output_pass(&m);
    const double v[31] = {
        m.sim_time, m.dvartheta, m.U_com, m.alpha, m.V, m.state[0], m.state[1], m.state[2], m.state[3],
        m.state[4], m.state[5], m.Mach, m.dvartheta_dt, m.dvartheta_dt_dt, m.dvartheta_int, m.AE, m.ITAE,
        m.IAE, m.ISE, m.ITSE, m.SE, m.TAE, m.TSE, m.K_alpha, m.mz, m.dCm_ddeltaz, m.CXa, m.CYa,
        m.deltaz_RP, m.U_com_PID, m.vartheta_zh};
    memcpy(sig31, v, sizeof(v));
    isa4[0] = m.T_isa; isa4[1] = m.a_isa; isa4[2] = m.rho; isa4[3] = m.qq;
}
