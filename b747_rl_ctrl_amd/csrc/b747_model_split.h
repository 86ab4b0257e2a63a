// b747_model_split.h -- one model_simple_step (dll@0x16d0; core/model.py:247-250 per call) of every env of a
// b747_model_batch with every env split over three waves, as the per-step env kernel (b747_split.h
// k_env_step_split): flight (the air data / alpha / lookup / force chain of the four RK4 stages and the RK4 of
// X0..X8), ahead (each stage's attitude and atmosphere, one stage early) and control (the actuator's delta of all four
// stages, the PID side X9..X17, the MAJOR-only updates), handing off through LDS progress counters.  It is
// b747_model_step's kernel for n_steps = 1 with the DLL's default constants in the FAST variant -- BASELINE config 2's
// one-step launches; k_model_steps_split below is its K-step form -- and writes the 31 exported signals of the stage-4 pass (what core/model.py's properties read
// after step()) from the role that computes each.  64 envs per workgroup: one wave per role, and the three waves of
// a workgroup run on three SIMDs of one CU (the small-batch regime: config 2's 4,096 envs are 64 workgroups), so no
// role waits for another's issue slots.
#pragma once

#include "b747_split.h"

namespace {

constexpr int kMsEnvs = 64;               // envs per workgroup
constexpr int kMsBlock = 3 * kMsEnvs;     // flight, ahead, control wave

// The FAST table image, a third of it per role: each role issues its entries first, inside its own branch (no load
// is pending where the roles' code paths split: k_env_step_split's prologue), then its state, then the LDS writes.
constexpr int kMsTbQ = (kSplitTbEnd - T_FAST_LO + kMsBlock - 1) / kMsBlock;
__device__ __forceinline__ void ms_table_loads(double *tv)
{
#pragma unroll
    for (int q = 0; q < kMsTbQ; ++q) {
        const int jq = T_FAST_LO + (int)threadIdx.x + q * kMsBlock;
        tv[q] = (jq < kSplitTbEnd) ? split_image<false>(jq) : 0.0;
    }
}
__device__ __forceinline__ void ms_stage_tables(double *tb, const double *tv)
{
#pragma unroll
    for (int q = 0; q < kMsTbQ; ++q) {
        const int jq = T_FAST_LO + (int)threadIdx.x + q * kMsBlock;
        if (jq < kSplitTbEnd) tb[jq] = tv[q];
    }
}
__device__ __forceinline__ void ms_prologue_barrier()
{
    sched_fence();
    wg_barrier();                                  // the tables and the counters before anyone uses them
    sched_fence();
}

// The flight side's exported signals of the stage-4 pass (b747::pass's read-out): its pass and the stage input's X0,
// h, Vx, Vy, w (the control side writes its 18 in place: as a helper they cost the K-step kernel 68 B of scratch)
__device__ __forceinline__ void ms_flight_signals(double *sig, int64_t n, int64_t i, const FlightPass &fp, double x0,
                                                  double h, double vx, double vy, double w)
{
    sig[S_ALPHA * n + i] = fp.alpha;
    sig[S_V * n + i] = fp.V;
    sig[S_STATE0 * n + i] = x0;
    sig[S_STATE1 * n + i] = h;
    sig[S_STATE2 * n + i] = vx;
    sig[S_STATE3 * n + i] = vy;
    sig[S_STATE5 * n + i] = w;
    sig[S_MACH * n + i] = fp.M;
    sig[S_K_ALPHA * n + i] = fp.Ka;
    sig[S_MZ * n + i] = fp.mz_aero;
    sig[S_DCM * n + i] = fp.dCm;
    sig[S_CXA * n + i] = fp.CXa;
    sig[S_CYA * n + i] = fp.CYa;
}

template <typename XT>
__global__ __launch_bounds__(kMsBlock) B747_NO_FMAC void k_model_step_split(b747_model_batch b)
{
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double xa[3][kAheadF][kMsEnvs];   // ahead -> flight, control: attitude and atmosphere of stages 1-3
    __shared__ int xai[3][kMsEnvs];              // ahead -> flight: the dCm altitude interval of stages 1-3
    __shared__ double xp[2][2][kMsEnvs];         // flight -> ahead: Vy, w of the input of stages 1-2
    __shared__ double xdl[4][kMsEnvs];           // control -> flight: delta per stage
    __shared__ double xa0[3][kMsEnvs];           // ahead -> control: sin, cos theta and h of stage 0's input
    __shared__ unsigned c_ah[1], c_fl[1], c_dl[1], c_a0[1];
    const int role = (int)threadIdx.x / kMsEnvs;   // 0 flight, 1 ahead, 2 control (wave-uniform)
    const int el = threadIdx.x & (kMsEnvs - 1);
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * kMsEnvs + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;          // (lanes past n step a copy of env n - 1 and store nothing)
    if (threadIdx.x == 0) { c_ah[0] = 0u; c_fl[0] = 0u; c_dl[0] = 0u; c_a0[0] = 0u; }
    const XT *Xg = (const XT *)b.X;
    XT *Xw = (XT *)b.X;
    double *sig = b.sig;
    const double temp = 0.5 * H;
    const double t6 = H / 6.0;

    if (role == 0) {
        // ---- flight wave (k_env_step_split's, with the pass's flight-side signals at stage 4)
        double tv[kMsTbQ];
        ms_table_loads(tv);
        double x[kNF], y[kNF], acc[kNF];
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        double km[5];                                           // 1 + aero_err (load_params)
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = b.aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        ms_stage_tables(tb, tv);
    ms_prologue_barrier();
        const FlightK fk = flight_consts();
#pragma unroll
        for (int j = 0; j < kNF; ++j) { y[j] = x[j]; acc[j] = 0.0; }
        FlightAhead a = flight_ahead<false>(x, split_kfit(0), fk);
        unsigned seen_ah = 0u, seen_dl = 0u;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));
#endif
            if (st > 0) {
                pair_wait_seen(&c_ah[0], (unsigned)st, seen_ah);
                a.sth = xa[st - 1][0][el]; a.cth = xa[st - 1][1][el]; a.h = xa[st - 1][2][el];
                a.inva = xa[st - 1][3][el]; a.rho = xa[st - 1][4][el];
                a.q0n = xa[st - 1][5][el]; a.q3n = xa[st - 1][6][el];
                a.iDC0 = xai[st - 1][el];
            }
            FlightPass fp{};
            flight_pre<false>(x, tb + zoff, split_kfit(zoff), km, fp, fk, a);
            pair_wait_seen(&c_dl[0], (unsigned)st + 1u, seen_dl);
            double dX[kNF];
            flight_post(x, xdl[st][el], fp, dX, fk);
            if (st == 3 && sig && valid)                        // the stage-4 read-out
                ms_flight_signals(sig, n, i, fp, x[0], x[1], x[4], x[5], x[6]);
            const double c = (st == 2) ? H : temp;              // RK4 combine (b747::major_step, dll@0x2c60)
            const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
            for (int j = 0; j < kNF; ++j) {
                acc[j] = acc[j] + wm * dX[j];
                x[j] = c * dX[j] + y[j];
            }
            if (st < 2) {
                xp[st][0][el] = x[5];
                xp[st][1][el] = x[6];
                pair_post(&c_fl[0], (unsigned)st + 1u);
            }
        }
        if (valid) {
#pragma unroll
            for (int j = 0; j < kNF; ++j) st_state(&Xw[kFX[j] * n + i], (XT)(acc[j] * t6 + y[j]));
        }
        return;
    }

    if (role == 1) {
        // ---- ahead wave (k_env_step_split's)
        double tv[kMsTbQ];
        ms_table_loads(tv);
        double xq[3] = {(double)Xg[1 * n + il], (double)Xg[2 * n + il], (double)Xg[5 * n + il]};   // h, q0, q3
        double vy = (double)Xg[7 * n + il], w = (double)Xg[8 * n + il];
        ms_stage_tables(tb, tv);
    ms_prologue_barrier();
        const FlightK fk = flight_consts();
        const double yq[3] = {xq[0], xq[1], xq[2]};
        FlightAhead at;
        pitch_attitude(xq[1], xq[2], fk, at);
        xa0[0][el] = at.sth; xa0[1][el] = at.cth; xa0[2][el] = xq[0];
        pair_post(&c_a0[0], 1u);
        int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(zoff));
#endif
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            if (st > 0) {
                pair_wait<0>(&c_fl[0], (unsigned)st);
                vy = xp[st - 1][0][el];
                w = xp[st - 1][1][el];
            }
            const double dq[3] = {vy, dq0_of(w, at.q3n), dq3_of(w, at.q0n)};
            const double c = (st == 2) ? H : temp;
#pragma unroll
            for (int q = 0; q < 3; ++q) xq[q] = c * dq[q] + yq[q];
            at = flight_ahead<false>(xq[1], xq[2], xq[0], split_kfit(zoff), fk);
            xa[st][0][el] = at.sth; xa[st][1][el] = at.cth; xa[st][2][el] = at.h;
            xa[st][3][el] = at.inva; xa[st][4][el] = at.rho; xa[st][5][el] = at.q0n; xa[st][6][el] = at.q3n;
            xai[st][el] = at.iDC0;
            pair_post(&c_ah[0], (unsigned)st + 1u);
        }
        return;
    }

    // ---- control wave: the delta table, the PID side X9..X17 and the MAJOR-only updates (b747::major_step with the
    // parameters of the batch: load_params)
    double tv[kMsTbQ];
    ms_table_loads(tv);
    const uint32_t k = b.k[il];
    Disc D;
    D.x_dss = b.disc[0 * n + il];
    D.y_dss = b.disc[1 * n + il];
    D.rl_prevY = b.disc[2 * n + il];
    const uint32_t flags = b.flags[il];
    const double deltaz = b.deltaz[il];
    ms_stage_tables(tb, tv);
    ms_prologue_barrier();
    D.e_prev = b.disc[3 * n + il];
    D.ed_prev = b.disc[4 * n + il];
    double x[kNC], y[kNC], acc[kNC];
#pragma unroll
    for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
    uint32_t mem = b.mem[il];
    const double vartheta = b.vartheta[il];
    const double h_zh = b.h_zh[il];
    sched_fence();
    const Hist3 uh = load_hist3(b.disc, n, il, k);
    // delta of a stage depends on that stage's pitch error (SS PID, dead zone): then the triple posts it per stage
    const bool lock = wave_any((flags & (F_PID_SS | F_RL)) != 0u);
    const double tk = t_of(k);
    const double tnew = (double)(k + 1u) * H;
    const bool dss_hit = (k % 5u) == 0u;
    const uint32_t mem_held = mem;
    double ud = 0.0;
    if (wave_any(dss_hit)) {
        ud = delay_out3(k, uh);
        D.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
    }
    if (!lock) {
        // every lane MANUAL without the dead zone: delta = the rate limiter's saturated output (RP) or deltaz
        const bool rp = (flags & F_RP) != 0u;
        double dl[4];
        delta_table(k, D, ud, dl);
        xdl[0][el] = rp ? dl[0] : deltaz;
        xdl[1][el] = rp ? dl[1] : deltaz;
        xdl[2][el] = rp ? dl[2] : deltaz;
        xdl[3][el] = rp ? dl[3] : deltaz;
        pair_post(&c_dl[0], 4u);
    }
    FlightAhead att[4];
    double hst[4];
    {
        unsigned seen_a0 = 0u;
        pair_wait_seen(&c_a0[0], 1u, seen_a0);
        att[0].sth = xa0[0][el];
        att[0].cth = xa0[1][el];
        hst[0] = xa0[2][el];
    }
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
    auto cstage = [&](int st, int zoff) __attribute__((always_inline)) {
        const double t = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
        const double theta = unit_atan2(att[st].sth, att[st].cth, split_kfit(zoff));
        double dX[kNC];
        const double delta = control_pass(x, t, theta, hst[st], P, R, dX, o, thPID);
        if (lock) {
            xdl[st][el] = delta;
            pair_post(&c_dl[0], (unsigned)st + 1u);
        }
        if (st == 3 && sig && valid) {                          // the pass's read-out (b747::pass), control side
            const double e = o.e, se = e * e, ae = fabs(e);
            sig[S_SIM_TIME * n + i] = t;
            sig[S_DVARTHETA * n + i] = e;
            sig[S_U_COM * n + i] = o.Ucom;
            sig[S_STATE4 * n + i] = theta;
            sig[S_DVARTHETA_DT * n + i] = o.ed;
            sig[S_DVARTHETA_DT_DT * n + i] = o.edd;
            sig[S_DVARTHETA_INT * n + i] = x[4];
            sig[S_AE * n + i] = ae;
            sig[S_ITAE * n + i] = x[5];
            sig[S_IAE * n + i] = x[6];
            sig[S_ISE * n + i] = x[7];
            sig[S_ITSE * n + i] = x[8];
            sig[S_SE * n + i] = se;
            sig[S_TAE * n + i] = ae * t;
            sig[S_TSE * n + i] = se * t;
            sig[S_DELTAZ_RP * n + i] = sat(o.r, B747_SAT4_LO, B747_SAT4_UP);   // (actuator's dRP)
            sig[S_U_COM_PID * n + i] = o.UPID;
            sig[S_VARTHETA_ZH * n + i] = thPID;
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
                st_state(&b.disc[(int64_t)(5u + (k & 3u)) * n + i], o.Ucom);   // (hist_put: slot k & 3)
                b.k[i] = k + 1u;
                b.mem[i] = (uint8_t)mem;
            }
        }
        const double c = (st == 2) ? H : temp;
        const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
            acc[j] = acc[j] + wm * dX[j];
            x[j] = c * dX[j] + y[j];
        }
    };
    int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(zoff));
#endif
    cstage(0, zoff);
    unsigned seen_ah = 0u;
#pragma unroll
    for (int st = 1; st < 4; ++st) {
        pair_wait_seen(&c_ah[0], (unsigned)st, seen_ah);
        att[st].sth = xa[st - 1][0][el];
        att[st].cth = xa[st - 1][1][el];
        hst[st] = xa[st - 1][2][el];
        cstage(st, zoff);
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < kNC; ++j) st_state(&Xw[(9 + j) * n + i], (XT)(acc[j] * t6 + y[j]));
    }
}

// K model steps per launch (b747_model_step with n_steps > 1; BASELINE config 2's 100-step launches, config 1) with the
// same three roles and the state in registers across the steps, as k_rollout_split does for the env: the progress
// counters count RK4 stages g = 4 s + st over the launch, the hand-off arrays are rings indexed by g, and
//   flight   stages g of every step; after each combine it posts (Vy, w) of the next stage's input (after stage 3: the
//            step's end state, the next step's stage-0 input); it waits for the ahead values of stage g (g >= 1) and
//            the delta of stage g;
//   ahead    the attitude and atmosphere of every stage g >= 1 from stage g - 1's input (xp), integrating h, q0, q3
//            itself -- the RK4 combine of a step's end included, with the flight wave's operations -- and stage g's
//            theta inputs and h for the control wave (g = 0 too); a ring of kMkRC stages, with back-pressure from the
//            control wave's progress;
//   control  the delay / DSS update and the delta table of step s + 1 right after its MAJOR update of step s (the
//            0.03 s transport delay keeps step s's command out of it; lock step posts per stage), its stages, the
//            MAJOR-only updates with the U_com history in registers.
// The state is loaded once and stored once; the 31 signals are those of the last step's stage-4 pass.
constexpr int kMkRA = 4, kMkRC = 8, kMkRP = 4, kMkRD = 4;   // ring sizes: ahead -> flight, ahead -> control, xp, delta steps

template <typename XT>
__global__ __launch_bounds__(kMsBlock) B747_NO_FMAC void k_model_steps_split(b747_model_batch b, int32_t n_steps)
{
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double xa[kMkRA][kAheadF][kMsEnvs];  // ahead -> flight: stage g's attitude and atmosphere (slot g % kMkRA)
    __shared__ int xai[kMkRA][kMsEnvs];             // ahead -> flight: stage g's dCm altitude interval
    __shared__ double xc[kMkRC][3][kMsEnvs];        // ahead -> control: stage g's sin, cos theta and h (slot g % kMkRC)
    __shared__ double xp[kMkRP][2][kMsEnvs];        // flight -> ahead: Vy, w of stage j's input (slot j % kMkRP)
    __shared__ double xdl[kMkRD][4][kMsEnvs];       // control -> flight: delta of step s's stages (slot s % kMkRD)
    __shared__ unsigned c_ah[1], c_fl[1], c_dl[1], c_cs[1];
    const int role = (int)threadIdx.x / kMsEnvs;
    const int el = threadIdx.x & (kMsEnvs - 1);
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * kMsEnvs + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    if (threadIdx.x == 0) { c_ah[0] = 0u; c_fl[0] = 0u; c_dl[0] = 0u; c_cs[0] = 0u; }
    const XT *Xg = (const XT *)b.X;
    XT *Xw = (XT *)b.X;
    double *sig = b.sig;
    const unsigned G = 4u * (unsigned)n_steps;      // stages of the launch
    const double temp = 0.5 * H;
    const double t6 = H / 6.0;

    if (role == 0) {
        // ---- flight wave
        double tv[kMsTbQ];
        ms_table_loads(tv);
        double x[kNF], y[kNF], acc[kNF];
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        double km[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = b.aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        ms_stage_tables(tb, tv);
    ms_prologue_barrier();
        const FlightK fk = flight_consts();
        unsigned seen_ah = 0u, seen_dl = 0u;
#pragma unroll 1
        for (unsigned s = 0; s < (unsigned)n_steps; ++s) {
#pragma unroll
            for (int j = 0; j < kNF; ++j) { y[j] = x[j]; acc[j] = 0.0; }
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const unsigned g = 4u * s + (unsigned)st;
                int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                asm volatile("" : "+s"(zoff));
#endif
                FlightAhead a;
                if (g == 0u) {
                    a = flight_ahead<false>(x, split_kfit(zoff), fk);   // the launch's first stage: its own
                } else {
                    pair_wait_seen(&c_ah[0], g + 1u, seen_ah);
                    const int r = (int)(g % (unsigned)kMkRA);
                    a.sth = xa[r][0][el]; a.cth = xa[r][1][el]; a.h = xa[r][2][el];
                    a.inva = xa[r][3][el]; a.rho = xa[r][4][el]; a.q0n = xa[r][5][el]; a.q3n = xa[r][6][el];
                    a.iDC0 = xai[r][el];
                }
                FlightPass fp{};
                flight_pre<false>(x, tb + zoff, split_kfit(zoff), km, fp, fk, a);
                pair_wait_seen(&c_dl[0], g + 1u, seen_dl);
                double dX[kNF];
                flight_post(x, xdl[s % (unsigned)kMkRD][st][el], fp, dX, fk);
                if (st == 3 && s + 1u == (unsigned)n_steps && sig && valid)   // the last step's stage-4 read-out
                    ms_flight_signals(sig, n, i, fp, x[0], x[1], x[4], x[5], x[6]);
                const double c = (st == 2) ? H : temp;
                const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
                for (int j = 0; j < kNF; ++j) {
                    acc[j] = acc[j] + wm * dX[j];
                    x[j] = c * dX[j] + y[j];
                }
                if (st == 3) {                                  // the step's end state (major_step)
#pragma unroll
                    for (int j = 0; j < kNF; ++j) x[j] = acc[j] * t6 + y[j];
                }
                if (g + 1u < G) {                               // (Vy, w) of stage g + 1's input, to the ahead wave
                    const int r = (int)((g + 1u) % (unsigned)kMkRP);
                    xp[r][0][el] = x[5];
                    xp[r][1][el] = x[6];
                    pair_post(&c_fl[0], g + 1u);
                }
            }
        }
        if (valid) {
#pragma unroll
            for (int j = 0; j < kNF; ++j) st_state(&Xw[kFX[j] * n + i], (XT)x[j]);
        }
        return;
    }

    if (role == 1) {
        // ---- ahead wave
        double tv[kMsTbQ];
        ms_table_loads(tv);
        double xq[3] = {(double)Xg[1 * n + il], (double)Xg[2 * n + il], (double)Xg[5 * n + il]};   // h, q0, q3
        double vy = (double)Xg[7 * n + il], w = (double)Xg[8 * n + il];
        ms_stage_tables(tb, tv);
    ms_prologue_barrier();
        const FlightK fk = flight_consts();
        unsigned seen_fl = 0u, seen_cs = 0u;
        int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(zoff));
#endif
        // post stage g's values: the flight ring (g >= 1) and the control ring (after the control wave has read the
        // stage kMkRC earlier from the same slot)
        auto post = [&](unsigned g, const FlightAhead &at) __attribute__((always_inline)) {
            if (g >= (unsigned)kMkRC) pair_wait_seen(&c_cs[0], g - (unsigned)kMkRC + 1u, seen_cs);
            const int rc = (int)(g % (unsigned)kMkRC);
            xc[rc][0][el] = at.sth; xc[rc][1][el] = at.cth; xc[rc][2][el] = at.h;
            const int ra = (int)(g % (unsigned)kMkRA);
            xa[ra][0][el] = at.sth; xa[ra][1][el] = at.cth; xa[ra][2][el] = at.h;
            xa[ra][3][el] = at.inva; xa[ra][4][el] = at.rho; xa[ra][5][el] = at.q0n; xa[ra][6][el] = at.q3n;
            xai[ra][el] = at.iDC0;
            pair_post(&c_ah[0], g + 1u);
        };
        FlightAhead at = flight_ahead<false>(xq[1], xq[2], xq[0], split_kfit(zoff), fk);
        post(0u, at);
#pragma unroll 1
        for (unsigned s = 0; s < (unsigned)n_steps; ++s) {
            const double yq[3] = {xq[0], xq[1], xq[2]};
            double accq[3] = {0.0, 0.0, 0.0};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const unsigned g = 4u * s + (unsigned)st;
                if (g > 0u) {                                   // stage g's input Vy, w from the flight wave
                    pair_wait_seen(&c_fl[0], g, seen_fl);
                    const int r = (int)(g % (unsigned)kMkRP);
                    vy = xp[r][0][el];
                    w = xp[r][1][el];
                }
                const double dq[3] = {vy, dq0_of(w, at.q3n), dq3_of(w, at.q0n)};
                const double c = (st == 2) ? H : temp;
                const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    accq[q] = accq[q] + wm * dq[q];
                    xq[q] = c * dq[q] + yq[q];
                }
                if (st == 3) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) xq[q] = accq[q] * t6 + yq[q];
                }
                if (g + 1u < G) {
                    at = flight_ahead<false>(xq[1], xq[2], xq[0], split_kfit(zoff), fk);
                    post(g + 1u, at);
                }
            }
        }
        return;
    }

    // ---- control wave
    double tv[kMsTbQ];
    ms_table_loads(tv);
    uint32_t k = b.k[il];
    Disc D;
    D.x_dss = b.disc[0 * n + il];
    D.y_dss = b.disc[1 * n + il];
    D.rl_prevY = b.disc[2 * n + il];
    D.e_prev = b.disc[3 * n + il];
    D.ed_prev = b.disc[4 * n + il];
#pragma unroll
    for (int j = 0; j < 4; ++j) D.u_hist[j] = b.disc[(5 + j) * n + il];
    const uint32_t flags = b.flags[il];
    const double deltaz = b.deltaz[il];
    ms_stage_tables(tb, tv);
    ms_prologue_barrier();
    double x[kNC], y[kNC], acc[kNC];
#pragma unroll
    for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
    uint32_t mem = b.mem[il];
    Params P{};
    P.deltaz = deltaz; P.vartheta = b.vartheta[il]; P.h_zh = b.h_zh[il]; P.flags = flags;
    const bool lock = wave_any((flags & (F_PID_SS | F_RL)) != 0u);
    const bool rp = (flags & F_RP) != 0u;
    // the delta table of the step at counter kk (every lane MANUAL without the dead zone), into ring slot s
    auto post_table = [&](uint32_t kk, double ud, unsigned s) __attribute__((always_inline)) {
        double dl[4];
        delta_table(kk, D, ud, dl);
        const int r = (int)(s % (unsigned)kMkRD);
#pragma unroll
        for (int st = 0; st < 4; ++st) xdl[r][st][el] = rp ? dl[st] : deltaz;
        pair_post(&c_dl[0], 4u * (s + 1u));
    };
    if (!lock) post_table(k, delay_out(k, D.u_hist), 0u);
    unsigned seen_ah = 0u;
    PassOut o{};
    double thPID = 0.0;
#pragma unroll 1
    for (unsigned s = 0; s < (unsigned)n_steps; ++s) {
        const double tk = t_of(k);
        const double tnew = (double)(k + 1u) * H;
        const bool dss_hit = (k % 5u) == 0u;
        const double ud = delay_out(k, D.u_hist);                // (major_step's start of step)
        D.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
        PassRef R{};
        R.has_ref = (k != 0u);
        R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
        R.e_ref = D.e_prev; R.ed_ref = D.ed_prev; R.rl_prevY = D.rl_prevY;
        R.y_dss = D.y_dss; R.mem = mem;
        const uint32_t mem_held = mem;
#pragma unroll
        for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const unsigned g = 4u * s + (unsigned)st;
            int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+s"(zoff));
#endif
            pair_wait_seen(&c_ah[0], g + 1u, seen_ah);
            const int rc = (int)(g % (unsigned)kMkRC);
            const double sth = xc[rc][0][el], cth = xc[rc][1][el], h = xc[rc][2][el];
            pair_post(&c_cs[0], g + 1u);                         // (slot rc read: the ahead wave may reuse it)
            const double t = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
            const double theta = unit_atan2(sth, cth, split_kfit(zoff));
            double dX[kNC];
            const double delta = control_pass(x, t, theta, h, P, R, dX, o, thPID);
            if (lock) {
                xdl[s % (unsigned)kMkRD][st][el] = delta;
                pair_post(&c_dl[0], g + 1u);
            }
            if (st == 3 && s + 1u == (unsigned)n_steps && sig && valid) {
                const double e = o.e, se = e * e, ae = fabs(e);
                sig[S_SIM_TIME * n + i] = t;
                sig[S_DVARTHETA * n + i] = e;
                sig[S_U_COM * n + i] = o.Ucom;
                sig[S_STATE4 * n + i] = theta;
                sig[S_DVARTHETA_DT * n + i] = o.ed;
                sig[S_DVARTHETA_DT_DT * n + i] = o.edd;
                sig[S_DVARTHETA_INT * n + i] = x[4];
                sig[S_AE * n + i] = ae;
                sig[S_ITAE * n + i] = x[5];
                sig[S_IAE * n + i] = x[6];
                sig[S_ISE * n + i] = x[7];
                sig[S_ITSE * n + i] = x[8];
                sig[S_SE * n + i] = se;
                sig[S_TAE * n + i] = ae * t;
                sig[S_TSE * n + i] = se * t;
                sig[S_DELTAZ_RP * n + i] = sat(o.r, B747_SAT4_LO, B747_SAT4_UP);
                sig[S_U_COM_PID * n + i] = o.UPID;
                sig[S_VARTHETA_ZH * n + i] = thPID;
            }
            if (st == 0) {   // MAJOR-only updates (dll@0x271a)
                D.x_dss = dss_hit ? B747_DSS_A * D.x_dss + B747_DSS_B * ud : D.x_dss;
                hist_put(D.u_hist, k, o.Ucom);
                D.rl_prevY = o.r;
                D.e_prev = o.e;
                D.ed_prev = o.ed;
                mem = o.and3_bits;
                R.has_ref = true; R.t_ref = tk; R.e_ref = o.e; R.ed_ref = o.ed; R.rl_prevY = o.r;
                R.mem = mem_held;
                // the next step's delta table: it needs only this MAJOR update (the transport delay keeps this step's
                // command out of the next step's delay output)
                if (!lock && s + 1u < (unsigned)n_steps) post_table(k + 1u, delay_out(k + 1u, D.u_hist), s + 1u);
            }
            const double c = (st == 2) ? H : temp;
            const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
            for (int j = 0; j < kNC; ++j) {
                acc[j] = acc[j] + wm * dX[j];
                x[j] = c * dX[j] + y[j];
            }
        }
#pragma unroll
        for (int j = 0; j < kNC; ++j) x[j] = acc[j] * t6 + y[j];
        k += 1u;
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < kNC; ++j) st_state(&Xw[(9 + j) * n + i], (XT)x[j]);
        store_disc(b.disc, n, i, D);
        b.k[i] = k;
        b.mem[i] = (uint8_t)mem;
    }
}

}  // namespace
