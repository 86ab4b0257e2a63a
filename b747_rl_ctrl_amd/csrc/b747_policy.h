// b747_policy.h -- fused PPO actor-critic step for the on-GPU rollout (BASELINE config 5).
//
// The reference trains stable-baselines3 PPO('MlpPolicy') (neural/agent.py:167-171 with hp = {},
// SB3 1.4 defaults): separate pi / vf extractors Linear(obs,64)-tanh-Linear(64,64)-tanh, an
// action_net Linear(64,1), a value_net Linear(64,1) and a state-independent log_std.  One rollout
// step of SB3's collect_rollouts = policy forward, Gaussian sample, log-prob, value, clip to the
// action space.  Here that is ONE kernel per step (instead of ~15 framework kernels): one lane per
// env, the small layers on the VALU from an LDS copy of the parameters, activations in registers,
// and the two 64x64 hidden layers on the matrix cores as v_mfma_f32_32x32x16_f16 with an f16
// hi/lo split of both operands (x = hi + lo; hi*hi + hi*lo + lo*hi accumulated in f32 keeps ~22
// significant bits -- within 2e-5 of the f32 torch policy, tests/test_gpu_ppo.py).  The f16
// MFMAs take 1/5 of the f32-MFMA time and, unlike them, run beside the VALU.  The second hidden
// layer is never materialised (folded straight into the 64->1 head).  tanh is 1 - 2/(2^(2x/ln2)+1)
// on the hardware exp2/rcp, with its scale and affine part folded into derived parameters.
#pragma once

#include "b747_karg.h"

namespace b747 {

constexpr int PH = 64;   // SB3 default hidden width

// Offsets in the flat parameter buffer (ActorCritic.flat_params(), include/b747.h).
struct PolicyLayout {
    int od;
    int pi_w1, pi_b1, pi_w2, pi_b2, vf_w1, vf_b1, vf_w2, vf_b2, wa, ba, wv, bv, log_std, total;
    B747_HD static constexpr PolicyLayout of(int od)
    {
        PolicyLayout L{};
        L.od = od;
        int o = 0;
        L.pi_w1 = o; o += PH * od; L.pi_b1 = o; o += PH; L.pi_w2 = o; o += PH * PH; L.pi_b2 = o; o += PH;
        L.vf_w1 = o; o += PH * od; L.vf_b1 = o; o += PH; L.vf_w2 = o; o += PH * PH; L.vf_b2 = o; o += PH;
        L.wa = o; o += PH; L.ba = o; o += 1; L.wv = o; o += PH; L.bv = o; o += 1; L.log_std = o; o += 1;
        L.total = o;
        return L;
    }
};
// tanh folded into the neighbouring layers.  With s = 2 / ln 2 and sig(u) = 1 / (2^u + 1)
// (v_exp_f32 + v_rcp_f32): tanh(z) = 1 - 2 sig(s z), so
//   layer 1:  r1 = sig(s b1 + s W1 obs)                          (h1 = 1 - 2 r1 never formed)
//   layer 2:  s z2 = s (b2 + W2 1) + (-2 s W2) r1                 (the MFMA operand is -2 s W2)
//   head:     out = (b + sum w) + sum (-2 w) sig(s z2)
// -- the scale, the "1 -" and the "-2" of every tanh move into parameters that b747_policy_pack
// derives once per update: two VALU per tanh fewer (512 per env).  Errors stay at the f32 level
// (|W2 1| and |W2 r1| are both O(|W2|); the f16 hi/lo split keeps ~22 bits of -2 s W2).
constexpr float kTanhScale = 2.8853900817779268f;   // 2 / ln 2
__device__ __forceinline__ float sig2(float u) { return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(u) + 1.0f); }

// Derived section (after the packed layers), read through LDS by the kernels:
//   l1[head][PH][od + 1] = s W1[j][0..od-1], s b1[j]      acc0[head][PH] = s (b2 + W2 1)
//   hw[head][PH] = -2 head_w      c[head] = head_b + sum head_w      log_std
struct PolicyDerived {
    int l1, acc0, hw, c, log_std, total;
    B747_HD static constexpr PolicyDerived of(int od)
    {
        PolicyDerived D{};
        int o = 0;
        D.l1 = o; o += 2 * PH * (od + 1);
        D.acc0 = o; o += 2 * PH;
        D.hw = o; o += 2 * PH;
        D.c = o; o += 2;
        D.log_std = o; o += 1;
        D.total = o;
        return D;
    }
};
constexpr int kPolicyMaxDerived = PolicyDerived::of(10).total;   // od <= 10

// Layer-2 weights of both heads, scaled by -2 s and repacked for the MFMA A operand of
// v_mfma_f32_32x32x16_f16 as an f16 hi/lo split (w = hi + lo, each f16; the products hi*hi +
// hi*lo + lo*hi carry ~22 significant bits, accumulated in f32): per head, half-element
// [((mt*4 + s)*2 + part)*64 + lane]*8 + j  =  part(-2 s W2[mt*32 + (lane & 31)][16s + 8(lane >> 5) + j])
// so each lane loads its 8 halves of one (mt, s, part) fragment with one dwordx4.
constexpr int kPackPerHead = 64 * PH;            // floats (= 2 * 4096 halves)
B747_HD int policy_packed_offset(int od) { return PolicyLayout::of(od).total; }
B747_HD int policy_derived_offset(int od) { return PolicyLayout::of(od).total + 2 * kPackPerHead; }
// Layer 1 on the matrix cores (obs_dim <= kL1MaxOD): per head and 32-unit tile mt, the A fragment of ONE
// v_mfma_f32_32x32x16_f16 whose K = 16 slots hold, for unit u (s = kTanhScale, x = hi + lo f16 split),
//   A[u] = [hi(s W1[u][0..od-1]), hi(s W1[u][..]), lo(s W1[u][..]), hi(s b1[u]), lo(s b1[u]), 0 ...]
// against the per-env B column
//   B[e] = [hi(obs[e][0..od-1]),  lo(obs[e][..]),   hi(obs[e][..]),  1,           1,           0 ...]
// so one product gives s (W1 obs + b1) with the hi*hi + hi*lo + lo*hi terms of the f16 split (~22 bits):
// 4 MFMAs per head replace 64 x od VALU FMAs.  Half [((head * 2 + mt) * 64 + lane) * 8 + j] = A[mt * 32 +
// (lane & 31)][8 (lane >> 5) + j]: one dwordx4 per lane per fragment.  Starts 16-byte aligned.
constexpr int kL1MaxOD = 4;                      // 3 od + 2 <= 16
constexpr int kL1PackFloats = 2 * 2 * 64 * 4;    // 1024 floats = 2048 halves
B747_HD int policy_l1pack_offset(int od) { return (policy_derived_offset(od) + PolicyDerived::of(od).total + 3) & ~3; }
B747_HD int policy_total_params(int od) { return policy_l1pack_offset(od) + kL1PackFloats; }


#ifndef B747_POLICY_NO_KERNELS
// One thread per packed half-element, then one per derived float, then one per layer-1 fragment half.
B747_HD constexpr int policy_pack_threads(int od) { return 4 * kPackPerHead + PolicyDerived::of(od).total + 2 * kL1PackFloats; }
__global__ void k_policy_pack(float *params, int od)
{
    const PolicyLayout L = PolicyLayout::of(od);
    const PolicyDerived D = PolicyDerived::of(od);
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int l1i = idx - (4 * kPackPerHead + D.total);
    if (l1i >= 0) {   // layer-1 A fragments (policy_l1pack_offset): half ((head * 2 + mt) * 64 + lane) * 8 + j
        if (l1i >= 2 * kL1PackFloats) return;
        const int j = l1i & 7, lane = (l1i >> 3) & 63, frag = l1i >> 9, mt = frag & 1, head = frag >> 1;
        const int u = mt * 32 + (lane & 31), k = 8 * (lane >> 5) + j;
        const int w1 = head ? L.vf_w1 : L.pi_w1, b1 = head ? L.vf_b1 : L.pi_b1;
        auto split = [](float x, bool lo) {
            const _Float16 h = (_Float16)x;
            return lo ? (_Float16)(x - (float)h) : h;
        };
        _Float16 v = (_Float16)0.0f;
        if (od <= kL1MaxOD) {
            if (k < 2 * od) v = split(kTanhScale * params[w1 + u * od + (k % od)], false);       // hi, hi
            else if (k < 3 * od) v = split(kTanhScale * params[w1 + u * od + (k - 2 * od)], true);  // lo
            else if (k == 3 * od) v = split(kTanhScale * params[b1 + u], false);
            else if (k == 3 * od + 1) v = split(kTanhScale * params[b1 + u], true);
        }
        reinterpret_cast<_Float16 *>(params + policy_l1pack_offset(od))[l1i] = v;
        return;
    }
    if (idx < 2 * 2 * kPackPerHead) {
        const int head = idx / (2 * kPackPerHead), rem = idx % (2 * kPackPerHead);
        const int j = rem & 7, lane = (rem >> 3) & 63, frag = rem >> 9;  // frag = (mt*4 + s)*2 + part
        const int part = frag & 1, s = (frag >> 1) & 3, mt = frag >> 3;
        const int w2 = head ? L.vf_w2 : L.pi_w2;
        const float x = -2.0f * kTanhScale * params[w2 + (mt * 32 + (lane & 31)) * PH + 16 * s + 8 * (lane >> 5) + j];
        const _Float16 hi = (_Float16)x;
        const _Float16 v = part ? (_Float16)(x - (float)hi) : hi;
        reinterpret_cast<_Float16 *>(params + policy_packed_offset(od) + head * kPackPerHead)[rem] = v;
        return;
    }
    const int d = idx - 2 * 2 * kPackPerHead;
    if (d >= D.total) return;
    float v;
    if (d < D.acc0) {
        const int head = d / (PH * (od + 1)), rem = d % (PH * (od + 1)), j = rem / (od + 1), k = rem % (od + 1);
        const int w1 = head ? L.vf_w1 : L.pi_w1, b1 = head ? L.vf_b1 : L.pi_b1;
        v = kTanhScale * (k < od ? params[w1 + j * od + k] : params[b1 + j]);
    } else if (d < D.hw) {
        const int head = (d - D.acc0) / PH, row = (d - D.acc0) % PH;
        const int w2 = head ? L.vf_w2 : L.pi_w2, b2 = head ? L.vf_b2 : L.pi_b2;
        float a = params[b2 + row];
        for (int k = 0; k < PH; ++k) a += params[w2 + row * PH + k];
        v = kTanhScale * a;
    } else if (d < D.c) {
        const int head = (d - D.hw) / PH, row = (d - D.hw) % PH;
        v = -2.0f * params[(head ? L.wv : L.wa) + row];
    } else if (d < D.log_std) {
        const int head = d - D.c;
        float a = params[head ? L.bv : L.ba];
        for (int k = 0; k < PH; ++k) a += params[(head ? L.wv : L.wa) + k];
        v = a;
    } else {
        v = params[L.log_std];
    }
    params[policy_derived_offset(od) + d] = v;
}
#endif  // B747_POLICY_NO_KERNELS

// The derived section's LDS copy: loads issued by load(), LDS writes by store() (callers put other
// loads in between), a __syncthreads / wg_barrier after store().
template <int OD, int BLOCK>
struct PolicyStage {
    static constexpr int kN = PolicyDerived::of(OD).total, kQ = (kN + BLOCK - 1) / BLOCK;
    float v[kQ];
    __device__ __forceinline__ void load(const float *__restrict__ params, int tid)
    {
        const float *d = params + policy_derived_offset(OD);
#pragma unroll
        for (int q = 0; q < kQ; ++q) v[q] = (tid + BLOCK * q < kN) ? d[tid + BLOCK * q] : 0.0f;
    }
    __device__ __forceinline__ void store(float *w, int tid) const
    {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            if (tid + BLOCK * q < kN) w[tid + BLOCK * q] = v[q];
    }
};

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void swap_halves(float &x, float &y)
{
    // lanes 32-63 of x <-> lanes 0-31 of y (v_permlane32_swap_b32)
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}

// Both extractors + heads for the wave's 64 envs (lane = env):
//   out_h = head_w . tanh(W2_h tanh(W1_h obs + b1_h) + b2_h) + head_b      (h = pi, vf)
// Layer 1 on the VALU (K = obs_dim is tiny); layer 2 as D[out][env] = W2 . H1^T on
// v_mfma_f32_32x32x16_f16 (2 x 2 tiles of 32 x 32 per head, 4 K-steps, 3 split products): the
// B fragments of K-step s are the lanes' own h1[16s..16s+15] after one half-swap per register,
// so H1 never leaves registers; the head dot product is taken per lane over its 32 rows of D and
// completed with one more swap.
union H8 {
    half8 h;
    uint32_t u[4];
    uint4 v;
};

// A fragments of one head: [mt][s][part] (16 fragments, 64 VGPRs)
__device__ __forceinline__ void load_packed(const float *__restrict__ packed, int lane, H8 *A)
{
    const uint4 *p = reinterpret_cast<const uint4 *>(packed) + lane;
#pragma unroll
    for (int f = 0; f < 16; ++f) A[f].v = p[f * 64];
}

// The f16 hi/lo split of a pair of f32 values into two packed dwords: hi = RNE(x) (one v_cvt_pk_f16_f32 per
// pair), lo = RNE(x - hi) (x - hi is exact in f32).  (A v_fma_mixlo/mixhi_f16 form of lo -- 2 VALU per pair
// instead of 3 -- measured 0.4 us/step SLOWER in the fused rollout: tools/ab_ppo.sh, profiles/EXPERIMENTS.md.)
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
// gfx950 hazard (tests/test_isa_packed_hazard.py): a VALU read issued fewer than 2 wait states after
// a packed-fp32 write sees stale lanes 48-63, and this compiler does not pad it.  The pair's x - hi is one
// v_pk_add_f32 (neg on the second operand) written as inline asm with its own s_nop 1, so every reader is at least
// 2 wait states behind by construction (the compiler's own packed add is the round-3 form that needs the padding).
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t &hi, uint32_t &lo)
{
    const half2v h = __builtin_convertvector((float2v){x0, x1}, half2v);
    hi = __builtin_bit_cast(uint32_t, h);
#if defined(__HIP_DEVICE_COMPILE__)
    const float2v hf = {(float)h[0], (float)h[1]};
    float2v d;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]\n\ts_nop 1" : "=v"(d) : "v"((float2v){x0, x1}), "v"(hf));
    const half2v l = __builtin_convertvector(d, half2v);
#else
    const half2v l = {(_Float16)(x0 - (float)h[0]), (_Float16)(x1 - (float)h[1])};
#endif
    lo = __builtin_bit_cast(uint32_t, l);
}

// B fragments of K-step s for both env tiles from the lanes' own h1 (f16 hi/lo split + one half
// swap per register): tile 0 = envs 0..31, tile 1 = envs 32..63.
__device__ __forceinline__ void b_frags(const float *h1, int s, H8 &b0h, H8 &b0l, H8 &b1h, H8 &b1l)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        split_pair(h1[16 * s + 2 * r], h1[16 * s + 2 * r + 1], b0h.u[r], b0l.u[r]);
        split_pair(h1[16 * s + 8 + 2 * r], h1[16 * s + 8 + 2 * r + 1], b1h.u[r], b1l.u[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        auto th = __builtin_amdgcn_permlane32_swap(b0h.u[r], b1h.u[r], false, false);
        auto tl = __builtin_amdgcn_permlane32_swap(b0l.u[r], b1l.u[r], false, false);
        b0h.u[r] = th[0]; b1h.u[r] = th[1];
        b0l.u[r] = tl[0]; b1l.u[r] = tl[1];
    }
}

#define B747_MFMA16(acc, a, b) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16((a).h, (b).h, acc, 0, 0, 0)

// K-step s of D[out][env] = C + W2 . H1^T for one head (3 split products on 2 x 2 tiles); step 0's
// first MFMA of each tile reads the bias tile (c0 for rows 0-31, c1 for rows 32-63) as its C operand.
__device__ __forceinline__ void layer2_step(const H8 *A, const float *h1, int s, const f32x16 &c0, const f32x16 &c1,
                                            f32x16 &d00, f32x16 &d01, f32x16 &d10, f32x16 &d11)
{
    H8 b0h, b0l, b1h, b1l;
    b_frags(h1, s, b0h, b0l, b1h, b1l);
    const H8 &a0h = A[(0 * 4 + s) * 2], &a0l = A[(0 * 4 + s) * 2 + 1];
    const H8 &a1h = A[(1 * 4 + s) * 2], &a1l = A[(1 * 4 + s) * 2 + 1];
    if (s == 0) {
        d00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b0h.h, c0, 0, 0, 0);
        d01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b1h.h, c0, 0, 0, 0);
        d10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b0h.h, c1, 0, 0, 0);
        d11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b1h.h, c1, 0, 0, 0);
    } else {
        B747_MFMA16(d00, a0h, b0h); B747_MFMA16(d01, a0h, b1h); B747_MFMA16(d10, a1h, b0h); B747_MFMA16(d11, a1h, b1h);
    }
    B747_MFMA16(d00, a0h, b0l); B747_MFMA16(d01, a0h, b1l); B747_MFMA16(d10, a1h, b0l); B747_MFMA16(d11, a1h, b1l);
    B747_MFMA16(d00, a0l, b0h); B747_MFMA16(d01, a0l, b1h); B747_MFMA16(d10, a1l, b0h); B747_MFMA16(d11, a1l, b1h);
}

__device__ __forceinline__ void layer2(const H8 *A, const float *h1, const f32x16 &c0, const f32x16 &c1,
                                       f32x16 &d00, f32x16 &d01, f32x16 &d10, f32x16 &d11)
{
#pragma unroll
    for (int s = 0; s < 4; ++s) layer2_step(A, h1, s, c0, c1, d00, d01, d10, d11);
}

// ---- layer 1 on the matrix cores (obs_dim <= kL1MaxOD; the A fragments are b747_policy_pack's l1 section) ----
// The B operand of both env tiles from the lanes' own observations: lane l holds env l's K column
// [hi(obs), lo(obs), hi(obs), 1, 1, 0...] as halves 0-7 (V_lo) and 8-15 (V_hi); one half swap per dword gives
// tile 0 (envs 0-31: lanes < 32 their own V_lo, lanes >= 32 the V_hi of env l - 32) and tile 1 (envs 32-63).
template <int OD>
__device__ __forceinline__ void l1_obs_frags(const float *obs, H8 &t0, H8 &t1)
{
    static_assert(3 * OD + 2 <= 16, "layer-1 K column");
    _Float16 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = (_Float16)0.0f;
#pragma unroll
    for (int k = 0; k < OD; ++k) {
        // |obs| beyond the f16 range would give hi = +-inf and lo = -+inf, so inf - inf = NaN where the f32 policy
        // saturates: clamp to +-65504 first (the layer's tanh is saturated there either way; NaN stays NaN)
        // (selects, not branches: the nested conditional compiled to two divergent branches per component)
        const float x0 = obs[k];
        const float x1 = B747_UNPRED(x0 > 65504.0f) ? 65504.0f : x0;
        const float x = B747_UNPRED(x1 < -65504.0f) ? -65504.0f : x1;
        const _Float16 h = (_Float16)x;
        v[k] = h;
#if defined(__HIP_DEVICE_COMPILE__)
        float d;   // x - hi as a plain v_sub_f32 the SLP vectoriser cannot pack (the hazard of split_pair)
        asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(x), "v"((float)h));
        v[OD + k] = (_Float16)d;
#else
        v[OD + k] = (_Float16)(x - (float)h);
#endif
        v[2 * OD + k] = h;
    }
    v[3 * OD] = (_Float16)1.0f;
    v[3 * OD + 1] = (_Float16)1.0f;
    H8 lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) { lo.h[j] = v[j]; hi.h[j] = v[8 + j]; }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        auto w = __builtin_amdgcn_permlane32_swap(lo.u[r], hi.u[r], false, false);
        t0.u[r] = w[0];
        t1.u[r] = w[1];
    }
}

// Layer-2 B fragments of K-step s from layer-1 activations in the MFMA C/D layout (r[mt][nt], lane l: env
// nt*32 + (l & 31), unit mt*32 + (e & 3) + 8 (e >> 2) + 4 (l >> 5) for element e): K-step s reads rows
// 16 (s & 1) .. +15 of tile mt = s >> 1; lanes < 32 need rows +0..7, lanes >= 32 rows +8..15, and one half
// swap per pair of elements (8q + j, 8q + 4 + j) hands each half the four rows it lacks.
__device__ __forceinline__ void b_frags_d(f32x16 (&r)[2][2], int s, H8 &b0h, H8 &b0l, H8 &b1h, H8 &b1l)
{
    const int mt = s >> 1, q = s & 1;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x = r[mt][nt][8 * q + j], y = r[mt][nt][8 * q + 4 + j];
            swap_halves(x, y);
            v[j] = x;
            v[4 + j] = y;
        }
        H8 &bh = nt ? b1h : b0h, &bl = nt ? b1l : b0l;
#pragma unroll
        for (int r = 0; r < 4; ++r) split_pair(v[2 * r], v[2 * r + 1], bh.u[r], bl.u[r]);
    }
}

__device__ __forceinline__ void layer2_d(const H8 *A, f32x16 (&r)[2][2], const f32x16 &c0, const f32x16 &c1,
                                         f32x16 &d00, f32x16 &d01, f32x16 &d10, f32x16 &d11)
{
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        H8 b0h, b0l, b1h, b1l;
        b_frags_d(r, s, b0h, b0l, b1h, b1l);
        const H8 &a0h = A[(0 * 4 + s) * 2], &a0l = A[(0 * 4 + s) * 2 + 1];
        const H8 &a1h = A[(1 * 4 + s) * 2], &a1l = A[(1 * 4 + s) * 2 + 1];
        if (s == 0) {
            d00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b0h.h, c0, 0, 0, 0);
            d01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b1h.h, c0, 0, 0, 0);
            d10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b0h.h, c1, 0, 0, 0);
            d11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b1h.h, c1, 0, 0, 0);
        } else {
            B747_MFMA16(d00, a0h, b0h); B747_MFMA16(d01, a0h, b1h); B747_MFMA16(d10, a1h, b0h); B747_MFMA16(d11, a1h, b1h);
        }
        B747_MFMA16(d00, a0h, b0l); B747_MFMA16(d01, a0h, b1l); B747_MFMA16(d10, a1h, b0l); B747_MFMA16(d11, a1h, b1l);
        B747_MFMA16(d00, a0l, b0h); B747_MFMA16(d01, a0l, b1h); B747_MFMA16(d10, a1l, b0h); B747_MFMA16(d11, a1l, b1h);
    }
}

// Layer 1 of one head: r[mt][nt] = sig(s (W1 obs + b1)) in the C/D layout, 4 MFMAs
__device__ __forceinline__ void layer1_mfma(const H8 &a0, const H8 &a1, const H8 &ob0, const H8 &ob1, f32x16 (&r)[2][2])
{
    const f32x16 zero = {};
    r[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0.h, ob0.h, zero, 0, 0, 0);
    r[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0.h, ob1.h, zero, 0, 0, 0);
    r[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1.h, ob0.h, zero, 0, 0, 0);
    r[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1.h, ob1.h, zero, 0, 0, 0);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int e = 0; e < 16; ++e) r[mt][nt][e] = sig2(r[mt][nt][e]);
}

// The bias tiles of a head in the C/D layout (row (r & 3) + 8 (r >> 2) + 4 (lane >> 5), +32 for c1)
__device__ __forceinline__ void bias_tiles(const float *__restrict__ w, int o_acc0, int hb, f32x16 &c0, f32x16 &c1)
{
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row0 = (r & 3) + 8 * (r >> 2) + hb;
        c0[r] = w[o_acc0 + row0];
        c1[r] = w[o_acc0 + 32 + row0];
    }
}

// Epilogue slice r of a head: lane-partial sums over rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
// and 32 + that, for both env tiles (C/D map: col = lane & 31, row as above).  w = the LDS copy of
// the derived section; d = s z2 (bias included by layer2).
__device__ __forceinline__ void head_slice(const float *__restrict__ w, int o_hw, const f32x16 &d00,
                                           const f32x16 &d01, const f32x16 &d10, const f32x16 &d11, int r,
                                           int hb, float &p0, float &p1)
{
    const int row0 = (r & 3) + 8 * (r >> 2) + hb, row1 = 32 + row0;
    const float w0 = w[o_hw + row0], w1 = w[o_hw + row1];
    p0 = fmaf(w0, sig2(d00[r]), p0);
    p0 = fmaf(w1, sig2(d10[r]), p0);
    p1 = fmaf(w0, sig2(d01[r]), p1);
    p1 = fmaf(w1, sig2(d11[r]), p1);
}

// r1[j] = sig(s b1[j] + s W1[j] . obs): the unit's od + 1 derived floats are contiguous.  g = the
// derived section in global memory: the addresses are wave-uniform, so these are scalar loads
// (s_load_dwordx*, issued many units ahead into SGPRs) instead of LDS reads that each wait out
// the LDS latency one unit ahead.
template <int OD>
__device__ __forceinline__ float layer1_unit(const float *__restrict__ g, int o_l1, const float *obs, int j)
{
    const float *u = g + o_l1 + j * (OD + 1);
    float a = u[OD];
#pragma unroll
    for (int k = 0; k < OD; ++k) a = fmaf(u[k], obs[k], a);
    return sig2(a);
}

// Both heads, overlapped by the scheduler (layer-1 work of one head beside the other's MFMAs).
// w = LDS copy of the derived section (PolicyStage); params = the flat buffer (global, the packed
// layers at policy_packed_offset).  Layer 1 reads the derived section from g: the global copy
// (scalar loads; the fused rollout kernel, whose scalar cache is warm after its first step) or w
// (LDS; k_policy_act, one step per launch: there 32 cold scalar-cache lines cost more, 24.7 vs
// 23.8 us per two-launch rollout step).
// fr (nullable): the matrix-core A fragments staged in LDS by the caller (kPolicyFragUint4 uint4, layout
// [f][64 lanes]: f 0-3 the layer-1 fragments (head * 2 + mt), 4-19 the policy head's layer-2 fragments, 20-35
// the value head's) -- a multi-step kernel reads them from there instead of from L2 every step.
constexpr int kPolicyFragUint4 = (4 + 2 * 16) * 64;
// HEADS (the matrix-core layer-1 path only; the others evaluate both): bit 0 the policy head (mean), bit 1 the
// value head (value); a head left out returns its bias alone.
template <int OD, int HEADS = 3>
__device__ __forceinline__ void actor_critic(const float *__restrict__ w, const float *__restrict__ params,
                                             const float *__restrict__ g, const float *obs, int lane, float &mean,
                                             float &value, const uint4 *fr = nullptr)
{
    static_assert(HEADS >= 1 && HEADS <= 3, "HEADS: bit 0 policy, bit 1 value");
    constexpr bool kPi = (HEADS & 1) != 0, kVf = (HEADS & 2) != 0;
    const float *__restrict__ packed = params + policy_packed_offset(OD);
    constexpr PolicyDerived D = PolicyDerived::of(OD);
    constexpr int l1v = D.l1 + PH * (OD + 1);
    const int hb = 4 * (lane >> 5);
    float pp0 = 0.0f, pp1 = 0.0f, vp0 = 0.0f, vp1 = 0.0f;
    if constexpr (OD <= kL1MaxOD) {
        // layer 1 on the matrix cores (policy_l1pack_offset), then layer 2 straight from its C/D layout
        const uint4 *l1 = fr ? fr + lane : reinterpret_cast<const uint4 *>(params + policy_l1pack_offset(OD)) + lane;
        H8 A1[4];
#pragma unroll
        for (int f = 0; f < 4; ++f)   // (head * 2 + mt)
            if ((f < 2) ? kPi : kVf) A1[f].v = l1[f * 64];
        H8 Ap[16], Av[16];
        if (fr) {
#pragma unroll
            for (int f = 0; f < 16; ++f) {
                if (kPi) Ap[f].v = fr[(4 + f) * 64 + lane];
                if (kVf) Av[f].v = fr[(20 + f) * 64 + lane];
            }
        } else {
            if (kPi) load_packed(packed, lane, Ap);
            if (kVf) load_packed(packed + kPackPerHead, lane, Av);
        }
        H8 ob0, ob1;
        l1_obs_frags<OD>(obs, ob0, ob1);
        f32x16 rp[2][2], rv[2][2];
        f32x16 c0, c1, p00, p01, p10, p11, v00, v01, v10, v11;   // [mt][nt]
        if constexpr (HEADS == 3) {
            layer1_mfma(A1[0], A1[1], ob0, ob1, rp);
            layer1_mfma(A1[2], A1[3], ob0, ob1, rv);
            bias_tiles(w, D.acc0, hb, c0, c1);
            layer2_d(Ap, rp, c0, c1, p00, p01, p10, p11);
            bias_tiles(w, D.acc0 + PH, hb, c0, c1);
            layer2_d(Av, rv, c0, c1, v00, v01, v10, v11);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                head_slice(w, D.hw, p00, p01, p10, p11, r, hb, pp0, pp1);
                head_slice(w, D.hw + PH, v00, v01, v10, v11, r, hb, vp0, vp1);
            }
        } else if constexpr (kPi) {
            layer1_mfma(A1[0], A1[1], ob0, ob1, rp);
            bias_tiles(w, D.acc0, hb, c0, c1);
            layer2_d(Ap, rp, c0, c1, p00, p01, p10, p11);
#pragma unroll
            for (int r = 0; r < 16; ++r) head_slice(w, D.hw, p00, p01, p10, p11, r, hb, pp0, pp1);
        } else {
            layer1_mfma(A1[2], A1[3], ob0, ob1, rv);
            bias_tiles(w, D.acc0 + PH, hb, c0, c1);
            layer2_d(Av, rv, c0, c1, v00, v01, v10, v11);
#pragma unroll
            for (int r = 0; r < 16; ++r) head_slice(w, D.hw + PH, v00, v01, v10, v11, r, hb, vp0, vp1);
        }
        (void)g;
        (void)l1v;
    } else {
        float hp[PH], hv[PH];
        H8 Ap[16], Av[16];
        load_packed(packed, lane, Ap);                     // global loads first: in flight during layer 1
        load_packed(packed + kPackPerHead, lane, Av);
#pragma unroll
        for (int j = 0; j < PH; ++j) {
            hp[j] = layer1_unit<OD>(g, D.l1, obs, j);
            hv[j] = layer1_unit<OD>(g, l1v, obs, j);
        }
        f32x16 c0, c1, p00, p01, p10, p11, v00, v01, v10, v11;   // [mt][nt]
        bias_tiles(w, D.acc0, hb, c0, c1);
        layer2(Ap, hp, c0, c1, p00, p01, p10, p11);
        bias_tiles(w, D.acc0 + PH, hb, c0, c1);
        layer2(Av, hv, c0, c1, v00, v01, v10, v11);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            head_slice(w, D.hw, p00, p01, p10, p11, r, hb, pp0, pp1);
            head_slice(w, D.hw + PH, v00, v01, v10, v11, r, hb, vp0, vp1);
        }
    }
    // lane l < 32 (env l): x0(l) + x0(l + 32); lane l >= 32 (env l): x1(l - 32) + x1(l)
    swap_halves(pp0, pp1);
    swap_halves(vp0, vp1);
    mean = (pp0 + pp1) + w[D.c];
    value = (vp0 + vp1) + w[D.c + 1];
}

// The Gaussian draw of env id `env` at rollout counter ctr (Philox4x32-10 keyed by seed), shared by
// k_policy_act and the fused rollout kernel so both sample the same noise.
__device__ __forceinline__ float policy_noise(uint64_t seed, uint64_t ctr, uint64_t env)
{
    Rng r;
    r.init(seed ^ (ctr >> 32) * 0x9E3779B97F4A7C15ull, env, (uint32_t)ctr);
    const float u1 = ((float)(r.u32() >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(r.u32() >> 8) * (1.0f / 16777216.0f);
    // Box-Muller on the hardware v_log_f32 (log2) / v_sqrt_f32 / v_cos_f32 (argument in revolutions):
    // u1 >= 2^-24 is a normal float and u2 in [0, 1) is inside v_cos_f32's range, so ocml's range
    // reduction and denormal handling buy nothing here (tools/ab_ppo.sh: fused rollout -0.2 us/step,
    // two-launch -0.4; an opaque per-call Philox key to keep the round keys off the SGPR spill lanes
    // measured +0.1 to +0.3 and was dropped)
    return __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1)) * __builtin_amdgcn_cosf(u2);
}

#ifndef B747_POLICY_NO_KERNELS
// obs [N][OD] -> obs_out (copy, nullable), act_out (unclipped sample), logp_out, value_out,
// env_action (clipped to [act_lo, act_hi]).  noise [N] (nullable): standard normal draws; when
// NULL they come from Philox4x32-10 keyed by seed with counter (env id, *step_base + step) --
// step_base lives in device memory so a captured rollout graph draws fresh noise per replay.
// Every wave runs the MFMA part with all 64 lanes (lanes past N compute on env N-1's obs and
// store nothing).
template <int OD>
__global__ __launch_bounds__(256) void k_policy_act(const float *__restrict__ params, int64_t n,
                                                    const float *__restrict__ obs, const float *__restrict__ noise,
                                                    uint64_t seed, const uint64_t *step_base, uint32_t step,
                                                    int64_t env_offset,
                                                    float *obs_out, float *act_out, float *logp_out,
                                                    float *value_out, float *env_action, float act_lo, float act_hi)
{
    constexpr PolicyDerived D = PolicyDerived::of(OD);
    __shared__ float w[D.total];
    prefetch_kernargs_wait(prefetch_kernargs_issue<128>());   // 17 arguments, 2 lines
    // Stage the derived section (the 64x64 layers feed the MFMAs from the packed copy)
    PolicyStage<OD, 256> stage;
    stage.load(params, threadIdx.x);
    stage.store(w, threadIdx.x);
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = i0 < n ? i0 : n - 1;
    const int lane = threadIdx.x & 63;

    float o[OD];
#pragma unroll
    for (int k = 0; k < OD; ++k) o[k] = obs[i * OD + k];
    float mean, value;
    actor_critic<OD>(w, params, w, o, lane, mean, value);
    if (i0 >= n) return;
    if (obs_out) {
#pragma unroll
        for (int k = 0; k < OD; ++k) obs_out[i * OD + k] = o[k];
    }
    const float z = noise ? noise[i] : policy_noise(seed, (step_base ? *step_base : 0u) + step, (uint64_t)(env_offset + i));
    const float log_std = w[D.log_std];
    const float a = mean + expf(log_std) * z;
    act_out[i] = a;
    // log N(a; mean, std) with a - mean = std * z
    logp_out[i] = -0.5f * z * z - log_std - 0.918938533204672742f;
    value_out[i] = value;
    env_action[i] = fminf(fmaxf(a, act_lo), act_hi);
}

// The value head over R observation rows (obs [R][OD] -> value_out [R]): the fused rollout's deferred value
// pass -- V(obs_t) for every row t * n + i of the rollout's obs_buf, with the rollout's
// parameters, in one batched launch instead of inside the latency-bound rollout loop.  Each wave evaluates
// kValueTiles tiles of 64 rows with its matrix-core A fragments loaded once; 124 VGPRs, four waves per SIMD.
// Rows past R compute on row R - 1 and store nothing (every wave runs the MFMAs with all 64 lanes).
// step_base (nullable): the rollout's Philox counter base, advanced by `advance` here -- the launch after the rollout
// kernel's last read of it -- so that a captured rollout graph needs no separate counter kernel (ABI 10).
constexpr int kValueTiles = 4;   // (1, 4 or 16 tiles per wave, 2 or 4 waves per SIMD: all within 2.51-2.62 us per step)
template <int OD>
__global__ __launch_bounds__(256, 2) void k_policy_value(const float *__restrict__ params, int64_t rows,
                                                     const float *__restrict__ obs, float *__restrict__ value_out,
                                                     uint64_t *step_base, uint32_t advance)
{
    if (step_base && blockIdx.x == 0 && threadIdx.x == 0)   // (one lane's vector atomic)
        __hip_atomic_fetch_add(step_base, (uint64_t)advance, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    static_assert(OD <= kL1MaxOD, "k_policy_value: the matrix-core layer 1");
    constexpr PolicyDerived D = PolicyDerived::of(OD);
    __shared__ float w[D.total];
    PolicyStage<OD, 256> stage;
    stage.load(params, threadIdx.x);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hb = 4 * (lane >> 5);
    const uint4 *l1 = reinterpret_cast<const uint4 *>(params + policy_l1pack_offset(OD)) + lane;
    H8 A1[2], Av[16];
    A1[0].v = l1[2 * 64];      // the value head's layer-1 fragments (head 1, mt 0 / 1)
    A1[1].v = l1[3 * 64];
    load_packed(params + policy_packed_offset(OD) + kPackPerHead, lane, Av);
    stage.store(w, threadIdx.x);
    __syncthreads();
    const float bias = w[D.c + 1];
    auto row_of = [&](int t) -> int64_t { return (((int64_t)blockIdx.x * kValueTiles + t) * 4 + wave) * 64 + lane; };
    float on[OD];   // the next tile's observation, in flight while this tile computes
    {
        const int64_t r = row_of(0) < rows ? row_of(0) : rows - 1;
#pragma unroll
        for (int k = 0; k < OD; ++k) on[k] = obs[r * OD + k];
    }
#pragma unroll 1
    for (int t = 0; t < kValueTiles; ++t) {
        const int64_t r0 = row_of(t);
        float o[OD];
#pragma unroll
        for (int k = 0; k < OD; ++k) o[k] = on[k];
        if (t + 1 < kValueTiles) {
            const int64_t r1 = row_of(t + 1) < rows ? row_of(t + 1) : rows - 1;
#pragma unroll
            for (int k = 0; k < OD; ++k) on[k] = obs[r1 * OD + k];
        }
        H8 ob0, ob1;
        l1_obs_frags<OD>(o, ob0, ob1);
        f32x16 rv[2][2], c0, c1, v00, v01, v10, v11;
        layer1_mfma(A1[0], A1[1], ob0, ob1, rv);
        bias_tiles(w, D.acc0 + PH, hb, c0, c1);
        layer2_d(Av, rv, c0, c1, v00, v01, v10, v11);
        float vp0 = 0.0f, vp1 = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) head_slice(w, D.hw + PH, v00, v01, v10, v11, q, hb, vp0, vp1);
        swap_halves(vp0, vp1);
        if (r0 < rows) value_out[r0] = (vp0 + vp1) + bias;
    }
}
B747_HD constexpr int64_t policy_value_blocks(int64_t rows) { return (rows + 256 * kValueTiles - 1) / (256 * kValueTiles); }
#endif  // B747_POLICY_NO_KERNELS

}  // namespace b747
