// b747_policy.h -- fused PPO actor-critic step for the on-GPU rollout (BASELINE config 5).
//
// The reference trains stable-baselines3 PPO('MlpPolicy') (neural/agent.py:167-171 with hp = {},
// SB3 1.4 defaults): separate pi / vf extractors Linear(obs,64)-tanh-Linear(64,64)-tanh, an
// action_net Linear(64,1), a value_net Linear(64,1) and a state-independent log_std.  One rollout
// step of SB3's collect_rollouts = policy forward, Gaussian sample, log-prob, value, clip to the
// action space.  Here that is ONE kernel per step (instead of ~15 framework kernels): one lane per
// env, the 64x64 hidden layers on the f32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32
// fma chains, the same numerics as VALU fmaf), the small layers on the VALU from an LDS copy of
// the parameters, activations in registers, the second hidden layer never materialised (folded
// straight into the 64->1 head).  tanh is 1 - 2/(exp(2x)+1) with the hardware exp2/rcp,
// within ~2e-7 (absolute) of libm.
#pragma once

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
constexpr int kPolicyMaxParams = 2 * (PH * 10 + PH + PH * PH + PH) + 2 * (PH + 1) + 1;   // od <= 10

// tanh(x) = 1 - 2 / (2^(2x log2 e) + 1) on the transcendental unit (v_exp_f32, v_rcp_f32):
// 5 instructions, absolute error ~2e-7 (saturates correctly to +-1 through exp2 -> inf / 0).
__device__ __forceinline__ float tanh_fast(float x)
{
    const float t = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);   // 2 / ln 2
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(t + 1.0f), 1.0f);
}

// Layer-2 weights of both heads repacked for the MFMA A operand (b747_policy_pack): element
// [head][q][lane][e] = W2[mt*32 + (lane & 31)][2*s + (lane >> 5)] with j = 4q + e, mt = j >> 5,
// s = j & 31 -- each lane then loads its 64 A values with 16 coalesced dwordx4 loads.
constexpr int kPackPerHead = 64 * PH;
B747_HD int policy_total_params(int od) { return PolicyLayout::of(od).total + 2 * kPackPerHead; }

__global__ void k_policy_pack(float *params, int od)
{
    const PolicyLayout L = PolicyLayout::of(od);
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= 2 * kPackPerHead) return;
    const int head = idx / kPackPerHead, rem = idx % kPackPerHead;
    const int q = rem / 256, lane = (rem % 256) / 4, e = rem % 4;
    const int j = 4 * q + e, mt = j >> 5, st = j & 31;
    const int w2 = head ? L.vf_w2 : L.pi_w2;
    params[L.total + idx] = params[w2 + (mt * 32 + (lane & 31)) * PH + 2 * st + (lane >> 5)];
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void swap_halves(float &x, float &y)
{
    // lanes 32-63 of x <-> lanes 0-31 of y (v_permlane32_swap_b32)
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}

// Both extractors + heads for the wave's 64 envs (lane = env), interleaved so the two MFMA
// chains and the two VALU streams overlap:
//   out_h = head_w . tanh(W2_h tanh(W1_h obs + b1_h) + b2_h) + head_b      (h = pi, vf)
// Layer 1 on the VALU (K = obs_dim is tiny); layer 2 as D[out][env] = W2 . H1^T on
// v_mfma_f32_32x32x2_f32 (2 x 2 tiles of 32 x 32 per head, 32 K-steps): the B operand of K-step
// s is the lanes' own h1[2s] / h1[2s+1] after one half-swap, so H1 never leaves registers; the
// head dot product is taken per lane over its 32 rows of D and completed with one more swap.
__device__ __forceinline__ void load_packed(const float *__restrict__ packed, int lane, float *A)
{
    const float4 *p4 = reinterpret_cast<const float4 *>(packed) + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const float4 v = p4[q * 64];
        A[4 * q] = v.x; A[4 * q + 1] = v.y; A[4 * q + 2] = v.z; A[4 * q + 3] = v.w;
    }
}

// Epilogue slice r of a head: lane-partial sums over rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
// and 32 + that, for both env tiles (C/D map: col = lane & 31, row as above).
__device__ __forceinline__ void head_slice(const float *__restrict__ w, int o_b2, int o_hw, const f32x16 &d00,
                                           const f32x16 &d01, const f32x16 &d10, const f32x16 &d11, int r,
                                           int hb, float &p0, float &p1)
{
    const int row0 = (r & 3) + 8 * (r >> 2) + hb, row1 = 32 + row0;
    const float w0 = w[o_hw + row0], w1 = w[o_hw + row1];
    const float c0 = w[o_b2 + row0], c1 = w[o_b2 + row1];
    p0 = fmaf(w0, tanh_fast(d00[r] + c0), p0);
    p0 = fmaf(w1, tanh_fast(d10[r] + c1), p0);
    p1 = fmaf(w0, tanh_fast(d01[r] + c0), p1);
    p1 = fmaf(w1, tanh_fast(d11[r] + c1), p1);
}

template <int OD>
__device__ __forceinline__ float layer1_unit(const float *__restrict__ w, int o_w1, int o_b1, const float *obs, int j)
{
    float a = w[o_b1 + j];
#pragma unroll
    for (int k = 0; k < OD; ++k) a = fmaf(w[o_w1 + j * OD + k], obs[k], a);
    return tanh_fast(a);
}

// Software-pipelined over the two heads so the VALU work hides under the MFMA chains:
//   phase 1: pi layer-1 (VALU)
//   phase 2: pi MFMAs      | vf layer-1 units 2s, 2s+1 (VALU)
//   phase 3: vf MFMAs      | pi epilogue slices (VALU)
//   phase 4: vf epilogue (VALU)
template <int OD>
__device__ __forceinline__ void actor_critic(const float *__restrict__ w, const float *__restrict__ packed,
                                             const PolicyLayout &L, const float *obs, int lane, float &mean,
                                             float &value)
{
    float hp[PH], hv[PH], Ap[PH], Av[PH];
    load_packed(packed, lane, Ap);                     // global loads first: in flight during layer 1
    load_packed(packed + kPackPerHead, lane, Av);
#pragma unroll
    for (int j = 0; j < PH; ++j) hp[j] = layer1_unit<OD>(w, L.pi_w1, L.pi_b1, obs, j);
    f32x16 p00 = {}, p01 = {}, p10 = {}, p11 = {}, v00 = {}, v01 = {}, v10 = {}, v11 = {};   // [mt][nt]
#pragma unroll
    for (int st = 0; st < 32; ++st) {
        float b0 = hp[2 * st], b1 = hp[2 * st + 1];
        swap_halves(b0, b1);                           // b0: env tile 0 operand, b1: env tile 1
        p00 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ap[st], b0, p00, 0, 0, 0);
        p01 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ap[st], b1, p01, 0, 0, 0);
        p10 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ap[32 + st], b0, p10, 0, 0, 0);
        p11 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ap[32 + st], b1, p11, 0, 0, 0);
        hv[2 * st] = layer1_unit<OD>(w, L.vf_w1, L.vf_b1, obs, 2 * st);
        hv[2 * st + 1] = layer1_unit<OD>(w, L.vf_w1, L.vf_b1, obs, 2 * st + 1);
    }
    const int hb = 4 * (lane >> 5);
    float pp0 = 0.0f, pp1 = 0.0f, vp0 = 0.0f, vp1 = 0.0f;
#pragma unroll
    for (int st = 0; st < 32; ++st) {
        float c0 = hv[2 * st], c1 = hv[2 * st + 1];
        swap_halves(c0, c1);
        v00 = __builtin_amdgcn_mfma_f32_32x32x2f32(Av[st], c0, v00, 0, 0, 0);
        v01 = __builtin_amdgcn_mfma_f32_32x32x2f32(Av[st], c1, v01, 0, 0, 0);
        v10 = __builtin_amdgcn_mfma_f32_32x32x2f32(Av[32 + st], c0, v10, 0, 0, 0);
        v11 = __builtin_amdgcn_mfma_f32_32x32x2f32(Av[32 + st], c1, v11, 0, 0, 0);
        if ((st & 1) == 0) head_slice(w, L.pi_b2, L.wa, p00, p01, p10, p11, st >> 1, hb, pp0, pp1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) head_slice(w, L.vf_b2, L.wv, v00, v01, v10, v11, r, hb, vp0, vp1);
    // lane l < 32 (env l): x0(l) + x0(l + 32); lane l >= 32 (env l): x1(l - 32) + x1(l)
    swap_halves(pp0, pp1);
    swap_halves(vp0, vp1);
    mean = (pp0 + pp1) + w[L.ba];
    value = (vp0 + vp1) + w[L.bv];
}

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
    constexpr PolicyLayout L = PolicyLayout::of(OD);
    __shared__ float w[kPolicyMaxParams];
    // Stage everything but the two 64x64 layers (those feed the MFMAs from the packed copy):
    // three small segments, compile-time trip counts, all loads issued before the LDS writes.
    constexpr int s1 = L.pi_w2, s2 = L.vf_w2 - L.pi_b2, s3 = L.total - L.vf_b2;
    static_assert(s1 <= 4 * 256 && s2 <= 4 * 256 && s3 <= 4 * 256, "policy staging");
    float st1[4], st2[4], st3[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = threadIdx.x + 256 * q;
        st1[q] = j < s1 ? params[j] : 0.0f;
        st2[q] = j < s2 ? params[L.pi_b2 + j] : 0.0f;
        st3[q] = j < s3 ? params[L.vf_b2 + j] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = threadIdx.x + 256 * q;
        if (j < s1) w[j] = st1[q];
        if (j < s2) w[L.pi_b2 + j] = st2[q];
        if (j < s3) w[L.vf_b2 + j] = st3[q];
    }
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = i0 < n ? i0 : n - 1;
    const int lane = threadIdx.x & 63;
    float o[OD];
#pragma unroll
    for (int k = 0; k < OD; ++k) o[k] = obs[i * OD + k];
    float mean, value;
    actor_critic<OD>(w, params + L.total, L, o, lane, mean, value);
    if (i0 >= n) return;
    if (obs_out) {
#pragma unroll
        for (int k = 0; k < OD; ++k) obs_out[i * OD + k] = o[k];
    }
    float z;
    if (noise) {
        z = noise[i];
    } else {
        Rng r;
        const uint64_t ctr = (step_base ? *step_base : 0u) + step;
        r.init(seed ^ (ctr >> 32) * 0x9E3779B97F4A7C15ull, (uint64_t)(env_offset + i), (uint32_t)ctr);
        const float u1 = ((float)(r.u32() >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
        const float u2 = (float)(r.u32() >> 8) * (1.0f / 16777216.0f);
        z = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
    }
    const float log_std = w[L.log_std];
    const float a = mean + expf(log_std) * z;
    act_out[i] = a;
    // log N(a; mean, std) with a - mean = std * z
    logp_out[i] = -0.5f * z * z - log_std - 0.918938533204672742f;
    value_out[i] = value;
    env_action[i] = fminf(fmaxf(a, act_lo), act_hi);
}

}  // namespace b747
