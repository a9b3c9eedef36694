// device_common.h -- device helpers shared by the rollout kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "kernels.h"

namespace bcmpc {

typedef float f4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- Philox ---
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0;
        const uint32_t n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Uniform action j of global candidate g at step h (oracle.device_rng_actions).
__device__ __forceinline__ double rng_action(uint64_t seed, uint64_t g, int h, int j,
                                             double lo, double hi) {
    uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)h, (uint32_t)(j >> 1)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t a = (j & 1) ? c[2] : c[0];
    const uint32_t b = (j & 1) ? c[3] : c[1];
    // NumPy legacy random_sample: ((a >> 5) * 2^26 + (b >> 6)) / 2^53 (exact in f64)
    const double u = ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
    return __dadd_rn(lo, __dmul_rn(__dsub_rn(hi, lo), u));   // low + (high-low)*u, no FMA
}

// Actions 2p and 2p + 1 of (g, h) from their ONE shared Philox block (words 0-1 and 2-3):
// bit-identical to rng_action(.., 2p, ..) and rng_action(.., 2p + 1, ..) at half the VALU.
__device__ __forceinline__ void rng_action_pair(uint64_t seed, uint64_t g, int h, int p, double lo0, double hi0,
                                                double lo1, double hi1, double& a0, double& a1) {
    uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)h, (uint32_t)p};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u0 = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) / 9007199254740992.0;
    const double u1 = ((double)(c[2] >> 5) * 67108864.0 + (double)(c[3] >> 6)) / 9007199254740992.0;
    a0 = __dadd_rn(lo0, __dmul_rn(__dsub_rn(hi0, lo0), u0));
    a1 = __dadd_rn(lo1, __dmul_rn(__dsub_rn(hi1, lo1), u1));
}

// CEM sample (DESIGN.md "CEM"): z = Irwin-Hall(12) - 6 from three Philox blocks
// (twelve 24-bit uniforms; their integer sum is exact, so z is exact in f64 and
// restatable bit-for-bit), a = clip(mu + sd*z, lo, hi) with np.clip's NaN rule.
// Counter (lo32(g), hi32(g), h, 0x40000000 | it<<8 | j<<2 | c), key = seed.
__device__ __forceinline__ double cem_normal(uint64_t seed, uint64_t g, int h, int j, int it) {
    uint32_t sum = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t x[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)h,
                         0x40000000u | ((uint32_t)it << 8) | ((uint32_t)j << 2) | (uint32_t)c};
        philox4x32_10(x, (uint32_t)seed, (uint32_t)(seed >> 32));
        sum += (x[0] >> 8) + (x[1] >> 8) + (x[2] >> 8) + (x[3] >> 8);
    }
    return __dsub_rn((double)sum * (1.0 / 16777216.0), 6.0);
}

__device__ __forceinline__ double cem_action(uint64_t seed, uint64_t g, int h, int j, int it, double mu, double sd,
                                             double lo, double hi) {
    const double a = __dadd_rn(mu, __dmul_rn(sd, cem_normal(seed, g, h, j, it)));
    return a < lo ? lo : (a > hi ? hi : a);          // np.clip = minimum(maximum(a, lo), hi)
}

// a / b correctly rounded from r = RN(1/b) (host-computed): q0 = a r is within an
// ulp, the residual a - q0 b is exact in one fma, and one Newton correction gives
// RN(a/b) (Markstein; checked exhaustively on 2e7 random pairs).  3 f64 ops instead
// of the ~10 of __ddiv_rn.  Non-finite q0 (inf / NaN operands) is returned as is.
__device__ __forceinline__ double div_rn(double a, double b, double r) {
    const double q0 = __dmul_rn(a, r);
    const double e = __fma_rn(-q0, b, a);
    const double q = __fma_rn(e, r, q0);
    return __builtin_isfinite(q0) ? q : q0;
}

// ------------------------------------------------------------ activation ---
// Branch-free tanh: odd Taylor polynomial below |x| = 0.4, else
// 1 - 2/(1 + e^{2|x|}) with v_exp_f32 / v_rcp_f32 (<= ~4 ulp vs float64 tanh,
// np.tanh itself is ~1.4 ulp; see DESIGN.md "numerics").
__device__ __forceinline__ float tanh_fast(float x) {
    const float ax = fabsf(x);
    const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);   // exp(2|x|)
    const float r = __builtin_amdgcn_rcpf(1.0f + e);
    const float big = __builtin_copysignf(fmaf(-2.0f, r, 1.0f), x);
    const float x2 = x * x;
    float p = -1382.0f / 155925.0f;
    p = fmaf(p, x2, 62.0f / 2835.0f);
    p = fmaf(p, x2, -17.0f / 315.0f);
    p = fmaf(p, x2, 2.0f / 15.0f);
    p = fmaf(p, x2, -1.0f / 3.0f);
    const float small = fmaf(x * x2, p, x);
    return ax < 0.4f ? small : big;
}

template <int ACT>
__device__ __forceinline__ float activate(float v) {
    if constexpr (ACT == BCMPC_ACT_RELU) return fmaxf(v, 0.f);
    else return tanh_fast(v);
}

// bias + activation of one output tile (tf.layers.dense: BiasAdd then act)
template <int ACT>
__device__ __forceinline__ f4 bias_act(const f4 acc, const float* __restrict__ bias, int t, int q) {
    const f4 bv = *reinterpret_cast<const f4*>(bias + 16 * t + 4 * q);
    f4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = activate<ACT>(acc[r] + bv[r]);
    return v;
}

// ---------------------------------------------------------- dense layers ---
// Standard normal from two Philox uniforms (Box-Muller, f32): the stochastic
// policy branch (DiagGaussianPd.sample = mean + std * N(0,1), ppo_bc_policy.py:85)
__device__ __forceinline__ float rng_normal(uint64_t seed, uint64_t g, int h, int j) {
    uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)h, 0x80000000u | (uint32_t)j};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)(c[0] >> 8) + 0.5f) * (1.0f / 16777216.0f);
    const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);
    return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// Raw buffer load of one 16-B weight fragment: voffset = lane*16 (VGPR),
// soffset = fragment position (SGPR).  Reads past the layer's num_records
// return 0 (hardware range check), so the prefetch may run off the end.
__device__ __forceinline__ f4 wload(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t layer_rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

// LDS carve-up of one block: [consts 2 KiB][biases L*HP + 32 floats][per-wave slabs]
__host__ __device__ constexpr int pol_param_bytes(int PL, int PHP) {
    return PHP == 0 ? 0 : (((PL * PHP + kPolParams) * 4) + 15) & ~15;
}

__host__ __device__ constexpr int param_bytes(int L, int HP) {
    return ((kConstRows * kConstCols * 8 + (L * HP + 32) * 4) + 15) & ~15;
}

struct Best {
    double c;
    int64_t i;
};

// np.argmin: a NaN beats every number (first NaN wins); else smaller value;
// equal values -> lower index.
__device__ __forceinline__ bool better(const Best& a, const Best& b) {
    const bool an = a.c != a.c, bn = b.c != b.c;
    if (an != bn) return an;
    if (!an && a.c != b.c) return a.c < b.c;
    return a.i < b.i;
}


}  // namespace bcmpc
