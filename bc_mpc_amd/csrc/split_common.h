// split_common.h -- helpers shared by the split-f16 rollout kernels (rollout_x3.hip,
// rollout_team.hip): the hi/lo f16 operand split, the tanh epilogue on element pairs and
// the cross-row lane exchanges.  Internal to libbcmpc.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"

namespace bcmpc {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

// 2 log2(e): hidden-layer biases and result scales carry this factor, so the
// epilogue's pre-activation is z = 2 log2(e) y with no extra multiply
constexpr float kTanhK = 2.8853900817779268f;

// (a, b) -> packed f16 hi = RNE(a, b) and lo = RNE(a - hi, b - hi): v_cvt_pk_f16_f32,
// two v_fma_mix_f32 (x - hi with hi read as f16, exact), v_cvt_pk_f16_f32.
__device__ __forceinline__ void split2(float a, float b, h2& hi, h2& lo) {
    hi = __builtin_convertvector((f2){a, b}, h2);
    float la, lb;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(la) : "v"(hi), "v"(a));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hi), "v"(b));
    lo = __builtin_convertvector((f2){la, lb}, h2);
}

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        h2 h, l;
        split2(v[i], v[i + 1], h, l);
        hi[i] = h[0]; hi[i + 1] = h[1];
        lo[i] = l[0]; lo[i + 1] = l[1];
    }
}

// cross-row exchanges on the VALU (gfx950 v_permlane16/32_swap) instead of LDS
// round trips: max over the lane rows r^1 / r^2, and row 1's value in row 0
__device__ __forceinline__ float max_rows16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_rows32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float add_rows(float v) {       // sum over the 4 lane rows (same in every row)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}
__device__ __forceinline__ int partner_row16(int v) {    // the value of row (r ^ 1), same column
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)r[0] == v ? (int)r[1] : (int)r[0];          // (equal values: either is right)
}

#ifndef BCMPC_FLOAD_AUX           // cache-policy bits of the weight-fragment loads (variant builds)
#define BCMPC_FLOAD_AUX 0
#endif
__device__ __forceinline__ h8 fload(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, BCMPC_FLOAD_AUX));
}

__device__ __forceinline__ h8 sread(const f4* p) { return __builtin_bit_cast(h8, *p); }
__device__ __forceinline__ void swrite(f4* p, h8 v) { *p = __builtin_bit_cast(f4, v); }

// Epilogue of one tile pair (t0, t0 + 1) for one candidate column: BiasAdd (f32, after
// undoing the operand scales; f and the biases carry the 2 log2(e) factor), tanh x 2^12 as
// 4096 - 8192 / (1 + 2^z) (fma / add / fma as packed f32 ops, bit-identical to the scalar
// form; exp / rcp per element), split.  The pair's accumulators are exactly one k-step B
// fragment of the next layer (the host's k-order permutation, capi.cpp pack_x3_layer).
#ifndef BCMPC_EPI_PK             // 0: scalar (default: rollout_pp 0.831 -> 0.822 ms, profiles/r05_epi_scalar_ab.txt), 1: packed f32 fma / add (v_pk_*_f32)
#define BCMPC_EPI_PK 0
#endif
__device__ __forceinline__ void epi_pair_tanh(const f4& a0, const f4& a1, float f, const float* __restrict__ bias,
                                              int t0, int q, h8& hi, h8& lo) {
    const f4 b0 = *reinterpret_cast<const f4*>(bias + 16 * t0 + 4 * q);
    const f4 b1 = *reinterpret_cast<const f4*>(bias + 16 * (t0 + 1) + 4 * q);
    float v[8];
    if constexpr (!BCMPC_EPI_PK) {
        // (the same IEEE operations one element at a time: bit-identical)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float z0 = fmaf(a0[r], f, b0[r]), z1 = fmaf(a1[r], f, b1[r]);
            const float r0 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z0) + 1.0f);
            const float r1 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z1) + 1.0f);
            v[r] = fmaf(-8192.0f, r0, 4096.0f);
            v[4 + r] = fmaf(-8192.0f, r1, 4096.0f);
        }
        split8(v, hi, lo);
        return;
    }
    const f2 one = {1.0f, 1.0f}, m8k = {-8192.0f, -8192.0f}, p4k = {4096.0f, 4096.0f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const f4& a = k < 2 ? a0 : a1;
        const f4& b = k < 2 ? b0 : b1;
        const int r = (k & 1) * 2;
        const f2 z = __builtin_elementwise_fma((f2){a[r], a[r + 1]}, (f2){f, f}, (f2){b[r], b[r + 1]});
        const f2 d = (f2){__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])} + one;
        const f2 rr = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
        const f2 u = __builtin_elementwise_fma(m8k, rr, p4k);
        v[2 * k] = u[0];
        v[2 * k + 1] = u[1];
    }
    split8(v, hi, lo);
}

// Single-pass "folded" epilogue (rollout_pp with FOLD): the weights carry 2 log2(e) and the accumulators
// start from the bias x 2 log2(e), so the MFMA result IS z = 2 log2(e) y; tanh(y) = 1 - 2 / (1 + 2^z) in
// f32 (exp, add, rcp, fma), rounded once to f16 -- one VALU operation per element fewer than
// epi_pair_tanh's, no power-of-two operand scales (the hidden activations are tanh in [-1, 1])
__device__ __forceinline__ h8 epi_pair_fold(const f4& a0, const f4& a1) {
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r] = fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(a0[r]) + 1.0f), 1.0f);
        v[4 + r] = fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(a1[r]) + 1.0f), 1.0f);
    }
    h8 hi;
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        const h2 h = __builtin_convertvector((f2){v[i], v[i + 1]}, h2);
        hi[i] = h[0];
        hi[i + 1] = h[1];
    }
    return hi;
}

}  // namespace bcmpc
