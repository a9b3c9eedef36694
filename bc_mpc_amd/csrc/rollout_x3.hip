// rollout_x3.hip -- "split" rollout kernel: fp32-accurate dense layers on the
// f16 matrix cores (v_mfma_f32_16x16x32_f16, 16x the f32 MFMA rate).
//
// Same contract as rollout_grp (one launch = one MPCcontroller.get_action,
// controllers.py:57-88, on this device's candidate shard: H serial
// NNDynamicsModel.predict steps, dynamics.py:106-119, with the f64
// normalise / de-normalise / residual and the cheetah cost, cost_functions.py:
// 10-30, 59-63, in registers), different arithmetic for the dense layers:
//
//   Every f32 operand x is carried as two f16 halves, x ~= hi + lo with
//   hi = f16(x), lo = f16(x - hi) (22 significant bits), and each product as
//   three MFMA passes  hi*hi + hi*lo + lo*hi  accumulated in f32 (the dropped
//   lo*lo term is 2^-22 relative).  Per dot product of n terms that is an
//   error of ~2^-21 sqrt(n) |x w|, below the ~2^-24 n |x w| by which two f32
//   summation orders (numpy sgemm vs any MFMA order) already differ.  Three
//   f16 MFMAs cost 48 cycles per 16x16x32 tile against 256 for the eight f32
//   16x16x4 MFMAs of the same tile: 5.3x the f32 matrix rate.
//
//   Range: f16 tops out at 65504, so operands are scaled by exact powers of
//   two.  Weights: per layer, host-chosen (max |W| s in [2^11, 2^12)).
//   Hidden activations: tanh only (|x| <= 1), carried as tanh * 2^12.  Layer-0
//   inputs (normalised state/action, unbounded): per candidate, the power of
//   two that puts the column's max |x| in [2^11, 2^12) -- a column scale of
//   B scales column of D by the same factor, undone exactly in the epilogue.
//
// Work split: one workgroup = NW waves = NC columns of 16 candidates.  Wave w
// owns output tiles [w*TW, (w+1)*TW) of every hidden layer for ALL NC columns,
// so each 1-KiB weight fragment it streams from L2 feeds 3*NC MFMAs (NC=4:
// 64 candidates per weight read -- the reason for the wide group: at the f16
// rate a 16-candidate group would need ~170 B/clk/CU of weights, over the
// L2's ~56).  The layer input is one LDS slab [k-step][column][hi|lo][lane];
// the accumulators of an output tile PAIR are exactly one k-step's B fragment
// of the next layer (host permutes the k order: slot 8q+i of k-step p is
// neuron 32p + 16(i>>2) + 4q + (i&3)), so the epilogue packs registers
// straight into the slab.  The output layer [h -> S] is K-split: wave w uses
// the k-steps it produced itself (no slab), partial tiles are summed in fixed
// wave order (deterministic).  Waves 0..NC-1 each own one column's f64 state,
// cost and the next step's layer-0 input.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"
#include "argmin_common.h"
#include "split_common.h"

namespace bcmpc {

// timing-only diagnostics (results wrong): no tanh / weights from a 16 KiB window /
// no owner phase (f64 state, cost, normalisation) / no MFMAs
#ifndef X3_DIAG_NOTANH
#define X3_DIAG_NOTANH 0
#endif
#ifndef X3_DIAG_SMALLW
#define X3_DIAG_SMALLW 0
#endif
#ifndef X3_DIAG_NOOWNER
#define X3_DIAG_NOOWNER 0
#endif
#ifndef X3_DIAG_NOMFMA
#define X3_DIAG_NOMFMA 0
#endif
#ifndef X3_DIAG_ONEPASS          // hidden layers: only the hi x hi MFMA pass (results inexact; timing only)
#define X3_DIAG_ONEPASS 0
#endif
#ifndef X3_DIAG_LOADS            // 1: only hi fragments are loaded (lo = hi); 2: no weight loads in mm
#define X3_DIAG_LOADS 0
#endif
#ifndef X3_DIAG_NOBAR            // no workgroup barriers inside the step loop
#define X3_DIAG_NOBAR 0
#endif
// widest hidden layer whose plain tanh split kernel takes the branch-free owner phase (v9, §6.4; at 1024 it
// measured +0.5% at cfg5, profiles/r04_bf1024_ab_rejected.jsonl)
#ifndef X3_BF_MAXHP
#define X3_BF_MAXHP 512
#endif
#ifndef X3_STAMP                 // per-phase s_memtime totals, printed by two blocks at exit
#define X3_STAMP 0
#endif
// The knobs above exist only for A/B timing builds: they are refused unless the build is a
// tools/build_variants.sh variant (which defines BCMPC_DIAG_VARIANT and writes build/variants/,
// loaded only through BCMPC_LIB); `make` / __graft_entry__.build() can never produce them.
#ifndef PP_DIAG_MFMA32          // rollout_pp's hidden layer as v_mfma_f32_32x32x16_f16 on the same operand bytes
#define PP_DIAG_MFMA32 0         // (wrong results: the timing of half the MFMA issue slots)
#endif
#if (X3_DIAG_NOTANH || X3_DIAG_SMALLW || X3_DIAG_NOOWNER || X3_DIAG_NOMFMA || X3_DIAG_ONEPASS || \
     X3_DIAG_LOADS || X3_DIAG_NOBAR || X3_STAMP || PP_DIAG_MFMA32) && !defined(BCMPC_DIAG_VARIANT)
#error "X3_DIAG_* / X3_STAMP are timing-only diagnostics (wrong results): build them with tools/build_variants.sh"
#endif
#define X3_ST(k)                                                        \
    do {                                                                \
        if constexpr (X3_STAMP) {                                       \
            const uint64_t t_ = __builtin_amdgcn_s_memtime();           \
            ph_[k] += t_ - tp_;                                         \
            tp_ = t_;                                                   \
        }                                                               \
    } while (0)

// X3_DIAG_NOBAR: 1 = every barrier off; or a bitmask 2 << id of single barriers to drop
// (id 0 Bx, 1 B1, 2 slab-free, 3 slab-ready, 4 B3, 5 B4)
#define X3_BARRIER_ID(id)                                                           \
    do {                                                                            \
        if constexpr (X3_DIAG_NOBAR != 1 && !((X3_DIAG_NOBAR >> ((id) + 1)) & 1)) __syncthreads(); \
    } while (0)
#define X3_BARRIER() X3_BARRIER_ID(-1)

// tanh(y) * 2^12 from z = 2 log2(e) y: 4096 - 8192 / (1 + e), e = 2^z = e^{2y} (4 VALU
// ops, two of them transcendental; no sign handling: e = inf -> 4096, e = 0 -> -4096).
// Absolute error ~1e-7 (x 4096) near 0, a few ulp elsewhere; NaN propagates.
__device__ __forceinline__ float tanh_x4096(float z) {
    if constexpr (X3_DIAG_NOTANH) return z * 1024.0f;
    const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z) + 1.0f);
    return fmaf(-8192.0f, r, 4096.0f);
}

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
    if constexpr (X3_DIAG_NOMFMA) return c + (f4){(float)a[0], (float)b[0], 0.f, 0.f};
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// slab index of (k-step p, column c, part) in f4 units of one lane (F1: the hi part only)
template <int NC, bool F1 = false>
__device__ __forceinline__ int sidx(int p, int c, int part, int lane) {
    return ((p * NC + c) * (F1 ? 1 : 2) + part) * 64 + lane;
}

// One operand unit: acc[g*G + j][c] += W[tile g*G + j] * X[c] for j < G (the G
// tiles' A fragments, hi / lo, in registers) and the k-step's B fragments (bh/bl,
// all NC columns, read by the caller).
// F1 (BCMPC_PREC_F16): the hi x hi pass only.
template <int TW, int NC, int G, bool F1 = false>
__device__ __forceinline__ void unit_x3(const h8 (&ah)[G], const h8 (&al)[G], const h8 (&bh)[NC],
                                        const h8 (&bl)[NC], int g, f4 (&acc)[TW][NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int j = 0; j < G; ++j) acc[g * G + j][c] = mfma16(ah[j], bh[c], acc[g * G + j][c]);
        if constexpr (X3_DIAG_ONEPASS || F1) continue;  // (ONEPASS: timing only)
#pragma unroll
        for (int j = 0; j < G; ++j) acc[g * G + j][c] = mfma16(ah[j], bl[c], acc[g * G + j][c]);
#pragma unroll
        for (int j = 0; j < G; ++j) acc[g * G + j][c] = mfma16(al[j], bh[c], acc[g * G + j][c]);
    }
}

// NG == 1 unit with the B fragments streamed per column (one column of lookahead,
// 16 VGPRs instead of 8*NC): for register-tight layouts (X3_BSTREAM)
template <int TW, int NC, int G>
__device__ __forceinline__ void unit_x3s(const h8 (&ah)[G], const h8 (&al)[G], const f4* slab, int p, int lane,
                                         f4 (&acc)[TW][NC]) {
    h8 bh = sread(slab + sidx<NC>(p, 0, 0, lane));
    h8 bl = sread(slab + sidx<NC>(p, 0, 1, lane));
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        h8 nbh = bh, nbl = bl;
        if (c + 1 < NC) {
            nbh = sread(slab + sidx<NC>(p, c + 1, 0, lane));
            nbl = sread(slab + sidx<NC>(p, c + 1, 1, lane));
        }
#pragma unroll
        for (int j = 0; j < G; ++j) acc[j][c] = mfma16(ah[j], bh, acc[j][c]);
#pragma unroll
        for (int j = 0; j < G; ++j) acc[j][c] = mfma16(ah[j], bl, acc[j][c]);
#pragma unroll
        for (int j = 0; j < G; ++j) acc[j][c] = mfma16(al[j], bh, acc[j][c]);
        bh = nbh;
        bl = nbl;
    }
}

#ifndef X3_BSTREAM
#define X3_BSTREAM 0
#endif
// (F1: the hi parts only; the lo operands are never read)
template <int NC, bool F1 = false>
__device__ __forceinline__ void bread_x3(const f4* slab, int p, int lane, h8 (&bh)[NC], h8 (&bl)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bh[c] = sread(slab + sidx<NC, F1>(p, c, 0, lane));
        bl[c] = F1 ? bh[c] : sread(slab + sidx<NC, F1>(p, c, 1, lane));
    }
}

template <int G, bool F1 = false>
__device__ __forceinline__ void aload_x3(__amdgpu_buffer_rsrc_t rs, int voff, int base, h8 (&ah)[G], h8 (&al)[G],
                                         bool diag = false) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int o = X3_DIAG_SMALLW ? ((base + j * 2048) & 16383) : base + j * 2048;
        if (diag && X3_DIAG_LOADS == 2) {
            ah[j] = ah[j] + (h8)(_Float16)1.0f;
            al[j] = al[j] + (h8)(_Float16)1.0f;
            continue;
        }
        ah[j] = fload(rs, voff, o);
        if constexpr (F1) al[j] = ah[j];
        else al[j] = (diag && X3_DIAG_LOADS == 1) ? ah[j] + (h8)(_Float16)1.0f : fload(rs, voff, o + 1024);
    }
}

// acc[j][c] += sum over the P k-steps of W[tile j] * X[c]: this wave's contiguous
// weight slice streamed from L2 in units of G tiles x one k-step (NG = TW/G units
// per k-step) through two register sets (ping-pong: unit u+1's loads are in
// flight while unit u's MFMAs run; set 0 arrives holding unit 0, loaded by the
// caller before its epilogue and clobbered here); the layer input from the slab,
// each k-step's B fragments read once at its first unit.
//
// OWN: the k-steps run in the order k0 = w*PW, w*PW+1, ... (mod P), and the first PW
// -- the ones this wave produced and already wrote to the slab itself -- need no
// other wave: bar() (the "layer input complete" barrier) runs after their MFMAs are
// issued, overlapping them with the slower waves' epilogues.  (A wave reads its own
// LDS writes in program order: no barrier.)
//
// NRES (the resident units, X3_RES): the wave's own NOWN units come from registers loaded once per launch
// (resh / resl) instead of the L2 stream; s0 then arrives holding unit NOWN.
template <int TW, int NC, int P, int G, bool OWN = false, int PW = 1, bool F1 = false, int NRES = 0,
          typename Bar = void (*)()>
__device__ __forceinline__ void mm_x3(__amdgpu_buffer_rsrc_t rs, int wbase, const f4* slab, f4 (&acc)[TW][NC],
                                      int lane, h8 (&s0h)[G], h8 (&s0l)[G], int k0 = 0, Bar bar = nullptr,
                                      const h8 (*resh)[G] = nullptr, const h8 (*resl)[G] = nullptr) {
    constexpr int NG = TW / G;
    static_assert(NG * G == TW && (NG == 1 || NG == 2), "one or two units per k-step");
    static_assert((P * NG) % 2 == 0, "ping-pong over unit pairs");
    constexpr int NU = P * NG;
    // units fed from registers (whole ping-pong pairs only; otherwise the rotated order from the slab)
    constexpr int NOWN = (OWN && (PW * NG) % 2 == 0) ? PW * NG : 0;
    static_assert(NU - NOWN >= 2, "a slab pair remains");
    constexpr int STEPB = TW * 2048;
    const int voff = lane * 16;
    auto kstep = [&](int u) {                           // k-step of unit u
        const int p = u / NG + k0;
        return p >= P ? p - P : p;
    };
    auto uoff = [&](int u) { return wbase + kstep(u) * STEPB + (u % NG) * G * 2048; };
    // unit u (even) is (k-step u/NG, group 0); unit u+1 is group 1 of the same
    // k-step (NG = 2) or the next k-step (NG = 1)
    constexpr int G1 = NG == 2 ? 1 : 0;
    h8 s1h[G], s1l[G], bh[NC], bl[NC];
    static_assert(NRES == 0 || (OWN && NRES == NOWN && NG == 1 && !F1), "resident units: the own k-steps");
    if constexpr (NRES > 0) {
#pragma unroll
        for (int u = 0; u < NRES; ++u) {
            bread_x3<NC, F1>(slab, kstep(u), lane, bh, bl);
            unit_x3<TW, NC, G, F1>(resh[u], resl[u], bh, bl, 0, acc);
        }
        bar();
    } else if constexpr (OWN) {
#pragma unroll
        for (int u = 0; u < NOWN; u += 2) {
            aload_x3<G, F1>(rs, voff, uoff(u + 1), s1h, s1l, true);
            __builtin_amdgcn_sched_barrier(0);
            bread_x3<NC, F1>(slab, kstep(u), lane, bh, bl);
            unit_x3<TW, NC, G, F1>(s0h, s0l, bh, bl, 0, acc);
            aload_x3<G, F1>(rs, voff, uoff(u + 2), s0h, s0l, true);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (NG == 1) bread_x3<NC, F1>(slab, kstep(u + 1), lane, bh, bl);
            unit_x3<TW, NC, G, F1>(s1h, s1l, bh, bl, G1, acc);
        }
        bar();
    }
    // (the last pair is peeled so that every load in the loop is unconditional: a
    // conditional load would make the compiler drain vmcnt to 0 at the merge)
    if constexpr (NG == 1 && X3_BSTREAM && !OWN) {
        for (int u = 0; u < NU - 2; u += 2) {
            aload_x3<G, F1>(rs, voff, uoff(u + 1), s1h, s1l, true);
            __builtin_amdgcn_sched_barrier(0);      // keep the loads ahead of the MFMAs they overlap
            unit_x3s<TW, NC, G>(s0h, s0l, slab, u, lane, acc);
            aload_x3<G, F1>(rs, voff, uoff(u + 2), s0h, s0l, true);
            __builtin_amdgcn_sched_barrier(0);
            unit_x3s<TW, NC, G>(s1h, s1l, slab, u + 1, lane, acc);
        }
        aload_x3<G, F1>(rs, voff, uoff(NU - 1), s1h, s1l, true);
        __builtin_amdgcn_sched_barrier(0);
        unit_x3s<TW, NC, G>(s0h, s0l, slab, NU - 2, lane, acc);
        unit_x3s<TW, NC, G>(s1h, s1l, slab, NU - 1, lane, acc);
        (void)bh; (void)bl;
        return;
    }
    for (int u = NOWN; u < NU - 2; u += 2) {
        aload_x3<G, F1>(rs, voff, uoff(u + 1), s1h, s1l, true);
        __builtin_amdgcn_sched_barrier(0);          // keep the loads ahead of the MFMAs they overlap
        bread_x3<NC, F1>(slab, kstep(u), lane, bh, bl);
        unit_x3<TW, NC, G, F1>(s0h, s0l, bh, bl, 0, acc);
        aload_x3<G, F1>(rs, voff, uoff(u + 2), s0h, s0l, true);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (NG == 1) bread_x3<NC, F1>(slab, kstep(u + 1), lane, bh, bl);
        unit_x3<TW, NC, G, F1>(s1h, s1l, bh, bl, G1, acc);
    }
    aload_x3<G, F1>(rs, voff, uoff(NU - 1), s1h, s1l, true);
    __builtin_amdgcn_sched_barrier(0);
    bread_x3<NC, F1>(slab, kstep(NU - 2), lane, bh, bl);
    unit_x3<TW, NC, G, F1>(s0h, s0l, bh, bl, 0, acc);
    if constexpr (NG == 1) bread_x3<NC, F1>(slab, kstep(NU - 1), lane, bh, bl);
    unit_x3<TW, NC, G, F1>(s1h, s1l, bh, bl, G1, acc);
}

// Epilogue of one tile pair (k-step) for one column: BiasAdd (f32, after undoing
// the operand scales; f and the LDS biases carry the 2 log2(e) factor), tanh,
// x 2^12, split.
__device__ __forceinline__ void epi_pair(const f4& a0, const f4& a1, float f, const float* __restrict__ bias,
                                         int t0, int q, h8& hi, h8& lo) {
    if constexpr (X3_DIAG_NOTANH) {
        const f4 b0 = *reinterpret_cast<const f4*>(bias + 16 * t0 + 4 * q);
        const f4 b1 = *reinterpret_cast<const f4*>(bias + 16 * (t0 + 1) + 4 * q);
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = tanh_x4096(fmaf(a0[r], f, b0[r]));
            v[4 + r] = tanh_x4096(fmaf(a1[r], f, b1[r]));
        }
        split8(v, hi, lo);
    } else {
        epi_pair_tanh(a0, a1, f, bias, t0, q, hi, lo);
    }
}

// relu / LayerNorm epilogue (AK != 0; bit 0 relu, bit 1 LayerNorm) of this wave's TW tiles x NC
// columns, in place: BiasAdd + activation in f32, then ONE exchange of per-column statistics
// across the NW waves (X3 barrier 6), then the split.
//   LN (dynamics.py:68-69, tf.contrib.layers.layer_norm): each wave's (mean, M2) over its valid
//     rows, merged in wave order (Chan et al.), var = M2 / hidden, the nn.batch_normalization form
//     x * inv + (beta - mean * inv), inv = rsqrt(var + eps) * gamma; output x hsc (host power of
//     two from |y| <= sqrt(hidden) max|gamma| + max|beta|).  A tanh net's activations are tanh x 2^12
//     here, so its eps is 1e-12 x 2^24 (the normalised output is the same).
//   relu without LN: the column max sets the column's power of two (max -> [2^11, 2^12)); the
//     next layer undoes it through fcol (its epilogue factor, or the output factor).
template <int AK, int TW, int NC, int NW>
__device__ __forceinline__ void epi_colx(f4 (&acc)[TW][NC], const float (&f)[NC], const float* __restrict__ bias,
                                         const float* __restrict__ lg, const float* __restrict__ lb, float hsc,
                                         int hidden, float* xch, int w, int lane, h8 (&xh)[TW / 2][NC],
                                         h8 (&xl)[TW / 2][NC], float (&fcol)[NC]) {
    constexpr bool RELU = (AK & 1) != 0, LNK = (AK & 2) != 0;
    const int q = lane >> 4, m = lane & 15;
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        const f4 b = *reinterpret_cast<const f4*>(bias + 16 * (w * TW + j) + 4 * q);
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float z = fmaf(acc[j][c][r], f[c], b[r]);
                acc[j][c][r] = RELU ? fmaxf(z, 0.f) : tanh_x4096(z);     // pad rows: exactly 0
            }
    }
    const int nwr = min(max(hidden - 16 * TW * w, 0), 16 * TW);        // this wave's valid rows
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        float s0 = 0.f, s1 = 0.f;
        if constexpr (LNK) {
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) s0 += acc[j][c][r];
            s0 = nwr > 0 ? add_rows(s0) / (float)nwr : 0.f;
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float d = acc[j][c][r] - s0;
                    s1 += (16 * (w * TW + j) + 4 * q + r < hidden) ? d * d : 0.f;
                }
            s1 = add_rows(s1);
        } else {
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) s0 = fmaxf(s0, acc[j][c][r]);
            s0 = max_rows32(max_rows16(s0));
        }
        if (q == 0) *reinterpret_cast<f2*>(xch + ((w * NC + c) * 16 + m) * 2) = (f2){s0, s1};
    }
    X3_BARRIER_ID(6);                                   // every wave's column statistics published
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if constexpr (LNK) {
            float mean = 0.f, m2 = 0.f;
            if (hidden == 16 * TW * NW) {
                // no padded rows: the merge weights nb / nn, n nb / nn below folded at compile time
                // (bit-identical; 2 NW dependent divisions per column off the critical path)
#pragma unroll
                for (int g = 0; g < NW; ++g) {
                    const float nb = (float)(16 * TW), n = (float)(16 * TW * g), nn = n + nb;
                    const f2 st = *reinterpret_cast<const f2*>(xch + ((g * NC + c) * 16 + m) * 2);
                    const float d = st[0] - mean;
                    mean = mean + d * (nb / nn);
                    m2 = m2 + st[1] + d * d * (n * nb / nn);
                }
            } else {
                float n = 0.f;
#pragma unroll
                for (int g = 0; g < NW; ++g) {
                    const float nb = (float)min(max(hidden - 16 * TW * g, 0), 16 * TW);
                    if (nb > 0.f) {
                        const f2 st = *reinterpret_cast<const f2*>(xch + ((g * NC + c) * 16 + m) * 2);
                        const float nn = n + nb, d = st[0] - mean;
                        mean = mean + d * (nb / nn);
                        m2 = m2 + st[1] + d * d * (n * nb / nn);
                        n = nn;
                    }
                }
            }
            const float eps = RELU ? 1e-12f : 1e-12f * 16777216.0f;
            // (the same quotient; a power-of-two width folds it to an exact multiply)
            const float var = hidden == 16 * TW * NW ? m2 / (float)(16 * TW * NW) : m2 / (float)hidden;
            const float rs = 1.0f / sqrtf(var + eps);
#pragma unroll
            for (int j = 0; j < TW; ++j) {
                const f4 gv = *reinterpret_cast<const f4*>(lg + 16 * (w * TW + j) + 4 * q);
                const f4 bv = *reinterpret_cast<const f4*>(lb + 16 * (w * TW + j) + 4 * q);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float inv = rs * gv[r];
                    acc[j][c][r] = (acc[j][c][r] * inv + (bv[r] - mean * inv)) * hsc;
                }
            }
        } else {
            float mx = 0.f;
#pragma unroll
            for (int g = 0; g < NW; ++g) mx = fmaxf(mx, xch[((g * NC + c) * 16 + m) * 2]);
            int e = 0;
            (void)frexpf(mx, &e);
            int sh = 12 - e;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
            const float sc = ldexpf(1.0f, sh);
            fcol[c] = ldexpf(1.0f, -sh);
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[j][c][r] *= sc;
        }
    }
#pragma unroll
    for (int pp = 0; pp < TW / 2; ++pp)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const float v[8] = {acc[2 * pp][c][0], acc[2 * pp][c][1], acc[2 * pp][c][2], acc[2 * pp][c][3],
                                acc[2 * pp + 1][c][0], acc[2 * pp + 1][c][1], acc[2 * pp + 1][c][2],
                                acc[2 * pp + 1][c][3]};
            split8(v, xh[pp][c], xl[pp][c]);
        }
}

#ifndef X3_NW256                // waves per workgroup at hidden 256 (4, or 8: one tile pair per wave)
#define X3_NW256 4
#endif
#ifndef X3_NW512                // waves per workgroup at hidden 512 (8: one 64-candidate group per CU;
#define X3_NW512 8               // 4: two 32-candidate groups per CU, out of phase)
#endif
#ifndef X3_NW1024               // waves per workgroup at hidden 1024 (8, or 16: four per SIMD)
#define X3_NW1024 8
#endif
#ifndef X3_ONLY_NC
#define X3_ONLY_NC 4
#endif
#ifndef X3_PRIO                  // 1: s_setprio 1 for the second-dispatched half of the waves
#define X3_PRIO 0
#endif
#ifndef X3_STAGGER               // diagnostic: odd workgroups start X3_STAGGER x 8k cycles late
#define X3_STAGGER 0
#endif
// tiles per streamed operand unit: a whole k-step up to 4 tiles per wave, else half
#ifndef X3_GMAX
#define X3_GMAX 4
#endif
__host__ __device__ constexpr int x3_group(int TW) { return TW <= X3_GMAX ? TW : TW / 2; }

#ifndef X3_OWN                   // hidden layers start with the k-steps the wave produced itself
#define X3_OWN 1
#endif
#ifndef X3_NCH
#define X3_NCH 4                 // steps of layer-0 action inputs staged in LDS per fill
#endif
#ifndef X3_RES                   // NC = 1 at hidden 512 (cfg2's layout): the wave's own two k-steps of the
#define X3_RES 1                 // hidden layer resident in registers for the whole launch (64 VGPRs)
#endif

// waves per SIMD the register allocator must allow: two whenever two workgroups
// (or two waves of one) should share a SIMD
__host__ __device__ constexpr int x3_waves_per_eu(int HP, int NC, int NW) {
    return NW >= 16 ? 4 : (NW >= 8 || HP <= 512) ? 2 : 1;
}

// LDS carve-up: consts | biases (L*HP + 32) | policy biases + params (PL*PHP + kPolParams) |
// column factors NC*16 | column max [2][NC*16] | penalty counts [2][NC*16] | action inputs
// NCH*16NC*A (16-B aligned; none with a policy) | layer-0 slab NC*2 KiB | slab P*NC*2 KiB (F1: the hi
// halves only, NC*1 KiB | P*NC*1 KiB)
// steps of action inputs staged per fill: X3_NCH, but 2 for the single-pass 4-wave groups (two of them
// share a CU's 160 KiB)
__host__ __device__ constexpr int x3_nch(int NW, bool F1) { return (F1 && NW <= 4) ? 2 : X3_NCH; }
// slab: 1-KiB fragments per candidate column (the layer input's P k-steps x hi | lo; at least the
// output-layer partials' 2 NW)
__host__ __device__ constexpr int x3_slab_frags(int HP, int NW, bool F1) {
    return (HP / 32) * (F1 ? 1 : 2) > 2 * NW ? (HP / 32) * (F1 ? 1 : 2) : 2 * NW;
}
__host__ __device__ constexpr int x3_xa_bytes(int NC, int A, int nch = X3_NCH) { return (nch * 16 * NC * A * 4 + 15) & ~15; }
// | AK != 0: column exchange [NW][NC*16][2] | LN gamma [L][HP], beta [L][HP]
__host__ __device__ constexpr int x3_lds_bytes_rt(int HP, int NC, int L, int A, int PL = 0, int PHP = 0, int AK = 0,
                                                  int NW = 8, bool F1 = false) {
    return param_bytes(L, HP) + pol_param_bytes(PL, PHP) + NC * 16 * 4 * 5 +
           (PHP > 0 ? 0 : x3_xa_bytes(NC, A, x3_nch(NW, F1))) + NC * (F1 ? 1024 : 2048) +
           x3_slab_frags(HP, NW, F1) * NC * 1024 + (AK != 0 ? NW * NC * 16 * 8 : 0) + ((AK & 2) ? 2 * L * HP * 4 : 0);
}

template <int HP, int NC, int NW, int PHP, bool RW, int AK, bool F1 = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(x3_waves_per_eu(HP, NC, NW), 8)))
void rollout_x3(const RolloutArgs a) {
    // AK: hidden activation kind, 0 tanh (activations tanh x 2^12: static scales); bit 0 relu,
    // bit 1 LayerNorm (epi_colx: one column exchange per hidden layer)
    constexpr bool RELU = (AK & 1) != 0, LNK = (AK & 2) != 0, DYN = RELU && !LNK;
    constexpr float kAct = RELU ? 1.0f : kTanhK;        // folded into the epilogue factors / biases
    static_assert(AK == 0 || (PHP == 0 && !RW), "relu / LayerNorm: the plain delta net only");
    // F1 (BCMPC_PREC_F16, BASELINE cfg3's "bf16 MFMA GEMM + fp32 cost accumulate" with f16's 11-bit
    // significand): every operand is its hi part alone, one MFMA pass, no lo loads / slab writes
    static_assert(!F1 || (PHP == 0 && !RW && AK == 0), "single-pass f16: the plain tanh delta net only");
    constexpr int T = HP / 16;          // hidden tiles
    constexpr int P = T / 2;            // hidden k-steps (32 wide)
    constexpr int TW = T / NW;          // output tiles per wave
    constexpr int PW = TW / 2;          // k-steps produced per wave
    constexpr int CB = 16 * NC;         // candidates per block
    constexpr int G = x3_group(TW);     // tiles per streamed operand unit
    static_assert(TW % 2 == 0 && TW * NW == T, "each wave must own whole tile pairs");
    static_assert(NC <= NW, "one owner wave per column");
    constexpr int NPT = F1 ? 1 : 2;     // slab parts per B fragment: hi | lo (F1: hi)
    constexpr int NCH = x3_nch(NW, F1); // steps of action inputs staged per fill
    // slab fragments per column: the layer input, or the output-layer partials [NW][2 tiles] that reuse it
    constexpr int SLABF = x3_slab_frags(HP, NW, F1);
    static_assert(SLABF >= P * NPT && SLABF >= 2 * NW, "the output-layer partials reuse the slab");
    // fused policy (MPCcontrollerPolicyNet): one policy tile per wave, split ownership
    constexpr int PPn = PHP / 32;                       // policy hidden k-steps
    static_assert(PHP == 0 || (PHP / 16 == NW && 2 * NC <= NW && PPn + NW / 2 <= P),
                  "policy: one hidden tile per wave, two state waves per column, partials in the slab");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;
    const int m = lane & 15;
    // State ownership.  SO (2*NC <= NW): two waves per column, wave w < 2*NC owns half
    // hv0 = w / NC of column w % NC (dims 16*hv0 + 4q + r), which halves the serial f64
    // phase; otherwise waves w < NC own both halves of column w.
    constexpr bool SO = 2 * NC <= NW;
    constexpr int NHV = SO ? 1 : 2;                     // halves per state wave
    const bool owner = w < (SO ? 2 * NC : NC);
    const int cw = owner ? w % NC : 0;                  // the owner's column
    const int hv0 = SO ? (owner ? w / NC : 0) : 0;      // the owner's first half
    const int64_t cand0 = (int64_t)blockIdx.x * CB;
    const int64_t cand = cand0 + 16 * cw + m;
    const bool valid = owner && cand < a.K;
    const int S = a.S, A = a.A, L = a.L;
    // RW (NNDynamicsRewardModel, dynamics.py:150-177): weights [trunk, delta head, delta out,
    // reward head, reward out], biases [trunk, delta head, reward head | out]
    const int LB = RW ? 3 : L;                          // hidden bias rows
    const int LO = RW ? 2 : L;                          // the (delta) output layer

    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < LB; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i] * kAct;
    float* const Bout = Bl + LB * HP;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bout[i] = a.b[LB][i];
    float* const Pb = Bout + 32;                        // policy: [PL][PHP] hidden biases (x 2 log2 e), params
    const int PL = a.pL;
    if constexpr (PHP > 0) {
        for (int l = 0; l < PL; ++l)
            for (int i = threadIdx.x; i < PHP; i += blockDim.x) Pb[l * PHP + i] = a.pb[l][i] * kTanhK;
        for (int i = threadIdx.x; i < kPolParams; i += blockDim.x) Pb[PL * PHP + i] = a.pparams[i];
    }
    float* colf = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + param_bytes(LB, HP) +
                                           pol_param_bytes(PHP > 0 ? PL : 0, PHP));
    float* colmax = colf + NC * 16;                     // [half][NC*16]: per-half column max (split owners)
    int* penbuf = reinterpret_cast<int*>(colmax + 2 * NC * 16);   // [step & 1][NC*16] penalty counts
    float* xa = reinterpret_cast<float*>(penbuf + 2 * NC * 16);   // [NCH][CB][A] normalised action inputs
    f4* slab0 = reinterpret_cast<f4*>(reinterpret_cast<char*>(xa) + (PHP > 0 ? 0 : x3_xa_bytes(NC, A, NCH)));
    f4* slab = slab0 + NC * NPT * 64;
    float* const xch = reinterpret_cast<float*>(slab + SLABF * NC * 64);   // AK: column exchange
    float* const lnp = xch + NW * NC * 16 * 2;                            // LN: gamma [L][HP], beta [L][HP]
    if constexpr (LNK)
        for (int l = 0; l < L; ++l)
            for (int i = threadIdx.x; i < HP; i += blockDim.x) {
                lnp[l * HP + i] = a.lng[l][i];
                lnp[(L + l) * HP + i] = a.lnb[l][i];
            }
    float fcol[NC];                                     // DYN: 2^-(column scale) of the last hidden layer
#pragma unroll
    for (int c = 0; c < NC; ++c) fcol[c] = 1.0f;
    __syncthreads();

    double s[NHV][4];                                   // dims 16*(hv0+k) + 4q + r
#pragma unroll
    for (int k = 0; k < NHV; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int d = 16 * (hv0 + k) + 4 * q + r;
            s[k][r] = (valid && d < S) ? (a.state_inline ? a.state_v[d] : a.state[cand * a.state_stride + d]) : 0.0;
        }
    if (a.traj && valid) {
#pragma unroll
        for (int k = 0; k < NHV; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * (hv0 + k) + 4 * q + r;
                if (d < S) a.traj[cand * S + d] = s[k][r];
            }
    }
    double cost = 0.0;                                  // trajectory_cost = 0 (cost_functions.py:60)
    double prog_prev = 0.0;                             // SO: the half-1 owner's progress term, one step late
    // action j of candidate c at step h: the caller's [H,K,A] array (np.random.uniform,
    // controllers.py:53), Philox, or the CEM sampler
    auto act_value = [&](int h, int64_t c, int j) __attribute__((always_inline)) -> double {
        const uint64_t g = (uint64_t)(a.cand_offset + c);
        if (a.cem_mu)
            return cem_action(a.seed, g, h, j, a.cem_iter, a.cem_mu[h * A + j], a.cem_sigma[h * A + j],
                              C[6 * 32 + j], C[7 * 32 + j]);
        return a.actions ? a.actions[((int64_t)h * a.K + c) * A + j]
                         : rng_action(a.seed, g, h, j, C[6 * 32 + j], C[7 * 32 + j]);
    };
    // stage NCH steps' action inputs from step h0: f64 normalise (dynamics.py:110),
    // cast to f32 (TF feed); threads [0, nt) of the block
    auto fill_actions = [&](int h0, int nt) __attribute__((always_inline)) {
        const int nhs = (a.H - h0 < NCH) ? a.H - h0 : NCH;
        if (!a.cem_mu && !a.actions) {
            // device Philox: one block feeds actions 2p and 2p + 1 (every thread's share of the
            // chunk's blocks halves: this fill runs on every wave, on the step's critical path)
            const int AP = (A + 1) >> 1, per = CB * AP;
            for (int i = threadIdx.x; i < nhs * per; i += nt) {
                const int hh = i / per, rem = i - hh * per, kl = rem / AP, p = rem - kl * AP;
                const int j0 = 2 * p, j1 = min(2 * p + 1, A - 1);
                float x0 = 0.f, x1 = 0.f;
                if (cand0 + kl < a.K) {
                    double v0, v1;
                    rng_action_pair(a.seed, (uint64_t)(a.cand_offset + cand0 + kl), h0 + hh, p, C[6 * 32 + j0],
                                    C[7 * 32 + j0], C[6 * 32 + j1], C[7 * 32 + j1], v0, v1);
                    x0 = (float)div_rn(__dsub_rn(v0, C[2 * 32 + j0]), C[3 * 32 + j0], C[9 * 32 + j0]);
                    x1 = (float)div_rn(__dsub_rn(v1, C[2 * 32 + j1]), C[3 * 32 + j1], C[9 * 32 + j1]);
                }
                float* const dst = xa + (hh * CB + kl) * A;
                dst[j0] = x0;
                if (2 * p + 1 < A) dst[j1] = x1;
            }
            return;
        }
        const int per = CB * A;
        for (int i = threadIdx.x; i < nhs * per; i += nt) {
            const int hh = i / per, rem = i - hh * per, kl = rem / A, j = rem - kl * A;
            float xv = 0.f;
            if (cand0 + kl < a.K)
                xv = (float)div_rn(__dsub_rn(act_value(h0 + hh, cand0 + kl, j), C[2 * 32 + j]), C[3 * 32 + j],
                                   C[9 * 32 + j]);
            xa[(hh * CB + kl) * A + j] = xv;
        }
    };
    if constexpr (PHP == 0) fill_actions(0, 64 * NW);
    __syncthreads();
    const int voff = lane * 16;
    const int kown = X3_OWN ? w * PW : 0;               // first k-step of this wave's hidden-layer sweep
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(a.w[0], a.wbytes[0]);
    const __amdgpu_buffer_rsrc_t rso = layer_rsrc(a.w[LO], a.wbytes[LO]);
    const float fo = a.winv[LO];
    // An opaque zero, refreshed every step, added to the step loop's weight offsets and LDS table bases:
    // the weights, biases and constants are the same every step, and without it the compiler hoists
    // their loop-invariant loads out of the step loop and keeps them in registers for the whole launch
    // (round 4: 76 spilled registers at the 4-wave single-pass layout).
    int wz = 0;
    const double* Cv = C;
    const float* Blv = Bl;

    // Operand sets in flight ahead of their MFMAs (issued before the preceding VALU phase):
    //   a0h/a0l : layer-0 fragments of the NEXT step (issued after the output MFMAs)
    //   uh/ul   : unit 0 of the next hidden layer, issued before each epilogue
    //   oh/ol   : the output layer's first OP k-step pairs (slot 2*(pp % OP) + v = k-step
    //             w*PW+pp, tile v), issued before the last epilogue; the rest stream in
#ifndef X3_OP
#define X3_OP 1             // output-layer k-step pairs prefetched before the last epilogue (2: the second pair in flight too -- measured equal, and it demotes the slots to scratch)
#endif
    constexpr int OP = PW < X3_OP ? PW : X3_OP;
    h8 a0h[TW], a0l[TW], uh[G], ul[G], oh[2 * OP], ol[2 * OP];
    if constexpr (PHP == 0) aload_x3<TW, F1>(rs0, voff, w * TW * 2048, a0h, a0l);
    // (the slot is a compile-time constant at every call: a runtime index into oh/ol would
    // demote the arrays to scratch memory)
    auto load_out = [&](int pp, auto SLOTc) __attribute__((always_inline)) {
        constexpr int slot = decltype(SLOTc)::value;
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int o = wz + (((w * PW + pp) * 2 + v) * 2) * 1024;
            oh[2 * slot + v] = fload(rso, voff, o);
            ol[2 * slot + v] = F1 ? oh[2 * slot + v] : fload(rso, voff, o + 1024);
        }
    };
    // Resident units (X3_RES; the one-column layout at hidden 512, cfg2's): a workgroup of 16 candidates
    // streams the whole split net from L2 every step, and that per-CU stream binds it; the
    // registers the layout leaves free hold the wave's own two k-steps of the hidden layer (1/8 of its
    // fragments) for the whole launch, so the stream carries 7/8 of it
    constexpr int NRES = (X3_RES && X3_OWN && NC == 1 && HP == 512 && PHP == 0 && !RW && AK == 0 && !F1 &&
                          G == TW && PW % 2 == 0) ? PW : 0;
    h8 rsh[NRES > 0 ? NRES : 1][G], rsl[NRES > 0 ? NRES : 1][G];
    if constexpr (NRES > 0)
        if (L >= 2)
#pragma unroll
            for (int u = 0; u < NRES; ++u)
                aload_x3<G>(layer_rsrc(a.w[1], a.wbytes[1]), voff, w * P * TW * 2048 + ((kown + u) % P) * TW * 2048,
                            rsh[u], rsl[u]);
    auto load_next = [&](int l_next) __attribute__((always_inline)) {
        if (l_next < L) {
            // (layer 1 with resident units: the stream starts at the first k-step past them)
            const int k1 = (NRES > 0 && l_next == 1) ? (kown + NRES) % P : kown;
            aload_x3<G, F1>(layer_rsrc(a.w[l_next], a.wbytes[l_next]), voff, wz + w * P * TW * 2048 + k1 * TW * 2048, uh, ul);
        } else {
            load_out(0, std::integral_constant<int, 0>{});
            if constexpr (OP > 1) load_out(1, std::integral_constant<int, OP - 1>{});
        }
    };

    // ---- fused policy (MlpPolicy.act, ppo_bc_policy.py:54-88; mixing controllers.py:196-206) ----
    // Same split-f16 arithmetic: obz = clip((f32(ob) - mean) / std, -5, 5) carried x 2^11, tanh
    // hidden layers x 2^12.  Wave w owns policy tile w of every hidden layer (its 16 neurons are
    // half w&1 of k-step w/2 of the next layer's input); the output layer (one 16-row tile,
    // action j at row S-16+j) is K-split over the waves, partials summed in fixed order by the
    // half-1 owners, whose lanes hold exactly the action dims.
#ifndef X3_POLDIAG                // timing only (results wrong): 1 no hidden->hidden layer, 2 no explore
#define X3_POLDIAG 0              // loads, 3 no partial sum / mixing, 4 no obz division
#endif
    auto policy_step = [&](int h, double (&pact)[4]) __attribute__((always_inline)) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        const float* pm = Pb + PL * PHP;                // [obmean 32][obstd 32][logstd 16][out bias 16]
        const bool actor = owner && hv0 == 1;
        // every layer's fragments of the first two layers and the output layer are requested
        // here, so one L2 latency (under the owners' obz and the first barrier) covers them
        const __amdgpu_buffer_rsrc_t pr0 = layer_rsrc(a.pw[0], a.pwbytes[0]);
        h8 ah = fload(pr0, voff, (w * 2 + 0) * 1024), al = fload(pr0, voff, (w * 2 + 1) * 1024);
        h8 nh[PPn > 0 ? PPn : 1], nl[PPn > 0 ? PPn : 1];
        auto load_layer = [&](int l) __attribute__((always_inline)) {
            const __amdgpu_buffer_rsrc_t rs = layer_rsrc(a.pw[l], a.pwbytes[l]);
#pragma unroll
            for (int p = 0; p < PPn; ++p) {
                nh[p] = fload(rs, voff, ((w * PPn + p) * 2 + 0) * 1024);
                nl[p] = fload(rs, voff, ((w * PPn + p) * 2 + 1) * 1024);
            }
        };
        if (PL > 1) load_layer(1);
        const __amdgpu_buffer_rsrc_t pro = layer_rsrc(a.pw[PL], a.pwbytes[PL]);    // output: k-step w/2
        const h8 oh = fload(pro, voff, ((w >> 1) * 2 + 0) * 1024), ol = fload(pro, voff, ((w >> 1) * 2 + 1) * 1024);
        double uu[4] = {0.0, 0.0, 0.0, 0.0};            // explore draws (controllers.py:191), issued early
        if (actor && a.pol_mode != BCMPC_POLICY_STOCHASTIC) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 + 4 * q + r - S;
                if (X3_POLDIAG != 2 && valid && j >= 0 && j < A && a.actions)   // the caller's array (no CEM)
                    uu[r] = a.actions[((int64_t)h * a.K + cand) * A + j];
            }
        }
        if (owner) {
            float z[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * hv0 + 4 * q + r;
                float v = 0.f;
                if (d < S) {
                    v = X3_POLDIAG == 4 ? ((float)s[0][r] - pm[d]) * pm[32 + d] : ((float)s[0][r] - pm[d]) / pm[32 + d];
                    v = fminf(fmaxf(v, -5.0f), 5.0f);
                }
                z[r] = v * 2048.0f;
            }
            h2 h01, l01, h23, l23;
            split2(z[0], z[1], h01, l01);
            split2(z[2], z[3], h23, l23);
            reinterpret_cast<h4*>(slab0 + (cw * 2 + 0) * 64 + lane)[hv0] = (h4){h01[0], h01[1], h23[0], h23[1]};
            reinterpret_cast<h4*>(slab0 + (cw * 2 + 1) * 64 + lane)[hv0] = (h4){l01[0], l01[1], l23[0], l23[1]};
        }
        X3_BARRIER();                                   // policy input published
        f4 pacc[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const h8 bh = sread(slab0 + (c * 2 + 0) * 64 + lane), bl = sread(slab0 + (c * 2 + 1) * 64 + lane);
            pacc[c] = mfma16(ah, bh, (f4){0.f, 0.f, 0.f, 0.f});
            pacc[c] = mfma16(ah, bl, pacc[c]);
            pacc[c] = mfma16(al, bh, pacc[c]);
        }
        h4 xh[NC], xl[NC];                              // this wave's tile of the current layer
        auto epi = [&](float f, const float* bias) __attribute__((always_inline)) {
            const f4 b = *reinterpret_cast<const f4*>(bias + 16 * w + 4 * q);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = tanh_x4096(fmaf(pacc[c][r], f, b[r]));
                h2 h01, l01, h23, l23;
                split2(v[0], v[1], h01, l01);
                split2(v[2], v[3], h23, l23);
                xh[c] = (h4){h01[0], h01[1], h23[0], h23[1]};
                xl[c] = (h4){l01[0], l01[1], l23[0], l23[1]};
            }
        };
        epi(a.pwinv[0] * kTanhK, Pb);
        for (int l = 1; l < (X3_POLDIAG == 1 ? 1 : PL); ++l) {
            if (l > 1) X3_BARRIER();                    // every wave is done reading the slab
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                reinterpret_cast<h4*>(slab + sidx<NC>(w >> 1, c, 0, lane))[w & 1] = xh[c];
                reinterpret_cast<h4*>(slab + sidx<NC>(w >> 1, c, 1, lane))[w & 1] = xl[c];
            }
            X3_BARRIER();                               // layer input complete
#pragma unroll
            for (int c = 0; c < NC; ++c) pacc[c] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int p = 0; p < PPn; ++p)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const h8 bh = sread(slab + sidx<NC>(p, c, 0, lane)), bl = sread(slab + sidx<NC>(p, c, 1, lane));
                    pacc[c] = mfma16(nh[p], bh, pacc[c]);
                    pacc[c] = mfma16(nh[p], bl, pacc[c]);
                    pacc[c] = mfma16(nl[p], bh, pacc[c]);
                }
            if (l + 1 < PL) load_layer(l + 1);
            epi(a.pwinv[l] * kTanhK, Pb + l * PHP);
        }
        // output layer, K-split: this wave's 16 neurons are one half of a k-step B fragment
        f4* part = slab + sidx<NC>(PPn, 0, 0, 0);      // [NW][NC] partial tiles, past the hidden input
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            h8 bh = (h8)(_Float16)0.0f, bl = (h8)(_Float16)0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bh[(w & 1) * 4 + i] = xh[c][i];
                bl[(w & 1) * 4 + i] = xl[c][i];
            }
            f4 po = mfma16(oh, bh, (f4){0.f, 0.f, 0.f, 0.f});
            po = mfma16(oh, bl, po);
            po = mfma16(ol, bh, po);
            part[(w * NC + c) * 64 + lane] = po;
        }
        X3_BARRIER();                                   // partials complete
        if (!actor || X3_POLDIAG == 3) return;
        f4 o = part[(0 * NC + cw) * 64 + lane];
#pragma unroll
        for (int g = 1; g < NW; ++g) o += part[(g * NC + cw) * 64 + lane];   // fixed summation order
        const float fo_p = a.pwinv[PL];
        const uint64_t gcand = (uint64_t)(a.cand_offset + cand);
        if (!a.actions && a.pol_mode != BCMPC_POLICY_STOCHASTIC) {   // Philox draws, computed in place
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 + 4 * q + r - S;
                if (valid && j >= 0 && j < A) uu[r] = rng_action(a.seed, gcand, h, j, C[6 * 32 + j], C[7 * 32 + j]);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = 16 + 4 * q + r - S;
            if (j < 0 || j >= A) continue;
            const float mean = o[r] * fo_p + pm[80 + 4 * q + r];       // dense bias (f32)
            if (a.pol_mode == BCMPC_POLICY_STOCHASTIC) {
                const float sd = expf(pm[64 + j]);
                pact[r] = (double)(mean + sd * rng_normal(a.seed ^ 0x9E3779B97F4A7C15ull, gcand, h, j));
            } else {
                // (1 - explore) * mean in f32 (NumPy keeps the f32 dtype), + explore * U in f64
                const float t1 = (float)(1.0 - a.explore) * mean;
                pact[r] = __dadd_rn((double)t1, __dmul_rn(a.explore, uu[r]));
            }
            if (a.act_out && h < a.act_out_steps && valid)          // action_paths (controllers.py:213)
                __hip_atomic_store(&a.act_out[((int64_t)h * a.K + cand) * A + j], pact[r], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);       // (sc1: read by the fused argmin)
        }
    };

    if constexpr (X3_PRIO == 1)
        if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (X3_STAGGER > 0)                     // diagnostic: de-phase alternate workgroups
        if (blockIdx.x & 1)
            for (int i = 0; i < X3_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    uint64_t ph_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tp_ = X3_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    for (int h = 0; h < a.H; ++h) {
        wz = 0;
        asm volatile("" : "+s"(wz));
        Cv = C + wz;
        Blv = Bl + wz;
        double pact[4] = {0.0, 0.0, 0.0, 0.0};            // policy actions of dims 16 + 4q + r (half-1 owners)
        if constexpr (PHP > 0) {
            policy_step(h, pact);
            // (with a policy the layer-0 fragments are fetched after it: registers)
            aload_x3<TW>(rs0, voff, w * TW * 2048, a0h, a0l);
        }
        X3_ST(0);
        float xin[4 * NHV];                               // layer-0 input slots 4*(hv0+k) + r
        float mx = 0.f;
        if (owner && !X3_DIAG_NOOWNER) {
            // ---- normalise the state (dynamics.py:109), cast to f32 (TF feed), column max ----
            const float* xr = xa + ((h % NCH) * CB + 16 * cw + m) * A;
            if constexpr (PHP > 0 || AK != 0 || F1 || HP > X3_BF_MAXHP) {
#pragma unroll
                for (int k = 0; k < NHV; ++k)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * (hv0 + k) + 4 * q + r;
                        float xv = 0.f;
                        if (d < S) {
                            xv = (float)div_rn(__dsub_rn(s[k][r], Cv[0 * 32 + d]), Cv[1 * 32 + d], Cv[8 * 32 + d]);
                        } else if (d < S + A) {
                            if constexpr (PHP > 0) {              // the policy's action (dynamics.py:110)
                                const int j = d - S;
                                xv = (float)div_rn(__dsub_rn(pact[r], Cv[2 * 32 + j]), Cv[3 * 32 + j], Cv[9 * 32 + j]);
                            } else {
                                xv = xr[d - S];
                            }
                        }
                        xin[4 * k + r] = xv;
                    }
            } else {
                // (branch-free: every slot's operands are requested first -- the constants table has 32
                //  columns, the action index is clamped -- and each slot picks its value after; per-slot
                //  branches issued each slot's LDS reads and waited for them before the next slot's.  Only the
                //  plain tanh split kernels up to hidden 512: the others have no registers to spare -- 2 to 14
                //  more spilled registers each)
                double c0[NHV][4], c1[NHV][4], c8[NHV][4];
                float av[NHV][4];
#pragma unroll
                for (int k = 0; k < NHV; ++k)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * (hv0 + k) + 4 * q + r;
                        c0[k][r] = Cv[0 * 32 + d];
                        c1[k][r] = Cv[1 * 32 + d];
                        c8[k][r] = Cv[8 * 32 + d];
                        av[k][r] = xr[min(max(d - S, 0), A - 1)];
                    }
                float xs_[NHV][4];
#pragma unroll
                for (int k = 0; k < NHV; ++k)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        xs_[k][r] = (float)div_rn(__dsub_rn(s[k][r], c0[k][r]), c1[k][r], c8[k][r]);
                        asm volatile("" : "+v"(xs_[k][r]));     // (every lane, every slot: not sunk into a branch)
                    }
#pragma unroll
                for (int k = 0; k < NHV; ++k)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * (hv0 + k) + 4 * q + r;
                        xin[4 * k + r] = d < S ? xs_[k][r] : (d < S + A ? av[k][r] : 0.f);
                    }
            }
#pragma unroll
            for (int i = 0; i < 4 * NHV; ++i) mx = fmaxf(mx, fabsf(xin[i]));
            mx = max_rows32(max_rows16(mx));
            if constexpr (SO) {
                if (q == 0) colmax[hv0 * NC * 16 + cw * 16 + m] = mx;
            }
        }
        if constexpr (SO) {
            X3_BARRIER_ID(0);                             // both halves' column maxima published
            if (owner && !X3_DIAG_NOOWNER) mx = fmaxf(mx, colmax[(1 - hv0) * NC * 16 + cw * 16 + m]);
        }
        if (owner && !X3_DIAG_NOOWNER) {
            // ---- column scale (max |x| -> [2^11, 2^12)), split, publish ----
            int e = 0;
            (void)frexpf(mx, &e);                         // mx in [2^(e-1), 2^e)
            int sh = 12 - e;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
            const float sc = ldexpf(1.0f, sh);
#pragma unroll
            for (int i = 0; i < 4 * NHV; ++i) xin[i] *= sc;
            if constexpr (SO) {
                typedef _Float16 h4 __attribute__((ext_vector_type(4)));
                h4 xh, xl;
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    h2 hh, ll;
                    split2(xin[i], xin[i + 1], hh, ll);
                    xh[i] = hh[0]; xh[i + 1] = hh[1];
                    xl[i] = ll[0]; xl[i + 1] = ll[1];
                }
                // this half's 4 slots are bytes [8*hv0, 8*hv0+8) of the lane's 16-byte B fragment
                reinterpret_cast<h4*>(slab0 + (cw * NPT + 0) * 64 + lane)[hv0] = xh;
                if constexpr (!F1) reinterpret_cast<h4*>(slab0 + (cw * NPT + 1) * 64 + lane)[hv0] = xl;
                if (hv0 == 0 && q == 0) colf[cw * 16 + m] = ldexpf(a.winv[0], -sh) * kAct;
            } else {
                h8 xh, xl;
                split8(xin, xh, xl);
                swrite(slab0 + (cw * NPT + 0) * 64 + lane, xh);
                if constexpr (!F1) swrite(slab0 + (cw * NPT + 1) * 64 + lane, xl);
                if (q == 0) colf[cw * 16 + m] = ldexpf(a.winv[0], -sh) * kAct;
            }
        }
        X3_ST(1);
        X3_BARRIER_ID(1);                              // layer-0 input published
        X3_ST(2);

        // ---- layer 0 [S+A -> h] ----
        f4 acc[TW][NC];
#pragma unroll
        for (int j = 0; j < TW; ++j)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
        {
            h8 bh[NC], bl[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                bh[c] = sread(slab0 + (c * NPT + 0) * 64 + lane);
                bl[c] = F1 ? bh[c] : sread(slab0 + (c * NPT + 1) * 64 + lane);
            }
#pragma unroll
            for (int c = 0; c < NC; ++c) {
#pragma unroll
                for (int j = 0; j < TW; ++j) acc[j][c] = mfma16(a0h[j], bh[c], acc[j][c]);
                if constexpr (F1) continue;
#pragma unroll
                for (int j = 0; j < TW; ++j) acc[j][c] = mfma16(a0h[j], bl[c], acc[j][c]);
#pragma unroll
                for (int j = 0; j < TW; ++j) acc[j][c] = mfma16(a0l[j], bh[c], acc[j][c]);
            }
        }
        if constexpr (RW)                                  // the reward head runs first
            aload_x3<G>(layer_rsrc(a.w[3], a.wbytes[3]), voff, w * P * TW * 2048 + kown * TW * 2048, uh, ul);
        else
            load_next(1);
        h8 xh[PW][NC], xl[PW][NC];                        // this wave's activations of the current layer
        if constexpr (AK != 0) {
            float f0[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) f0[c] = colf[c * 16 + m];
            epi_colx<AK, TW, NC, NW>(acc, f0, Blv, lnp, lnp + L * HP, a.hsc[0], a.hidden, xch, w, lane, xh, xl, fcol);
        } else {
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], colf[c * 16 + m], Blv, w * TW + 2 * pp, q,
                             xh[pp][c], xl[pp][c]);
        }
        X3_ST(3);

        f4 po1[NC];                                       // RW: the reward row's output partial (tile 1)
#pragma unroll
        for (int c = 0; c < NC; ++c) po1[c] = (f4){0.f, 0.f, 0.f, 0.f};
        if constexpr (RW) {
            // ---- both heads read the trunk's output from one slab (no barrier between them) ----
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    swrite(slab + sidx<NC>(w * PW + pp, c, 0, lane), xh[pp][c]);
                    swrite(slab + sidx<NC>(w * PW + pp, c, 1, lane), xl[pp][c]);
                }
            // reward head [h -> h] (dense_3), then its output row (dense_4) from registers
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
            {
                auto ready = [&]() __attribute__((always_inline)) { X3_BARRIER_ID(3); };   // trunk output complete
                mm_x3<TW, NC, P, G, X3_OWN != 0, PW>(layer_rsrc(a.w[3], a.wbytes[3]), w * P * TW * 2048, slab, acc,
                                                     lane, uh, ul, kown, ready);
                if constexpr (!X3_OWN) ready();
            }
            aload_x3<G>(layer_rsrc(a.w[1], a.wbytes[1]), voff, w * P * TW * 2048, uh, ul);   // delta head unit 0
            h8 rh[PW], rl[PW];
            {
                const __amdgpu_buffer_rsrc_t rsr = layer_rsrc(a.w[4], a.wbytes[4]);
#pragma unroll
                for (int pp = 0; pp < PW; ++pp) {
                    rh[pp] = fload(rsr, voff, ((w * PW + pp) * 2 + 0) * 1024);
                    rl[pp] = fload(rsr, voff, ((w * PW + pp) * 2 + 1) * 1024);
                }
            }
            const float fr = a.winv[3] * kTanhK;
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], fr, Blv + 2 * HP, w * TW + 2 * pp, q, xh[pp][c],
                             xl[pp][c]);
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    po1[c] = mfma16(rh[pp], xh[pp][c], po1[c]);
                    po1[c] = mfma16(rh[pp], xl[pp][c], po1[c]);
                    po1[c] = mfma16(rl[pp], xh[pp][c], po1[c]);
                }
            // delta head [h -> h] (dense_1)
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
            mm_x3<TW, NC, P, G>(layer_rsrc(a.w[1], a.wbytes[1]), w * P * TW * 2048, slab, acc, lane, uh, ul);
            load_next(L);                                  // delta out (L == 2)
            const float fd = a.winv[1] * kTanhK;
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], fd, Blv + HP, w * TW + 2 * pp, q, xh[pp][c],
                             xl[pp][c]);
        }
        // ---- hidden layers 1..L-1 [h -> h] through the slab ----
        for (int l = 1; l < (RW ? 1 : L); ++l) {
            // (l == 1: the slab's last readers were the owners' partial sums, before the barrier above)
            if (l > 1 && AK == 0) X3_BARRIER_ID(2);    // every wave is done reading the slab (AK: barrier 6 was)
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    swrite(slab + sidx<NC, F1>(w * PW + pp, c, 0, lane), xh[pp][c]);
                    if constexpr (!F1) swrite(slab + sidx<NC, F1>(w * PW + pp, c, 1, lane), xl[pp][c]);
                }
            auto ready = [&]() __attribute__((always_inline)) { X3_BARRIER_ID(3); };   // layer input complete
            X3_ST(4);
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
            const float f = a.winv[l] * kAct;
            // own k-steps first: this wave's slab writes need no barrier
            if (NRES > 0 && l == 1) {
                if constexpr (NRES > 0)
                    mm_x3<TW, NC, P, G, true, PW, F1, NRES>(layer_rsrc(a.w[l], a.wbytes[l]), w * P * TW * 2048, slab,
                                                            acc, lane, uh, ul, kown, ready, rsh, rsl);
            } else {
                mm_x3<TW, NC, P, G, X3_OWN != 0, PW, F1>(layer_rsrc(a.w[l], a.wbytes[l]), w * P * TW * 2048, slab, acc,
                                                         lane, uh, ul, kown, ready);
            }
            if constexpr (!X3_OWN) ready();
            X3_ST(5);
            load_next(l + 1);
            if constexpr (AK != 0) {
                float fl[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) fl[c] = DYN ? f * fcol[c] : f;
                epi_colx<AK, TW, NC, NW>(acc, fl, Blv + l * HP, lnp + l * HP, lnp + (L + l) * HP, a.hsc[l], a.hidden,
                                         xch, w, lane, xh, xl, fcol);
            } else {
#pragma unroll
                for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                    for (int c = 0; c < NC; ++c)
                        epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], f, Blv + l * HP, w * TW + 2 * pp, q,
                                 xh[pp][c], xl[pp][c]);
            }
        }
        X3_ST(6);

        // ---- output layer [h -> S] (2 tiles), K-split: this wave's own k-steps from registers ----
        f4 po[2][NC];
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int c = 0; c < NC; ++c) po[v][c] = v == 1 ? po1[c] : (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int pp = 0; pp < PW; ++pp) {
            const int slot = pp % OP;
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    po[v][c] = mfma16(oh[2 * slot + v], xh[pp][c], po[v][c]);
                    if constexpr (F1) continue;
                    po[v][c] = mfma16(oh[2 * slot + v], xl[pp][c], po[v][c]);
                    po[v][c] = mfma16(ol[2 * slot + v], xh[pp][c], po[v][c]);
                }
            if (pp + OP < PW) {
                if (slot == 0) load_out(pp + OP, std::integral_constant<int, 0>{});
                else load_out(pp + OP, std::integral_constant<int, OP - 1>{});
            }
        }
        __builtin_amdgcn_sched_barrier(0);              // (not hoisted above the MFMAs' operand waits)
        if constexpr (PHP == 0) aload_x3<TW, F1>(rs0, voff, wz + w * TW * 2048, a0h, a0l);   // next step's layer 0
        // the owners reach this point first (the older waves win the MFMA arbitration):
        // they stage the next chunk's action inputs while the others finish
        if constexpr (PHP == 0)
            if (owner && (h + 1) % NCH == 0 && h + 1 < a.H) fill_actions(h + 1, 64 * (SO ? 2 * NC : NC));
        X3_ST(7);
        X3_BARRIER_ID(4);                              // every wave is done reading the slab
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int c = 0; c < NC; ++c) slab[((w * 2 + v) * NC + c) * 64 + lane] = po[v][c];
        X3_BARRIER_ID(5);                              // partials complete
        X3_ST(8);
        if (!owner || X3_DIAG_NOOWNER) continue;

        f4 o[NHV];
#pragma unroll
        for (int k = 0; k < NHV; ++k) o[k] = slab[((0 * 2 + hv0 + k) * NC + cw) * 64 + lane];
#pragma unroll
        for (int g = 1; g < NW; ++g)                      // fixed summation order
#pragma unroll
            for (int k = 0; k < NHV; ++k) o[k] += slab[((g * 2 + hv0 + k) * NC + cw) * 64 + lane];

        // ---- cheetah penalties on the current state (cost_functions.py:16-26): dims 5, 6, 7
        //      live in lane row q = 1 of half 0; 0 + 10 + 10 + 10 in the reference's order is
        //      exactly 10 * count ----
        int npen = 0;
        if (hv0 == 0) npen = partner_row16((s[0][1] >= 0.2) + (s[0][2] >= 0.0) + (s[0][3] >= 0.0));
        const double s17 = s[NHV - 1][1];                 // dim 17: half 1, row q = 0, r = 1
        // ---- de-normalise + residual (dynamics.py:113,116), f64, no FMA ----
        float foc = fo;                                   // DYN: undo the last hidden layer's column scale
        if constexpr (DYN) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (c == cw) foc = fo * fcol[c];
        }
        if constexpr (PHP > 0 || AK != 0 || F1 || HP > X3_BF_MAXHP) {
#pragma unroll
            for (int k = 0; k < NHV; ++k) {
                const f4 bv = *reinterpret_cast<const f4*>(Blv + LB * HP + 16 * (hv0 + k) + 4 * q);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * (hv0 + k) + 4 * q + r;
                    if (d < S) {
                        const float dn = fmaf(o[k][r], foc, bv[r]);            // BiasAdd (f32)
                        const double ud = __dadd_rn(__dmul_rn((double)dn, Cv[5 * 32 + d]), Cv[4 * 32 + d]);
                        s[k][r] = __dadd_rn(s[k][r], ud);
                    }
                }
            }
        } else {
            // (branch-free, as the layer-0 input above: the constants of every slot requested first, every
            //  slot's update computed, the dims < S keep theirs)
            double c4[NHV][4], c5[NHV][4];
#pragma unroll
            for (int k = 0; k < NHV; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * (hv0 + k) + 4 * q + r;
                    c4[k][r] = Cv[4 * 32 + d];
                    c5[k][r] = Cv[5 * 32 + d];
                }
#pragma unroll
            for (int k = 0; k < NHV; ++k) {
                const f4 bv = *reinterpret_cast<const f4*>(Blv + LB * HP + 16 * (hv0 + k) + 4 * q);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * (hv0 + k) + 4 * q + r;
                    const float dn = fmaf(o[k][r], foc, bv[r]);                // BiasAdd (f32)
                    double sn = __dadd_rn(s[k][r], __dadd_rn(__dmul_rn((double)dn, c5[k][r]), c4[k][r]));
                    asm volatile("" : "+v"(sn));
                    s[k][r] = d < S ? sn : s[k][r];
                }
            }
        }
        if constexpr (RW) {
            // ---- learned reward (dynamics.py:236) * gamma**h, running sum (controllers.py:139,150):
            //      output row S (tile 1: S >= 16) in lane row q = (S & 15) >> 2, register S & 3 ----
            const int kS = 1 - hv0;                       // the half-1 slot of this owner's state
            if (kS < NHV && q == ((S & 15) >> 2)) {
                float o_s = 0.f;
#pragma unroll
                for (int k = 0; k < NHV; ++k)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (k == kS && r == (S & 3)) o_s = o[k][r];
                const float nr = fmaf(o_s, fo, Bout[S]);                   // BiasAdd (f32)
                const double rw = __dadd_rn(__dmul_rn((double)nr, a.std_reward), a.mean_reward);
                cost = __dadd_rn(cost, __dmul_rn(rw, a.gpow[h]));
            }
        }
        if (a.cost == BCMPC_COST_CHEETAH) {
            // score = pen - (s'17 - s17) / 0.01 (cost_functions.py:28), summed in step order (:59-63)
            if constexpr (SO) {
                // half 0 hands its penalty count to half 1 through LDS; half 1 adds step h-1's
                // score now (the count is visible after this step's barriers) and step H-1's
                // after the loop
                if (hv0 == 0) {
                    if (q == 0) penbuf[(h & 1) * NC * 16 + cw * 16 + m] = npen;
                } else {
                    if (h > 0) {
                        const double pen = 10.0 * (double)penbuf[((h - 1) & 1) * NC * 16 + cw * 16 + m];
                        cost = __dadd_rn(cost, __dsub_rn(pen, prog_prev));
                    }
                    prog_prev = div_rn(__dsub_rn(s[0][1], s17), 0.01, 1.0 / 0.01);
                }
            } else {
                const double score = __dsub_rn(10.0 * (double)npen, div_rn(__dsub_rn(s[1][1], s17), 0.01, 1.0 / 0.01));
                cost = __dadd_rn(cost, score);
            }
        }
        if (a.traj && valid) {
#pragma unroll
            for (int k = 0; k < NHV; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * (hv0 + k) + 4 * q + r;
                    if (d < S) a.traj[((int64_t)(h + 1) * a.K + cand) * S + d] = s[k][r];
                }
        }
    }
    if constexpr (SO) {
        __syncthreads();                                  // the last step's penalty counts
        if (a.cost == BCMPC_COST_CHEETAH && owner && hv0 == 1 && a.H > 0) {
            const double pen = 10.0 * (double)penbuf[((a.H - 1) & 1) * NC * 16 + cw * 16 + m];
            cost = __dadd_rn(cost, __dsub_rn(pen, prog_prev));
        }
    }
    // the cost holder: half 1, lane row 0 (cheetah) / the reward row's lanes (RW)
    const bool holder = valid && q == (RW ? (S & 15) >> 2 : 0) && (SO ? hv0 == 1 : true);
    if (a.costs && holder) a.costs[cand] = cost;
    if constexpr (X3_STAMP) {
        if (a.stamps && lane == 0)
            for (int k = 0; k < 10; ++k) a.stamps[((size_t)blockIdx.x * NW + w) * 10 + k] = ph_[k];
    }
    if (a.fused_argmin) {
        // ---- np.argmin / argmax (controllers.py:82,152) fused: this workgroup's best, then the
        //      last workgroup to finish reduces every workgroup's record (ticket; the agent-scope
        //      release / acquire recipe of cdna_hip_programming.md "In-launch split-K reduction") ----
        const ArgminArgs& m = a.amin;
        Best best{__builtin_inf(), INT64_MAX};
        if (holder) best = Best{m.maximize ? -cost : cost, cand};
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
            if (better(o, best)) best = o;
        }
        double* rc = reinterpret_cast<double*>(slab);          // (the slab is free after the last step)
        int64_t* ri = reinterpret_cast<int64_t*>(rc + 16);
        __syncthreads();
        if (lane == 0) { rc[w] = best.c; ri[w] = best.i; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < NW; ++k) {
                const Best o{rc[k], ri[k]};
                if (better(o, best)) best = o;
            }
            // write-through (sc1) record stores need no release fence; the policy's act_out rows
            // are stored the same way (cdna_hip_programming.md, in-launch reduction, sc1 form)
            __hip_atomic_store(&m.scratch_c[blockIdx.x], best.c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&m.scratch_i[blockIdx.x], best.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(a.amin_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool last = t == gridDim.x - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            ri[16] = last ? 1 : 0;
        }
        __syncthreads();
        if (ri[16] == 0) return;
        best = Best{__builtin_inf(), INT64_MAX};
        for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
            const Best o{m.scratch_c[b], m.scratch_i[b]};
            if (better(o, best)) best = o;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
            if (better(o, best)) best = o;
        }
        __syncthreads();
        if (lane == 0) { rc[w] = best.c; ri[w] = best.i; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < NW; ++k) {
                const Best o{rc[k], ri[k]};
                if (better(o, best)) best = o;
            }
            argmin_write(m, best);
            *a.amin_ticket = 0;                        // ready for the next launch (stream order)
        }
    }
}

// ------------------------------------------------------------ rollout_pp ----
// Single-pass f16 (BCMPC_PREC_F16) as a two-group software pipeline (round 4; the plain 2-layer tanh
// delta net at hidden 512).  rollout_x3's step is a lock-step chain: every wave of the workgroup runs the
// same phase at once (f64 state update, layer 0 and its tanh, the hidden layer's MFMAs, its tanh and the
// output layer), so the SIMDs' matrix pipes idle through the VALU phases and the VALU through the MFMA
// phase (PMC + stamps + ablations: profiles/r04_pmc_f16/).  Here a 512-thread workgroup holds TWO
// independent 64-candidate groups, waves 0-3 and 4-7 (waves w and w + 4 share a SIMD), each with its own
// hi-only slab.  A group's control step is three segments:
//   C  (wave wl owns column wl of its group, all 32 state dims): the output partials of the previous step
//      summed in fixed order, f64 de-normalise + residual + cheetah cost, f64 normalise of the next input
//      (column power-of-two scale), layer 0 for its OWN column from registers (all 32 tiles: the B fragment
//      is the lane's own 8 inputs, no slab, no barrier), its tanh, its column of the hidden-layer slab;
//   M  the hidden layer's MFMAs (wave wl: tiles [8wl, 8wl + 8) of all 4 columns, slab B fragments);
//   E  its tanh, the K-split output layer (the wave's own 4 k-steps from registers), the partials into
//      the slab, the next action inputs staged.
// Every segment ends at the workgroup barrier, and group 1 runs one segment ahead of group 0, so each
// barrier interval pairs C with E (VALU beside VALU: the two waves of a SIMD interleave their VALU), M with
// C and E with M (the matrix pipe of one wave beside the other's VALU).  C touches only its own column of
// the slab (partials and layer input alike: fragment index = c mod NC), so it needs no barrier of its own;
// M reads what every C of its group wrote (one interval earlier); E overwrites the slab only after every M
// of its group has read it (one interval earlier).  Arithmetic as rollout_x3<..., F1 = true>: the same
// f16 operands and power-of-two scales, f32 accumulate, f64 state / cost.
#ifndef PP_NCH
#define PP_NCH 4                 // steps of action inputs staged per fill
#endif
__host__ __device__ constexpr int pp_xa_bytes(int A) { return (PP_NCH * 64 * A * 4 + 15) & ~15; }
__host__ __device__ constexpr int pp_group_bytes(int HP, int A) { return pp_xa_bytes(A) + (HP / 32) * 4 * 1024; }
__host__ __device__ constexpr int pp_lds_bytes(int HP, int A) { return param_bytes(2, HP) + 2 * pp_group_bytes(HP, A); }
// (+ the groups' counters [2][2] ints | layer-0 slabs [2][NC] fragments | column factors [2][64])
__host__ __device__ constexpr int pp_lds_total(int HP, int A) { return pp_lds_bytes(HP, A) + 16 + 2 * 4 * 1024 + 2 * 64 * 4; }

// The hidden layer of one group (single pass, hi operands): acc[j][c] += W[tile j] x X[c] over the P
// k-steps, fully unrolled (no loop-carried operand sets: fixed accumulator registers).  Weights in units of
// PG tiles through PD + 1 register sets, PD units in flight ahead of the MFMAs (the wave is alone on its
// SIMD's matrix pipe in this segment: nothing else hides its L2 latency); s0 holds units 0..PD-1.
// (round 5, folded operands: PP_G 1 x PP_D 4 -- the same 4 KiB in flight per wave, one tile per unit --
//  measured 0.78 vs 0.785 ms, G2 x D2 / G1 x D6 / + a one-k-step B prefetch within +-0.5%: the segment is not
//  bound by its weight loads' latency; profiles/r05_pp_prefetch_ab.txt, profiles/r05_pp_prio_ab.txt)
#ifndef PP_G
#define PP_G 1
#endif
#ifndef PP_D
#define PP_D 4
#endif
#ifndef PP_BPRE
#define PP_BPRE 0
#endif
// wave priority per segment (s_setprio).  Without it the arbiter's age order favours group 0 in both of its
// segments (stamps: group 1's C segment 20k ticks, group 0's 13.7k; profiles/r04_pp_stamps.log).  C ahead
// of ME evens the groups out (profiles/r04_ppprio_stamps.log) but the interval stays bound by ME; ME ahead
// measured best by 1-2% (profiles/r04_ppprio_ab.jsonl: 0.860-0.867 vs 0.876-0.887 ms C-first, 0.867-0.873 none);
// round 5 with the folded operands (C and ME now ~18k ticks each): ME-first 0.785 ms, equal 0.811, C-first 0.835
// (profiles/r05_pp_prio_ab.txt)
#ifndef PP_PRIO_C
#define PP_PRIO_C 0
#endif
#ifndef PP_PRIO_ME
#define PP_PRIO_ME 2
#endif
// byte offset of operand j of mm_pp's first units (unit j / PP_G: k-step u / NG, tile group u % NG of the half
// [T0, T0 + TWH); the order mm_pp loads them in)
__device__ __forceinline__ constexpr int pp_unit_off(int j, int T0, int TW, int TWH) {
    return ((j / PP_G) / (TWH / PP_G)) * TW * 2048 + (T0 + ((j / PP_G) % (TWH / PP_G)) * PP_G + j % PP_G) * 2048;
}
template <int TW, int NC, int P, int PG, int PD, int TWH = TW, int T0 = 0, bool BIAS = false>
__device__ __forceinline__ void mm_pp(__amdgpu_buffer_rsrc_t rs, int wbase, const f4* slab, f4 (&acc)[TWH][NC],
                                      int lane, const h8 (&s0)[PD * PG], const f4* bias = nullptr) {
    // (BIAS: the first k-step's MFMAs take bias[tile] as their C operand -- the accumulators start from the
    //  bias, no separate initialisation)
    // (TWH < TW: tiles [T0, T0 + TWH) of the wave's TW only)
    constexpr int NG = TWH / PG, NU = P * NG, NS = PD + 1;
    const int voff = lane * 16;
    h8 sr[NS][PG], bh[NC];
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int j = 0; j < PG; ++j) sr[d][j] = s0[d * PG + j];
    if constexpr (PP_DIAG_MFMA32 && BIAS) {
#pragma unroll
        for (int j = 0; j < TWH; ++j)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[j][c] = bias[j];
    }
    // (PP_BPRE: the next k-step's B fragments are read one k-step ahead, a second register set)
    h8 bn[PP_BPRE ? NC : 1];
    if constexpr (PP_BPRE) {
#pragma unroll
        for (int c = 0; c < NC; ++c) bn[c] = sread(slab + sidx<NC, true>(0, c, 0, lane));
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        if (u + PD < NU) {
            const int un = u + PD;
#pragma unroll
            for (int j = 0; j < PG; ++j)
                sr[un % NS][j] = fload(rs, voff, wbase + (un / NG) * TW * 2048 + (T0 + (un % NG) * PG + j) * 2048);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (u % NG == 0) {
            if constexpr (PP_BPRE) {
#pragma unroll
                for (int c = 0; c < NC; ++c) bh[c] = bn[c];
                if (u / NG + 1 < P)
#pragma unroll
                    for (int c = 0; c < NC; ++c) bn[c] = sread(slab + sidx<NC, true>(u / NG + 1, c, 0, lane));
            } else {
#pragma unroll
                for (int c = 0; c < NC; ++c) bh[c] = sread(slab + sidx<NC, true>(u / NG, c, 0, lane));
            }
        }
        const int g = u % NG;
        if constexpr (PP_DIAG_MFMA32) {
            // tile unit t = g*PG + j as (row tile t/2, sub-step t%2); B fragment c as (column tile c/2,
            // sub-step c%2); accumulators [TWH][NC] f4 reinterpreted as [TWH/2][NC/2] f16-vectors
            typedef float f16v __attribute__((ext_vector_type(16)));
            static_assert(TWH % 2 == 0 && NC % 2 == 0, "pairs");
#pragma unroll
            for (int j = 0; j < PG; ++j) {
                const int t = g * PG + j;
#pragma unroll
                for (int ct = 0; ct < NC / 2; ++ct) {
                    f16v* av = reinterpret_cast<f16v*>(&acc[(t / 2) * 2][ct * 2]);
                    (void)av;
                    f16v x;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        x[e] = acc[(t / 2) * 2][ct * 2][e];
                        x[4 + e] = acc[(t / 2) * 2][ct * 2 + 1][e];
                        x[8 + e] = acc[(t / 2) * 2 + 1][ct * 2][e];
                        x[12 + e] = acc[(t / 2) * 2 + 1][ct * 2 + 1][e];
                    }
                    x = __builtin_amdgcn_mfma_f32_32x32x16_f16(sr[u % NS][j], bh[ct * 2 + (t & 1)], x, 0, 0, 0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        acc[(t / 2) * 2][ct * 2][e] = x[e];
                        acc[(t / 2) * 2][ct * 2 + 1][e] = x[4 + e];
                        acc[(t / 2) * 2 + 1][ct * 2][e] = x[8 + e];
                        acc[(t / 2) * 2 + 1][ct * 2 + 1][e] = x[12 + e];
                    }
                }
            }
            continue;
        }
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < PG; ++j)
                acc[g * PG + j][c] = mfma16(sr[u % NS][j], bh[c],
                                            BIAS && u < NG ? bias[g * PG + j] : acc[g * PG + j][c]);
    }
}

// FOLD (the default, BCMPC_PP_FOLD=0 turns it off): the host packs both hidden-producing layers as
// f16(W x 2 log2 e) with no power-of-two scales, the MFMAs start from the bias x 2 log2 e, so the
// accumulators are z and the epilogue is epi_pair_fold (one VALU operation per element fewer); the
// layer-0 input goes to f16 unscaled (|x| clamped below f16's overflow, NaN kept), no per-column power of
// two; the hidden activations are tanh in [-1, 1] (the output layer's scale is 1 / its weight scale)
template <int HP, bool FOLD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void rollout_pp(const RolloutArgs a) {
    constexpr int NC = 4;                         // 16-candidate columns per group
    constexpr int T = HP / 16, P = T / 2;         // hidden tiles, k-steps
    constexpr int TW = T / 4, PW = TW / 2;        // per wave (4 waves per group)
    constexpr int CB = 16 * NC;                   // candidates per group
    static_assert(T == 32 && TW == 8 && PW == 4, "hidden 512");
    static_assert(PP_D <= P * (TW / 2 / PP_G) && (TW / 2) % PP_G == 0, "prefetch within one tile half's units");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = w >> 2, wl = w & 3;
    const int q = lane >> 4, m = lane & 15;
    const int64_t gc0 = (int64_t)blockIdx.x * (2 * CB) + grp * CB;     // the group's first candidate
    const int64_t cand = gc0 + 16 * wl + m;                           // this lane's candidate (column wl)
    const bool valid = cand < a.K;
    const int S = a.S, A = a.A;

    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < 2; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i] * kTanhK;
    float* const Bout = Bl + 2 * HP;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bout[i] = a.b[2][i];
    char* const gbase = reinterpret_cast<char*>(lds) + param_bytes(2, HP) + grp * pp_group_bytes(HP, A);
    float* const xa = reinterpret_cast<float*>(gbase);                  // [PP_NCH][CB][A] normalised actions
    f4* const slab = reinterpret_cast<f4*>(gbase + pp_xa_bytes(A));     // [P][NC] hi fragments | partials

    // lane (q, m) holds dims 16k + 4q + r (k = 0, 1) of its candidate: the MFMA B-fragment order
    double s[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int d = 16 * k + 4 * q + r;
            s[k][r] = (valid && d < S) ? (a.state_inline ? a.state_v[d] : a.state[cand * a.state_stride + d]) : 0.0;
        }
    if (a.traj && valid) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * k + 4 * q + r;
                if (d < S) a.traj[cand * S + d] = s[k][r];
            }
    }
    double cost = 0.0;                                  // trajectory_cost = 0 (cost_functions.py:60)

    // the group's action inputs of PP_NCH steps from h0: f64 normalise (dynamics.py:110), f32 (the TF
    // feed); the group's 256 threads
    const int gt = threadIdx.x - 256 * grp;
    auto fill_actions = [&](int h0) __attribute__((always_inline)) {
        const int nhs = (a.H - h0 < PP_NCH) ? a.H - h0 : PP_NCH;
        if (!a.cem_mu && !a.actions) {
            const int AP = (A + 1) >> 1, per = CB * AP;
            for (int i = gt; i < nhs * per; i += 256) {
                const int hh = i / per, rem = i - hh * per, kl = rem / AP, p2 = rem - kl * AP;
                const int j0 = 2 * p2, j1 = min(2 * p2 + 1, A - 1);
                float x0 = 0.f, x1 = 0.f;
                if (gc0 + kl < a.K) {
                    double v0, v1;
                    rng_action_pair(a.seed, (uint64_t)(a.cand_offset + gc0 + kl), h0 + hh, p2, C[6 * 32 + j0],
                                    C[7 * 32 + j0], C[6 * 32 + j1], C[7 * 32 + j1], v0, v1);
                    x0 = (float)div_rn(__dsub_rn(v0, C[2 * 32 + j0]), C[3 * 32 + j0], C[9 * 32 + j0]);
                    x1 = (float)div_rn(__dsub_rn(v1, C[2 * 32 + j1]), C[3 * 32 + j1], C[9 * 32 + j1]);
                }
                float* const dst = xa + (hh * CB + kl) * A;
                dst[j0] = x0;
                if (2 * p2 + 1 < A) dst[j1] = x1;
            }
            return;
        }
        const int per = CB * A;
        for (int i = gt; i < nhs * per; i += 256) {
            const int hh = i / per, rem = i - hh * per, kl = rem / A, j = rem - kl * A;
            float xv = 0.f;
            if (gc0 + kl < a.K) {
                const int64_t c = gc0 + kl;
                const uint64_t gg = (uint64_t)(a.cand_offset + c);
                const double v = a.cem_mu ? cem_action(a.seed, gg, h0 + hh, j, a.cem_iter, a.cem_mu[(h0 + hh) * A + j],
                                                       a.cem_sigma[(h0 + hh) * A + j], C[6 * 32 + j], C[7 * 32 + j])
                                          : a.actions[((int64_t)(h0 + hh) * a.K + c) * A + j];
                xv = (float)div_rn(__dsub_rn(v, C[2 * 32 + j]), C[3 * 32 + j], C[9 * 32 + j]);
            }
            xa[(hh * CB + kl) * A + j] = xv;
        }
    };
    fill_actions(0);
    __syncthreads();

    const int voff = lane * 16;
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(a.w[0], a.wbytes[0]);
    const __amdgpu_buffer_rsrc_t rs1 = layer_rsrc(a.w[1], a.wbytes[1]);
    const __amdgpu_buffer_rsrc_t rso = layer_rsrc(a.w[2], a.wbytes[2]);
    const float f1 = a.winv[1] * kTanhK, fo = a.winv[2];
    const int wbase1 = wl * P * TW * 2048;              // this wave's hidden-layer weight slice
    f4* const slab0 = reinterpret_cast<f4*>(reinterpret_cast<char*>(lds) + pp_lds_bytes(HP, A) + 16) + grp * NC * 64;
    float* const colf = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + pp_lds_bytes(HP, A) + 16 +
                                                 2 * NC * 1024) + grp * CB;
    // per-group LDS counters (monotone over the steps): C's layer-0 inputs published, M's slab reads done
    int* const cnt = reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + pp_lds_bytes(HP, A)) + 2 * grp;
    if (threadIdx.x < 4) reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + pp_lds_bytes(HP, A))[threadIdx.x] = 0;
    __syncthreads();

    f4 acc[TW][NC];
    h8 uh[PP_D * PP_G];                                 // ME's first PP_D operand units (issued in C)
    // (X3_STAMP variant builds: s_memtime per phase; slots 0 C/owner, 1 C/wait for the group's inputs,
    //  2 C/layer 0 + tanh, 3 ME/MFMAs, 4 ME/tanh + output, 5 ME/group wait, 6 ME/partials + fill,
    //  7 barrier, 8 idle segments)
    uint64_t ph_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tp_ = X3_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    const int nseg = 2 * a.H + 1;                       // C(0) ME(0) ... ME(H-1) C(H) (the last cost)
    for (int k = 0; k < nseg + 1; ++k) {
        // (an opaque zero added to every weight offset and LDS table base: the weights and tables are the
        //  same every step, and without it the compiler hoists the loop-invariant loads out of the loop)
        int wz = 0;
        asm volatile("" : "+s"(wz));
        const double* const Cz = C + wz;
        const float* const Blz = Bl + wz;
        const float* const Boutz = Bout + wz;
        const int seg = k - (grp == 0 ? 1 : 0);         // group 1 runs one segment ahead
        if (seg >= 0 && seg < nseg) {
            const int h = seg >> 1;
            if ((seg & 1) == 0) {
                // ---------------- C(h) ----------------
                __builtin_amdgcn_s_setprio(PP_PRIO_C);
                // this wave's layer-0 fragments, in flight through the owner phase
                h8 a0[TW];
#pragma unroll
                for (int j = 0; j < TW; ++j) a0[j] = fload(rs0, voff, wz + (wl * TW + j) * 2048);
                if (h > 0) {
                    f4 o[2];
#pragma unroll
                    for (int v = 0; v < 2; ++v) o[v] = slab[((0 * 2 + v) * NC + wl) * 64 + lane];
#pragma unroll
                    for (int g2 = 1; g2 < 4; ++g2)                 // fixed summation order
#pragma unroll
                        for (int v = 0; v < 2; ++v) o[v] += slab[((g2 * 2 + v) * NC + wl) * 64 + lane];
                    // cheetah penalties on the current state (cost_functions.py:16-26): dims 5..7 in row q = 1
                    const int npen = partner_row16((s[0][1] >= 0.2) + (s[0][2] >= 0.0) + (s[0][3] >= 0.0));
                    const double s17 = s[1][1];
                    // de-normalise + residual (dynamics.py:113,116), f64, no FMA
#pragma unroll
                    for (int v = 0; v < 2; ++v) {
                        const f4 bv = *reinterpret_cast<const f4*>(Boutz + 16 * v + 4 * q);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int d = 16 * v + 4 * q + r;
                            if (d < S) {
                                const float dn = fmaf(o[v][r], fo, bv[r]);
                                const double ud = __dadd_rn(__dmul_rn((double)dn, Cz[5 * 32 + d]), Cz[4 * 32 + d]);
                                s[v][r] = __dadd_rn(s[v][r], ud);
                            }
                        }
                    }
                    if (a.cost == BCMPC_COST_CHEETAH) {
                        const double score = __dsub_rn(10.0 * (double)npen,
                                                       div_rn(__dsub_rn(s[1][1], s17), 0.01, 1.0 / 0.01));
                        cost = __dadd_rn(cost, score);
                    }
                    if (a.traj && valid) {
#pragma unroll
                        for (int v = 0; v < 2; ++v)
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int d = 16 * v + 4 * q + r;
                                if (d < S) a.traj[((int64_t)h * a.K + cand) * S + d] = s[v][r];
                            }
                    }
                }
                if (h < a.H) {
                    // normalise the state (dynamics.py:109), f32 (TF feed), the staged actions; the column's
                    // power-of-two scale; its B fragment into the layer-0 slab
                    const float* xr = xa + ((h % PP_NCH) * CB + 16 * wl + m) * A;
                    float xin[8];
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int d = 16 * v + 4 * q + r;
                            float xv = 0.f;
                            if (d < S) xv = (float)div_rn(__dsub_rn(s[v][r], Cz[0 * 32 + d]), Cz[1 * 32 + d], Cz[8 * 32 + d]);
                            else if (d < S + A) xv = xr[d - S];
                            xin[4 * v + r] = xv;
                        }
                    h8 bown;                                   // (the k order of pack_x3_layer)
                    if constexpr (FOLD) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) {          // |x| below f16's overflow, NaN kept
                            const float xc = fminf(fmaxf(xin[i], -65504.0f), 65504.0f);
                            bown[i] = (_Float16)(xin[i] == xin[i] ? xc : xin[i]);
                        }
                    } else {
                        float mx = 0.f;
#pragma unroll
                        for (int i = 0; i < 8; ++i) mx = fmaxf(mx, fabsf(xin[i]));
                        mx = max_rows32(max_rows16(mx));
                        int e = 0;
                        (void)frexpf(mx, &e);                  // column scale: max |x| -> [2^11, 2^12)
                        int sh = 12 - e;
                        sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
                        const float sc = ldexpf(1.0f, sh);
#pragma unroll
                        for (int i = 0; i < 8; ++i) bown[i] = (_Float16)(xin[i] * sc);
                        if (q == 0) colf[16 * wl + m] = ldexpf(a.winv[0], -sh) * kTanhK;
                    }
                    swrite(slab0 + wl * 64 + lane, bown);
                }
                // publish: a workgroup-scope release of this wave's LDS writes (slab0 / colf, and its reads of
                // the partials), then the count; LDS only ("local"), so the weight loads stay in flight
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                X3_ST(0);
                if (h < a.H) {
                    // the group's four layer-0 inputs published (and every partial of the slab read)
                    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4 * (h + 1))
                        __builtin_amdgcn_s_sleep(1);
                    // (acquire: the slab0 / colf reads below cannot move above the wait)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                    X3_ST(1);
                    // layer 0 [S+A -> h]: this wave's 8 tiles x the group's 4 columns
                    h8 b0[NC];
#pragma unroll
                    for (int c = 0; c < NC; ++c) b0[c] = sread(slab0 + c * 64 + lane);
                    f4 z4[TW];
#pragma unroll
                    for (int j = 0; j < TW; ++j)
                        z4[j] = FOLD ? *reinterpret_cast<const f4*>(Blz + 16 * (wl * TW + j) + 4 * q)
                                     : (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int c = 0; c < NC; ++c)
#pragma unroll
                        for (int j = 0; j < TW; ++j) acc[j][c] = mfma16(a0[j], b0[c], z4[j]);
                    // ME's first operand units, in flight through the tanh below and the barrier
#pragma unroll
                    for (int j = 0; j < PP_D * PP_G; ++j)          // (units 0..PP_D-1 of tile half 0)
                        uh[j] = fload(rs1, voff, wz + wbase1 + pp_unit_off(j, 0, TW, TW / 2));
                    // tanh, this wave's 4 k-steps of the hidden-layer slab (all 4 columns)
#pragma unroll
                    for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                        for (int c = 0; c < NC; ++c) {
                            h8 xh, xl;
                            if constexpr (FOLD)
                                xh = epi_pair_fold(acc[2 * pp][c], acc[2 * pp + 1][c]);
                            else
                                epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], colf[16 * c + m], Blz, wl * TW + 2 * pp,
                                         q, xh, xl);
                            swrite(slab + ((wl * PW + pp) * NC + c) * 64 + lane, xh);
                        }
                }
                X3_ST(2);
            } else {
                // ---------------- ME(h): the hidden layer's MFMAs, its tanh, the output layer ----------------
                __builtin_amdgcn_s_setprio(PP_PRIO_ME);
                f4 po[2][NC];
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int c = 0; c < NC; ++c) po[v][c] = (f4){0.f, 0.f, 0.f, 0.f};
                // in two halves of the wave's 8 tiles (64 accumulator registers instead of 128; each slab k-step
                // read twice): half 0's tanh and output MFMAs run after its MFMAs while half 1's first weight
                // units are in flight
                auto half = [&](auto HFc) __attribute__((always_inline)) {
                    constexpr int hf = decltype(HFc)::value;
                    constexpr int TWH = TW / 2;
                    f4 ah[TWH][NC];
                    if constexpr (FOLD) {
                        f4 bias1[TWH];                          // (the accumulators start from the bias)
#pragma unroll
                        for (int j = 0; j < TWH; ++j)
                            bias1[j] = *reinterpret_cast<const f4*>(Blz + HP + 16 * (wl * TW + hf * TWH + j) + 4 * q);
                        mm_pp<TW, NC, P, PP_G, PP_D, TWH, hf * TWH, true>(rs1, wz + wbase1, slab, ah, lane, uh, bias1);
                    } else {
#pragma unroll
                        for (int j = 0; j < TWH; ++j)
#pragma unroll
                            for (int c = 0; c < NC; ++c) ah[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
                        mm_pp<TW, NC, P, PP_G, PP_D, TWH, hf * TWH>(rs1, wz + wbase1, slab, ah, lane, uh);
                    }
                    if constexpr (hf == 0) {
#pragma unroll
                        for (int j = 0; j < PP_D * PP_G; ++j)      // half 1's first units
                            uh[j] = fload(rs1, voff, wz + wbase1 + pp_unit_off(j, TWH, TW, TWH));
                    } else {
                        // this wave's slab reads have returned: count it (the group's partials overwrite the
                        // slab only once all 4 waves have, below)
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                        if (lane == 0) __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
#pragma unroll
                    for (int pp2 = 0; pp2 < PW / 2; ++pp2) {
                        const int pp = hf * (PW / 2) + pp2;            // this wave's k-step of the output layer
                        h8 oh[2];
#pragma unroll
                        for (int v = 0; v < 2; ++v)
                            oh[v] = fload(rso, voff, wz + (((wl * PW + pp) * 2 + v) * 2) * 1024);
#pragma unroll
                        for (int c = 0; c < NC; ++c) {
                            h8 xh, xl;
                            if constexpr (FOLD)
                                xh = epi_pair_fold(ah[2 * pp2][c], ah[2 * pp2 + 1][c]);
                            else
                                epi_pair(ah[2 * pp2][c], ah[2 * pp2 + 1][c], f1, Blz + HP, wl * TW + 2 * pp, q, xh, xl);
#pragma unroll
                            for (int v = 0; v < 2; ++v) po[v][c] = mfma16(oh[v], xh, po[v][c]);
                        }
                    }
                };
                half(std::integral_constant<int, 0>{});
                half(std::integral_constant<int, 1>{});
                X3_ST(3);
                X3_ST(4);
                // every wave of the group has finished reading the slab (by now the others are normally long
                // past their MFMAs)
                while (__hip_atomic_load(cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4 * (h + 1))
                    __builtin_amdgcn_s_sleep(1);
                // (acquire: the partial writes below cannot move above the wait)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                X3_ST(5);
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int c = 0; c < NC; ++c) slab[((wl * 2 + v) * NC + c) * 64 + lane] = po[v][c];
                if ((h + 1) % PP_NCH == 0 && h + 1 < a.H) fill_actions(h + 1);
                X3_ST(6);
            }
        } else {
            X3_ST(8);
        }
        __syncthreads();
        X3_ST(7);
    }
    if constexpr (X3_STAMP) {
        if (a.stamps && lane == 0)
            for (int k2 = 0; k2 < 10; ++k2) a.stamps[((size_t)blockIdx.x * 8 + w) * 10 + k2] = ph_[k2];
    }

    const bool holder = valid && q == 0;                // cost in row 0 (dims 1, 17 and the penalty count)
    if (a.costs && holder) a.costs[cand] = cost;
    if (a.fused_argmin) {
        // np.argmin fused (as rollout_x3): this workgroup's best, the last workgroup reduces the records
        const ArgminArgs& am = a.amin;
        Best best{__builtin_inf(), INT64_MAX};
        if (holder) best = Best{am.maximize ? -cost : cost, cand};
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
            if (better(o, best)) best = o;
        }
        double* rc = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + param_bytes(2, HP) + pp_xa_bytes(A));
        int64_t* ri = reinterpret_cast<int64_t*>(rc + 16);
        if (lane == 0) { rc[w] = best.c; ri[w] = best.i; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < 8; ++k) {
                const Best o{rc[k], ri[k]};
                if (better(o, best)) best = o;
            }
            __hip_atomic_store(&am.scratch_c[blockIdx.x], best.c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&am.scratch_i[blockIdx.x], best.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned tk = __hip_atomic_fetch_add(a.amin_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool last = tk == gridDim.x - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            ri[16] = last ? 1 : 0;
        }
        __syncthreads();
        if (ri[16] == 0) return;
        best = Best{__builtin_inf(), INT64_MAX};
        for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
            const Best o{am.scratch_c[b], am.scratch_i[b]};
            if (better(o, best)) best = o;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
            if (better(o, best)) best = o;
        }
        __syncthreads();
        if (lane == 0) { rc[w] = best.c; ri[w] = best.i; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < 8; ++k) {
                const Best o{rc[k], ri[k]};
                if (better(o, best)) best = o;
            }
            argmin_write(am, best);
            *a.amin_ticket = 0;
        }
    }
}

// ------------------------------------------------------------ launchers ----
#ifndef X3_PROBE           // (tools/x3_probe.sh: one instantiation, resource report only)
// X3_PART splits the instantiations over two translation units so each can be built with its own
// scheduler (Makefile): 1 = the plain tanh delta net without a policy (cfg2..cfg5; built with
// -amdgpu-sched-strategy=iterative-ilp, measured -2% kernel time at cfg3), 2 = everything else plus
// the host helpers (built with max-ilp: -0.6..1.7%; iterative-ilp spills the policy + reward
// kernel), 0 = both in one unit (variant builds).
#ifndef X3_PART
#define X3_PART 0
#endif
hipError_t launch_rollout_x3_plain(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st);

template <int HP, int NC, int NW, int PHP = 0, bool RW = false, int AK = 0, bool F1 = false>
static hipError_t launch_x3_t(const RolloutArgs& a, hipStream_t st) {
    if constexpr (NC > NW || x3_lds_bytes_rt(HP, NC, 1, 1, 0, 0, AK, NW, F1) > 160 * 1024) {
        (void)a; (void)st;
        return hipErrorInvalidValue;
    } else {
        if (PHP > 0 && (a.pL < 1 || a.phidden_padded != PHP)) return hipErrorInvalidValue;
        static bool attr_set = false;
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)rollout_x3<HP, NC, NW, PHP, RW, AK, F1>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
        if (RW != (a.model == BCMPC_MODEL_REWARD) || (RW && (a.L != 2 || a.S < 16))) return hipErrorInvalidValue;
        if (AK != ((a.act == BCMPC_ACT_RELU ? 1 : 0) | (a.ln ? 2 : 0))) return hipErrorInvalidValue;
        if (F1 != (a.f16_single != 0)) return hipErrorInvalidValue;
        const size_t lds = (size_t)x3_lds_bytes_rt(HP, NC, RW ? 3 : a.L, a.A, PHP > 0 ? a.pL : 0, PHP, AK, NW, F1);
        if (lds > 160 * 1024) return hipErrorInvalidValue;
        const int64_t blocks = (a.K + 16 * NC - 1) / (16 * NC);
        hipLaunchKernelGGL((rollout_x3<HP, NC, NW, PHP, RW, AK, F1>), dim3((unsigned)blocks), dim3(64 * NW), lds, st, a);
        return hipGetLastError();
    }
}

#if X3_PART != 1
int x3_waves(int hidden_padded) {
    switch (hidden_padded) {
        case 64: return 2;
        case 128: return 4;
        case 256: return X3_NW256;
        case 512: return X3_NW512;
        case 1024: return X3_NW1024;
        default: return 8;          // 768
    }
}

// widest candidate group (16-candidate columns) the build instantiates for a width:
// the accumulators of TW tiles x NC columns must fit beside the operand sets
int x3_max_nc(int hidden_padded) {
#ifdef X3_ONLY
    return hidden_padded == X3_ONLY ? X3_ONLY_NC : 0;
#else
    const int tw = hidden_padded / 16 / x3_waves(hidden_padded);
    return tw >= 8 ? 2 : 4;
#endif
}

// fused policy: one 128-wide policy tile per wave of an 8-wave group
bool x3_policy_ok(int hidden_padded, int nc) {
#ifdef X3_ONLY
    return hidden_padded == X3_ONLY && X3_NW512 == 8 && 2 * nc <= 8 && hidden_padded >= 512;
#else
    return x3_waves(hidden_padded) == 8 && 2 * nc <= 8 && hidden_padded >= 512;
#endif
}

size_t x3_lds(int hidden_padded, int n_layers, int nc, int action_dim, int policy_layers, int policy_hidden_padded,
              int ak) {
    return (size_t)x3_lds_bytes_rt(hidden_padded, nc, n_layers, action_dim, policy_layers, policy_hidden_padded, ak,
                                   x3_waves(hidden_padded));
}

#endif  // X3_PART != 1

// the plain tanh delta net without a policy (X3_PART 1); F1: single-pass f16 (BCMPC_PREC_F16)
template <int NC, bool F1>
static hipError_t launch_x3_plain_ncf(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    switch (hidden_padded) {
        case 64: return launch_x3_t<64, NC, 2, 0, false, 0, F1>(a, st);
        case 128: return launch_x3_t<128, NC, 4, 0, false, 0, F1>(a, st);
        case 256: return launch_x3_t<256, NC, X3_NW256, 0, false, 0, F1>(a, st);
        case 512: return launch_x3_t<512, NC, X3_NW512, 0, false, 0, F1>(a, st);
        case 768:
            if constexpr (NC <= 2) return launch_x3_t<768, NC, 8, 0, false, 0, F1>(a, st);
            return hipErrorInvalidValue;
        case 1024:
            if constexpr (NC <= 2) return launch_x3_t<1024, NC, X3_NW1024, 0, false, 0, F1>(a, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}
// (the single-pass instantiations live in X3_PART 2: iterative-ILP crashes the compiler on them)
hipError_t launch_rollout_x3_f16(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st);
template <int NC>
static hipError_t launch_x3_plain_nc(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
#ifdef X3_ONLY
    if (a.f16_single) return hipErrorInvalidValue;
#else
    if (a.f16_single) return launch_rollout_x3_f16(a, hidden_padded, NC, st);
#endif
    return launch_x3_plain_ncf<NC, false>(a, hidden_padded, st);
}
#if X3_PART != 1 && !defined(X3_ONLY)
// Single-pass layouts beyond the split kernel's (the hi-only slab is half the size): at hidden 512,
// 128-candidate groups (NC = 8, 8 waves: each 1-KiB weight fragment feeds 8 MFMAs) and two 64-candidate
// 4-wave groups per CU (NC = 4, NW = 4: one group's serial f64 / epilogue chain beside the other's
// MFMAs); at hidden 768 / 1024, 64-candidate groups (NC = 4).
bool x3_f16_layout_ok(int hidden_padded, int nc, int nw) {
    const int nwd = x3_waves(hidden_padded);
    if (nw == nwd && (nc == 1 || nc == 2)) return true;
    if (nw == nwd && nc == 4) return true;
    if (hidden_padded == 512) return (nc == 8 && nw == 8) || (nc == 4 && nw == 4);
    return false;
}
size_t x3_f16_lds(int hidden_padded, int n_layers, int nc, int nw, int action_dim) {
    return (size_t)x3_lds_bytes_rt(hidden_padded, nc, n_layers, action_dim, 0, 0, 0, nw, true);
}
bool x3_pp_ok(int hidden_padded, int n_layers, int state_dim, int action_dim) {
    return hidden_padded == 512 && n_layers == 2 && state_dim + action_dim <= 32 &&
           pp_lds_total(512, action_dim) <= 160 * 1024;
}
hipError_t launch_rollout_x3_f16(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st) {
    if (a.x3_pp) {
        if (!x3_pp_ok(hidden_padded, a.L, a.S, a.A) || a.model != BCMPC_MODEL_DELTA || a.pL > 0 ||
            a.act != BCMPC_ACT_TANH || a.ln || !a.f16_single)
            return hipErrorInvalidValue;
        static bool attr_set = false;
        if (!attr_set) {
            for (const void* f : {(const void*)rollout_pp<512, false>, (const void*)rollout_pp<512, true>}) {
                const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                if (e != hipSuccess) return e;
            }
            attr_set = true;
        }
        const int64_t blocks = (a.K + 127) / 128;
        if (a.x3_pp == 2)
            hipLaunchKernelGGL((rollout_pp<512, true>), dim3((unsigned)blocks), dim3(512), (size_t)pp_lds_total(512, a.A),
                               st, a);
        else
            hipLaunchKernelGGL((rollout_pp<512, false>), dim3((unsigned)blocks), dim3(512), (size_t)pp_lds_total(512, a.A),
                               st, a);
        return hipGetLastError();
    }
    const int nw = a.x3_nw ? a.x3_nw : x3_waves(hidden_padded);
    if (!x3_f16_layout_ok(hidden_padded, nc, nw)) return hipErrorInvalidValue;
    if (hidden_padded == 512 && nw == 4) return launch_x3_t<512, 4, 4, 0, false, 0, true>(a, st);
    if (hidden_padded == 512 && nc == 8) return launch_x3_t<512, 8, 8, 0, false, 0, true>(a, st);
    if (nc == 4 && hidden_padded == 768) return launch_x3_t<768, 4, 8, 0, false, 0, true>(a, st);
    if (nc == 4 && hidden_padded == 1024) return launch_x3_t<1024, 4, X3_NW1024, 0, false, 0, true>(a, st);
    switch (nc) {
        case 1: return launch_x3_plain_ncf<1, true>(a, hidden_padded, st);
        case 2: return launch_x3_plain_ncf<2, true>(a, hidden_padded, st);
        case 4: return launch_x3_plain_ncf<4, true>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}
#endif
#ifdef X3_ONLY   // (variant builds carry no single-pass layouts: capi.cpp still links their shape queries)
bool x3_f16_layout_ok(int, int, int) { return false; }
size_t x3_f16_lds(int, int, int, int, int) { return 0; }
bool x3_pp_ok(int, int, int, int) { return false; }
hipError_t launch_rollout_x3_f16(const RolloutArgs&, int, int, hipStream_t) { return hipErrorInvalidValue; }
#endif

#if X3_PART == 1 && !defined(X3_ONLY)
hipError_t launch_rollout_x3_plain(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st) {
    switch (nc) {
        case 1: return launch_x3_plain_nc<1>(a, hidden_padded, st);
        case 2: return launch_x3_plain_nc<2>(a, hidden_padded, st);
        case 4: return launch_x3_plain_nc<4>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}
#endif

#if X3_PART != 1
// relu and / or LayerNorm nets (AK != 0): the plain delta net, hidden <= 512
template <int NC, int AK>
static hipError_t launch_x3_ak(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    switch (hidden_padded) {
        case 64: return launch_x3_t<64, NC, 2, 0, false, AK>(a, st);
        case 128: return launch_x3_t<128, NC, 4, 0, false, AK>(a, st);
        case 256: return launch_x3_t<256, NC, X3_NW256, 0, false, AK>(a, st);
        case 512: return launch_x3_t<512, NC, X3_NW512, 0, false, AK>(a, st);
        default: return hipErrorInvalidValue;
    }
}

template <int NC>
static hipError_t launch_x3_nc(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
#ifdef X3_ONLY          // variant builds (tools/build_variants.sh): one width, NC = 4 only
    if constexpr (NC == X3_ONLY_NC) {
        if (hidden_padded != X3_ONLY || a.model == BCMPC_MODEL_REWARD) return hipErrorInvalidValue;
        if constexpr (X3_ONLY <= 512) {   // relu / LayerNorm delta nets (the ppo_defaults net at 256)
            constexpr int NWO = X3_ONLY == 256 ? X3_NW256 : X3_ONLY == 512 ? X3_NW512 : X3_ONLY == 64 ? 2 : 4;
            if (a.act == BCMPC_ACT_RELU || a.ln) {
                if (a.pL > 0) return hipErrorInvalidValue;
                if (a.act == BCMPC_ACT_RELU)
                    return a.ln ? launch_x3_t<X3_ONLY, X3_ONLY_NC, NWO, 0, false, 3>(a, st)
                                : launch_x3_t<X3_ONLY, X3_ONLY_NC, NWO, 0, false, 1>(a, st);
                return launch_x3_t<X3_ONLY, X3_ONLY_NC, NWO, 0, false, 2>(a, st);
            }
        }
        if (a.pL > 0) {                   // the delta net with a fused policy (8-wave groups only)
            if constexpr (X3_NW512 == 8 && X3_ONLY >= 512) return launch_x3_t<X3_ONLY, X3_ONLY_NC, 8, 128>(a, st);
            return hipErrorInvalidValue;
        }
        return launch_x3_t<X3_ONLY, X3_ONLY_NC, X3_ONLY == 1024 ? X3_NW1024 : X3_NW512>(a, st);
    }
    return hipErrorInvalidValue;
#else
    if (a.act == BCMPC_ACT_RELU || a.ln) {
        if (a.model == BCMPC_MODEL_REWARD || a.pL > 0) return hipErrorInvalidValue;
        if (a.act == BCMPC_ACT_RELU) return a.ln ? launch_x3_ak<NC, 3>(a, hidden_padded, st)
                                                 : launch_x3_ak<NC, 1>(a, hidden_padded, st);
        return launch_x3_ak<NC, 2>(a, hidden_padded, st);
    }
    if (a.model == BCMPC_MODEL_REWARD) {      // NNDynamicsRewardModel (hidden <= 512)
        if (a.pL > 0) {
            if constexpr (X3_NW512 == 8)
                if (hidden_padded == 512 && a.phidden_padded == 128) return launch_x3_t<512, NC, 8, 128, true>(a, st);
            return hipErrorInvalidValue;
        }
        switch (hidden_padded) {
            case 64: return launch_x3_t<64, NC, 2, 0, true>(a, st);
            case 128: return launch_x3_t<128, NC, 4, 0, true>(a, st);
            case 256: return launch_x3_t<256, NC, X3_NW256, 0, true>(a, st);
            case 512: return launch_x3_t<512, NC, X3_NW512, 0, true>(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    if (a.pL > 0) {
        if (a.phidden_padded != 128) return hipErrorInvalidValue;
        switch (hidden_padded) {
            case 512:
                if constexpr (X3_NW512 == 8) return launch_x3_t<512, NC, 8, 128>(a, st);
                return hipErrorInvalidValue;
            case 768:
                if constexpr (NC <= 2) return launch_x3_t<768, NC, 8, 128>(a, st);
                return hipErrorInvalidValue;
            case 1024:
                if constexpr (NC <= 2) return launch_x3_t<1024, NC, 8, 128>(a, st);
                return hipErrorInvalidValue;
            default: return hipErrorInvalidValue;
        }
    }
#if X3_PART == 0
    return launch_x3_plain_nc<NC>(a, hidden_padded, st);
#else
    return launch_rollout_x3_plain(a, hidden_padded, NC, st);
#endif
#endif
}

hipError_t launch_rollout_x3(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st) {
    switch (nc) {
        case 1: return launch_x3_nc<1>(a, hidden_padded, st);
        case 2: return launch_x3_nc<2>(a, hidden_padded, st);
        case 4: return launch_x3_nc<4>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}
#endif  // X3_PART != 1
#endif  // X3_PROBE

}  // namespace bcmpc
