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

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"

namespace bcmpc {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// tanh(y) * 2^12: 4096 (1 - t) / (1 + t), t = e^{-2|y|}, sign restored.  Absolute
// error ~1e-7 (x 4096) near 0, a few ulp elsewhere; NaN propagates, +-inf -> +-4096.
__device__ __forceinline__ float tanh_x4096(float y) {
    const float t = __builtin_amdgcn_exp2f(fabsf(y) * -2.8853900817779268f);
    const float r = __builtin_amdgcn_rcpf(fmaf(t, 1.0f / 4096.0f, 1.0f / 4096.0f));
    return __builtin_copysignf(fmaf(-t, r, r), y);
}

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const _Float16 h = (_Float16)v[i];
        hi[i] = h;
        lo[i] = (_Float16)(v[i] - (float)h);
    }
}

__device__ __forceinline__ h8 fload(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

__device__ __forceinline__ h8 sread(const f4* p) { return __builtin_bit_cast(h8, *p); }
__device__ __forceinline__ void swrite(f4* p, h8 v) { *p = __builtin_bit_cast(f4, v); }

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// slab index of (k-step p, column c, part) in f4 units of one lane
template <int NC>
__device__ __forceinline__ int sidx(int p, int c, int part, int lane) {
    return ((p * NC + c) * 2 + part) * 64 + lane;
}

// acc[j][c] += sum over k-steps of W[tile j] * X[c]: weights streamed from L2
// (this wave's contiguous slice, one k-step ahead in registers), activations
// from the slab (one k-step ahead; the slab has one spare k-step at the end).
template <int TW, int NC, int P>
__device__ __forceinline__ void mm_x3(__amdgpu_buffer_rsrc_t rs, int wbase, const f4* slab, f4 (&acc)[TW][NC],
                                      int lane) {
    constexpr int STEPB = TW * 2048;
    const int voff = lane * 16;
    h8 ah[TW], al[TW], bh[NC], bl[NC];
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        ah[j] = fload(rs, voff, wbase + j * 2048);
        al[j] = fload(rs, voff, wbase + j * 2048 + 1024);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bh[c] = sread(slab + sidx<NC>(0, c, 0, lane));
        bl[c] = sread(slab + sidx<NC>(0, c, 1, lane));
    }
    for (int p = 0; p < P; ++p) {
        h8 nah[TW], nal[TW], nbh[NC], nbl[NC];
#pragma unroll
        for (int j = 0; j < TW; ++j) {
            nah[j] = fload(rs, voff, wbase + (p + 1) * STEPB + j * 2048);
            nal[j] = fload(rs, voff, wbase + (p + 1) * STEPB + j * 2048 + 1024);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            nbh[c] = sread(slab + sidx<NC>(p + 1, c, 0, lane));
            nbl[c] = sread(slab + sidx<NC>(p + 1, c, 1, lane));
        }
#pragma unroll
        for (int j = 0; j < TW; ++j)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(ah[j], bh[c], acc[j][c]);
#pragma unroll
        for (int j = 0; j < TW; ++j)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(ah[j], bl[c], acc[j][c]);
#pragma unroll
        for (int j = 0; j < TW; ++j)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(al[j], bh[c], acc[j][c]);
#pragma unroll
        for (int j = 0; j < TW; ++j) {
            ah[j] = nah[j];
            al[j] = nal[j];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            bh[c] = nbh[c];
            bl[c] = nbl[c];
        }
    }
}

// Epilogue of one tile pair (k-step) for one column: BiasAdd (f32, after undoing
// the operand scales with one exact power-of-two multiply), tanh, x 2^12, split.
__device__ __forceinline__ void epi_pair(const f4& a0, const f4& a1, float f, const float* __restrict__ bias,
                                         int t0, int q, h8& hi, h8& lo) {
    const f4 b0 = *reinterpret_cast<const f4*>(bias + 16 * t0 + 4 * q);
    const f4 b1 = *reinterpret_cast<const f4*>(bias + 16 * (t0 + 1) + 4 * q);
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r] = tanh_x4096(fmaf(a0[r], f, b0[r]));
        v[4 + r] = tanh_x4096(fmaf(a1[r], f, b1[r]));
    }
    split8(v, hi, lo);
}

template <int HP, int NC, int NW>
__host__ __device__ constexpr int x3_lds_bytes(int L) {
    // consts | biases (L*HP + 32) | column factors NC*16 | layer-0 slab NC*2 KiB | slab (P+1)*NC*2 KiB
    return param_bytes(L, HP) + NC * 16 * 4 + NC * 2048 + (HP / 32 + 1) * NC * 2048;
}

template <int HP, int NC, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW >= 8 ? 2 : 1, 8)))
void rollout_x3(const RolloutArgs a) {
    constexpr int T = HP / 16;          // hidden tiles
    constexpr int P = T / 2;            // hidden k-steps (32 wide)
    constexpr int TW = T / NW;          // output tiles per wave
    constexpr int PW = TW / 2;          // k-steps produced per wave
    static_assert(TW % 2 == 0 && TW * NW == T, "each wave must own whole tile pairs");
    static_assert(NC <= NW, "one owner wave per column");
    static_assert(P >= NW, "the output-layer partials reuse the slab");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;
    const int m = lane & 15;
    const bool owner = w < NC;
    const int cw = owner ? w : 0;                       // the owner's column
    const int64_t cand = (int64_t)blockIdx.x * (16 * NC) + 16 * cw + m;
    const bool valid = owner && cand < a.K;
    const int S = a.S, A = a.A, L = a.L;

    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < L; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i];
    float* const Bout = Bl + L * HP;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bout[i] = a.b[L][i];
    float* colf = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + param_bytes(L, HP));
    f4* slab0 = reinterpret_cast<f4*>(colf + NC * 16);
    f4* slab = slab0 + NC * 2 * 64;
    __syncthreads();

    double s[2][4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int d = 16 * v + 4 * q + r;
            s[v][r] = (valid && d < S) ? a.state[cand * a.state_stride + d] : 0.0;
        }
    if (a.traj && valid) {
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                if (d < S) a.traj[cand * S + d] = s[v][r];
            }
    }
    double cost = 0.0;                                  // trajectory_cost = 0 (cost_functions.py:60)
    const uint64_t gcand = (uint64_t)(a.cand_offset + cand);
    auto fetch_uniform = [&](int h, int j) -> double {
        if (!valid) return 0.0;
        if (a.cem_mu)
            return cem_action(a.seed, gcand, h, j, a.cem_iter, a.cem_mu[h * A + j], a.cem_sigma[h * A + j],
                              C[6 * 32 + j], C[7 * 32 + j]);
        return a.actions ? a.actions[((int64_t)h * a.K + cand) * A + j]
                         : rng_action(a.seed, gcand, h, j, C[6 * 32 + j], C[7 * 32 + j]);
    };
    const int voff = lane * 16;
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(a.w[0], a.wbytes[0]);
    const __amdgpu_buffer_rsrc_t rso = layer_rsrc(a.w[L], a.wbytes[L]);
    const float fo = a.winv[L];

    for (int h = 0; h < a.H; ++h) {
        // ---- layer-0 weights first (state-independent): this wave's TW tiles, one k-step ----
        h8 a0h[TW], a0l[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) {
            a0h[j] = fload(rs0, voff, (w * TW + j) * 2048);
            a0l[j] = fload(rs0, voff, (w * TW + j) * 2048 + 1024);
        }
        if (owner) {
            // ---- normalise (dynamics.py:109-110), cast to f32 (TF feed), column scale, split ----
            float x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int v = i >> 2, r = i & 3;
                const int d = 16 * v + 4 * q + r;
                float xv = 0.f;
                if (d < S) {
                    xv = (float)__ddiv_rn(__dsub_rn(s[v][r], C[0 * 32 + d]), C[1 * 32 + d]);
                } else if (d < S + A) {
                    const int j = d - S;
                    xv = (float)__ddiv_rn(__dsub_rn(fetch_uniform(h, j), C[2 * 32 + j]), C[3 * 32 + j]);
                }
                x[i] = xv;
            }
            float mx = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) mx = fmaxf(mx, fabsf(x[i]));
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            int e = 0;
            (void)frexpf(mx, &e);                         // mx in [2^(e-1), 2^e)
            int sh = 12 - e;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
            const float sc = ldexpf(1.0f, sh);
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] *= sc;
            h8 xh, xl;
            split8(x, xh, xl);
            swrite(slab0 + (cw * 2 + 0) * 64 + lane, xh);
            swrite(slab0 + (cw * 2 + 1) * 64 + lane, xl);
            if (q == 0) colf[cw * 16 + m] = ldexpf(a.winv[0], -sh);
        }
        __syncthreads();                                  // layer-0 input published

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
                bh[c] = sread(slab0 + (c * 2 + 0) * 64 + lane);
                bl[c] = sread(slab0 + (c * 2 + 1) * 64 + lane);
            }
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(a0h[j], bh[c], acc[j][c]);
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(a0h[j], bl[c], acc[j][c]);
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = mfma16(a0l[j], bh[c], acc[j][c]);
        }
        h8 xh[PW][NC], xl[PW][NC];                        // this wave's activations of the current layer
#pragma unroll
        for (int pp = 0; pp < PW; ++pp)
#pragma unroll
            for (int c = 0; c < NC; ++c)
                epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], colf[c * 16 + m], Bl, w * TW + 2 * pp, q,
                         xh[pp][c], xl[pp][c]);

        // ---- hidden layers 1..L-1 [h -> h] through the slab ----
        for (int l = 1; l < L; ++l) {
            // (l == 1: the slab's last readers were the owners' partial sums, before the barrier above)
            if (l > 1) __syncthreads();                   // every wave is done reading the slab
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    swrite(slab + sidx<NC>(w * PW + pp, c, 0, lane), xh[pp][c]);
                    swrite(slab + sidx<NC>(w * PW + pp, c, 1, lane), xl[pp][c]);
                }
            __syncthreads();                              // layer input complete
#pragma unroll
            for (int j = 0; j < TW; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[j][c] = (f4){0.f, 0.f, 0.f, 0.f};
            mm_x3<TW, NC, P>(layer_rsrc(a.w[l], a.wbytes[l]), w * P * TW * 2048, slab, acc, lane);
            const float f = a.winv[l];
#pragma unroll
            for (int pp = 0; pp < PW; ++pp)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    epi_pair(acc[2 * pp][c], acc[2 * pp + 1][c], f, Bl + l * HP, w * TW + 2 * pp, q, xh[pp][c],
                             xl[pp][c]);
        }

        // ---- output layer [h -> S] (2 tiles), K-split: this wave's own k-steps from registers ----
        f4 po[2][NC];
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int c = 0; c < NC; ++c) po[v][c] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int pp = 0; pp < PW; ++pp) {
            const int p = w * PW + pp;
            h8 oh[2], ol[2];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                oh[v] = fload(rso, voff, ((p * 2 + v) * 2 + 0) * 1024);
                ol[v] = fload(rso, voff, ((p * 2 + v) * 2 + 1) * 1024);
            }
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    po[v][c] = mfma16(oh[v], xh[pp][c], po[v][c]);
                    po[v][c] = mfma16(oh[v], xl[pp][c], po[v][c]);
                    po[v][c] = mfma16(ol[v], xh[pp][c], po[v][c]);
                }
        }
        __syncthreads();                                  // every wave is done reading the slab
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int c = 0; c < NC; ++c) slab[((w * 2 + v) * NC + c) * 64 + lane] = po[v][c];
        __syncthreads();                                  // partials complete
        if (!owner) continue;

        f4 o[2];
#pragma unroll
        for (int v = 0; v < 2; ++v) o[v] = slab[((0 * 2 + v) * NC + cw) * 64 + lane];
#pragma unroll
        for (int g = 1; g < NW; ++g)                      // fixed summation order
#pragma unroll
            for (int v = 0; v < 2; ++v) o[v] += slab[((g * 2 + v) * NC + cw) * 64 + lane];

        // ---- cheetah penalties on the current state (cost_functions.py:16-26) ----
        double pen = 0.0;
        if (s[0][1] >= 0.2) pen += 10.0;
        if (s[0][2] >= 0.0) pen += 10.0;
        if (s[0][3] >= 0.0) pen += 10.0;
        pen = __shfl(pen, m + 16);                        // dims 5,6,7 live in lane group q=1
        const double s17 = s[1][1];                       // dim 17 lives in lane group q=0
        // ---- de-normalise + residual (dynamics.py:113,116), f64, no FMA ----
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const f4 bv = *reinterpret_cast<const f4*>(Bout + 16 * v + 4 * q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                if (d < S) {
                    const float dn = fmaf(o[v][r], fo, bv[r]);             // BiasAdd (f32)
                    const double ud = __dadd_rn(__dmul_rn((double)dn, C[5 * 32 + d]), C[4 * 32 + d]);
                    s[v][r] = __dadd_rn(s[v][r], ud);
                }
            }
        }
        if (a.cost == BCMPC_COST_CHEETAH) {
            const double score = __dsub_rn(pen, __ddiv_rn(__dsub_rn(s[1][1], s17), 0.01));
            cost = __dadd_rn(cost, score);
        }
        if (a.traj && valid) {
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * v + 4 * q + r;
                    if (d < S) a.traj[((int64_t)(h + 1) * a.K + cand) * S + d] = s[v][r];
                }
        }
    }
    if (a.costs && valid && q == 0) a.costs[cand] = cost;
}

// ------------------------------------------------------------ launchers ----
template <int HP, int NC, int NW>
static hipError_t launch_x3_t(const RolloutArgs& a, hipStream_t st) {
    if constexpr (NC > NW || x3_lds_bytes<HP, NC, NW>(1) > 160 * 1024) {
        (void)a; (void)st;
        return hipErrorInvalidValue;
    } else {
        static bool attr_set = false;
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)rollout_x3<HP, NC, NW>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
        const size_t lds = (size_t)x3_lds_bytes<HP, NC, NW>(a.L);
        const int64_t blocks = (a.K + 16 * NC - 1) / (16 * NC);
        hipLaunchKernelGGL((rollout_x3<HP, NC, NW>), dim3((unsigned)blocks), dim3(64 * NW), lds, st, a);
        return hipGetLastError();
    }
}

int x3_waves(int hidden_padded) {
    switch (hidden_padded) {
        case 64: return 2;
        case 128: return 4;
        case 256: return 4;
        default: return 8;          // 512, 768, 1024
    }
}

size_t x3_lds(int hidden_padded, int n_layers, int nc) {
    const int P = hidden_padded / 32;
    return (size_t)param_bytes(n_layers, hidden_padded) + nc * 16 * 4 + nc * 2048 + (size_t)(P + 1) * nc * 2048;
}

template <int NC>
static hipError_t launch_x3_nc(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    switch (hidden_padded) {
        case 64: return launch_x3_t<64, NC, 2>(a, st);
        case 128: return launch_x3_t<128, NC, 4>(a, st);
        case 256: return launch_x3_t<256, NC, 4>(a, st);
        case 512: return launch_x3_t<512, NC, 8>(a, st);
        case 768:
            if constexpr (NC <= 2) return launch_x3_t<768, NC, 8>(a, st);
            return hipErrorInvalidValue;
        case 1024:
            if constexpr (NC <= 2) return launch_x3_t<1024, NC, 8>(a, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rollout_x3(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st) {
    switch (nc) {
        case 1: return launch_x3_nc<1>(a, hidden_padded, st);
        case 2: return launch_x3_nc<2>(a, hidden_padded, st);
        case 4: return launch_x3_nc<4>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace bcmpc
