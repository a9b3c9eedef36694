// rollout_grp.hip -- "group" rollout kernel: NW waves share 16 candidates.
//
// Same contract and numerics as rollout_fp32 (rollout.hip): one launch is
// one MPCcontroller.get_action (controllers.py:57-88) on this device's
// candidate shard; H serial NNDynamicsModel.predict steps (dynamics.py:
// 106-119) with every dense layer on v_mfma_f32_16x16x4_f32, the f64
// normalise / de-normalise / residual / cheetah cost (cost_functions.py:
// 10-30, 59-63) in registers.
//
// Work split (why): one workgroup = one group of NW waves = 16 candidates.
// Wave w owns output tiles [w*TW, (w+1)*TW) of every hidden layer (TW =
// T/NW) and keeps their accumulators in AGPRs for the whole layer; the layer
// INPUT is one shared LDS slab [tile][lane] read once per u-step by every
// wave (ds_read_b128).  Per-wave registers drop to ~200, so two groups'
// waves share each SIMD: one wave's VALU phase (bias + tanh epilogue, f64
// state update) overlaps the other's MFMA stream.  Two barriers per layer
// hand the new activations over through the slab.  The output layer [h -> S]
// is split over u (K) between the waves; the NW partial tiles are summed in
// fixed wave order through the slab (deterministic; every wave then owns the
// full f64 state update, wave 0 publishes cost / trajectory).
//
// Weights: packed [w][u][j][lane] with TB = TW (capi.cpp pack_layer), so each
// wave walks one contiguous stream; tile j's fragment for u-step u+1 is
// requested right after the four MFMAs that consume u-step u's (>= 4*TW-4
// MFMAs of lead time).  Reads past the layer end return 0 (buffer range
// check).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"

namespace bcmpc {

// waves per SIMD the register allocator must allow: 2-wave groups need ~250
// registers per wave; 4-wave groups fit 128 (4/SIMD) up to HP = 256 and
// ~134 (3/SIMD, spill-free) at HP = 512.
#ifndef GRP_WPE512
#define GRP_WPE512 3
#endif
#ifndef GRP_PRIO
#define GRP_PRIO 0
#endif
#ifndef GRP_STAGGER
#define GRP_STAGGER 0
#endif
#ifndef GRP_DIAG_SMALLW          // timing-only diagnostic: weights from a 16 KiB window (L1-resident)
#define GRP_DIAG_SMALLW 0
#endif
#ifndef GRP_DIAG_NOBAR           // timing-only diagnostic: no group barriers (results wrong)
#define GRP_DIAG_NOBAR 0
#endif
#ifndef GRP_LDS_PAD
#define GRP_LDS_PAD 0
#endif
constexpr int grp_waves_per_eu(int HP, int NW) {
    return NW == 2 ? 2
         : NW == 8 ? (HP >= 768 ? 3 : 4)
         : (HP >= 768 ? 2 : HP >= 512 ? GRP_WPE512 : 4);
}

// acc[j] += sum over u-steps [u0, u1) of W[tile j][u] * slab[u]
template <int TW, int UNR>
__device__ __forceinline__ void mm_slab(__amdgpu_buffer_rsrc_t rs, int wbase, int u0, int u1, const f4* slab,
                                        f4 (&acc)[TW], int lane) {
    constexpr int STEPB = TW * 1024;
    const int voff = lane * 16;
    f4 ring[TW];
#pragma unroll
    for (int j = 0; j < TW; ++j) ring[j] = wload(rs, voff, wbase + u0 * STEPB + j * 1024);
    f4 xc = slab[u0 * 64 + lane];
    if constexpr (GRP_PRIO) __builtin_amdgcn_s_setprio(1);
    for (int u = u0; u < u1; u += UNR) {
#pragma unroll
        for (int uu = 0; uu < UNR; ++uu) {
            const f4 xn = slab[(u + uu + 1) * 64 + lane];        // slab has one spare tile at the end
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < TW; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[j][r], xc[r], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TW; ++j)
                ring[j] = wload(rs, voff, GRP_DIAG_SMALLW ? (((u + uu + 1) * 4 + j) & 15) * 1024
                                                          : wbase + (u + uu + 1) * STEPB + j * 1024);
            xc = xn;
        }
    }
    if constexpr (GRP_PRIO) __builtin_amdgcn_s_setprio(0);
}

// group LayerNorm of the wave's TW activated tiles (tf.contrib.layers.layer_norm,
// dynamics.py:68-69): mean / variance over the true hidden width, across waves.
template <int TW, int NW>
__device__ __forceinline__ void group_layer_norm(f4 (&v)[TW], int tile0, const float* __restrict__ g,
                                                 const float* __restrict__ bta, int hidden, float* red,
                                                 int w, int lane) {
    const int q = lane >> 4, m = lane & 15;
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) sum += v[j][r];           // padded neurons are exactly 0
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    if (q == 0) red[w * 16 + m] = sum;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) tot += red[k * 16 + m];
    const float mean = tot / (float)hidden;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float d = v[j][r] - mean;
            ss += (16 * (tile0 + j) + 4 * q + r < hidden) ? d * d : 0.f;
        }
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    if (q == 0) red[(NW + w) * 16 + m] = ss;
    __syncthreads();
    float vs = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) vs += red[(NW + k) * 16 + m];
    const float rs = 1.0f / sqrtf(vs / (float)hidden + 1e-12f);
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        const f4 gv = *reinterpret_cast<const f4*>(g + 16 * (tile0 + j) + 4 * q);
        const f4 bv = *reinterpret_cast<const f4*>(bta + 16 * (tile0 + j) + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float inv = rs * gv[r];
            v[j][r] = v[j][r] * inv + (bv[r] - mean * inv);    // nn.batch_normalization form
        }
    }
}

// slab tiles: the T activation tiles + one spare (read-ahead) tile, and at least
// the 2*NW partial output tiles of the K-split output layer
__host__ __device__ constexpr int grp_slab_tiles(int T, int NW) { return (T + 1 > 2 * NW) ? T + 1 : 2 * NW; }

template <int HP, int NW>
__host__ __device__ constexpr int grp_slab_bytes() {
    return grp_slab_tiles(HP / 16, NW) * 64 * 16 + 2 * NW * 16 * 4;   // tiles + LN reduction area
}

template <int HP, int ACT, bool LN, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(grp_waves_per_eu(HP, NW), 8)))
void rollout_grp(const RolloutArgs a) {
    constexpr int T = HP / 16;          // hidden tiles
    constexpr int TW = T / NW;          // output tiles per wave
    constexpr int UO = T / NW;          // output-layer u-steps per wave
    static_assert(T % NW == 0, "hidden tiles must split evenly over the group");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;
    const int m = lane & 15;
    const int64_t cand = (int64_t)blockIdx.x * 16 + m;
    const bool valid = cand < a.K;
    const int S = a.S, A = a.A, L = a.L;

    // ---- per-block parameters in LDS: consts (f64) + all biases ----
    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < L; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i];
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bl[L * HP + i] = a.b[L][i];
    f4* slab = reinterpret_cast<f4*>(reinterpret_cast<char*>(lds) + param_bytes(L, HP));
    float* red = reinterpret_cast<float*>(slab + grp_slab_tiles(T, NW) * 64);
    for (int i = threadIdx.x; i < 64; i += blockDim.x) slab[T * 64 + i] = (f4){0.f, 0.f, 0.f, 0.f};
    if constexpr (GRP_STAGGER > 0) {            // de-phase co-resident groups (speed only)
        const int n = (blockIdx.x % 3) * GRP_STAGGER;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }
    __syncthreads();

    double s[2][4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int d = 16 * v + 4 * q + r;
            s[v][r] = (valid && d < S) ? a.state[cand * a.state_stride + d] : 0.0;
        }
    const bool writer = (w == 0) && valid;
    if (a.traj && writer) {
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                if (d < S) a.traj[cand * S + d] = s[v][r];
            }
    }
    double cost = 0.0;   // trajectory_cost = 0 (cost_functions.py:60)
    const uint64_t gcand = (uint64_t)(a.cand_offset + cand);
    auto fetch_action = [&](int h, int i) -> double {
        const int j = i - S;
        if (!valid || i < S || j >= A) return 0.0;
        return a.actions ? a.actions[((int64_t)h * a.K + cand) * A + j]
                         : rng_action(a.seed, gcand, h, j, C[6 * 32 + j], C[7 * 32 + j]);
    };
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(a.w[0], a.wbytes[0]);
    const __amdgpu_buffer_rsrc_t rsL = layer_rsrc(a.w[L], a.wbytes[L]);
    const int voff = lane * 16;
    const int tile0 = w * TW;

    for (int h = 0; h < a.H; ++h) {
        // ---- layer-0 weights of u-step 0 first: they do not depend on the state ----
        f4 ring[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) ring[j] = wload(rs0, voff, (w * 2 + 0) * TW * 1024 + j * 1024);

        // ---- normalise (dynamics.py:109-110), cast to f32 (TF feed) ----
        float x0[2][4];
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * v + 4 * q + r;
                float xv = 0.f;
                if (i < S) {
                    xv = (float)__ddiv_rn(__dsub_rn(s[v][r], C[0 * 32 + i]), C[1 * 32 + i]);
                } else if (i < S + A) {
                    const int j = i - S;
                    xv = (float)__ddiv_rn(__dsub_rn(fetch_action(h, i), C[2 * 32 + j]), C[3 * 32 + j]);
                }
                x0[v][r] = xv;
            }

        // ---- layer 0: [S+A -> h], my TW tiles, two u-steps through the ring ----
        f4 acc[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < TW; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[j][r], x0[u][r], acc[j], 0, 0, 0);
            if (u == 0) {
#pragma unroll
                for (int j = 0; j < TW; ++j) ring[j] = wload(rs0, voff, (w * 2 + 1) * TW * 1024 + j * 1024);
            }
        }
        for (int l = 0; l < L; ++l) {
            if (l > 0) {
                // ---- hidden layer l: [h -> h] from the slab ----
#pragma unroll
                for (int j = 0; j < TW; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
                mm_slab<TW, (TW >= 16 ? 1 : 2)>(layer_rsrc(a.w[l], a.wbytes[l]), w * T * TW * 1024, 0, T, slab, acc, lane);
            }
            // bias + activation (+ LN) in registers, then hand over through the slab
            f4 v[TW];
#pragma unroll
            for (int j = 0; j < TW; ++j) v[j] = bias_act<ACT>(acc[j], Bl + l * HP, tile0 + j, q);
            if constexpr (LN) group_layer_norm<TW, NW>(v, tile0, a.lng[l], a.lnb[l], a.hidden, red, w, lane);
            if constexpr (!GRP_DIAG_NOBAR) __syncthreads();   // every wave is done reading the slab
#pragma unroll
            for (int j = 0; j < TW; ++j) slab[(tile0 + j) * 64 + lane] = v[j];
            if constexpr (!GRP_DIAG_NOBAR) __syncthreads();   // new activations visible
        }

        // ---- output layer: [h -> S], u split over the group ----
        f4 po[2] = {(f4){0.f, 0.f, 0.f, 0.f}, (f4){0.f, 0.f, 0.f, 0.f}};
        mm_slab<2, (UO % 2 == 0) ? 2 : 1>(rsL, 0, w * UO, (w + 1) * UO, slab, po, lane);
        if constexpr (!GRP_DIAG_NOBAR) __syncthreads();       // done reading activations
        slab[(2 * w + 0) * 64 + lane] = po[0];
        slab[(2 * w + 1) * 64 + lane] = po[1];
        if constexpr (!GRP_DIAG_NOBAR) __syncthreads();
        f4 o[2] = {slab[0 * 64 + lane], slab[1 * 64 + lane]};
#pragma unroll
        for (int k = 1; k < NW; ++k) {                // fixed summation order
            o[0] += slab[(2 * k + 0) * 64 + lane];
            o[1] += slab[(2 * k + 1) * 64 + lane];
        }

        // ---- cheetah penalties on the current state (cost_functions.py:16-26) ----
        double pen = 0.0;
        if (s[0][1] >= 0.2) pen += 10.0;
        if (s[0][2] >= 0.0) pen += 10.0;
        if (s[0][3] >= 0.0) pen += 10.0;
        pen = __shfl(pen, m + 16);                    // dims 5,6,7 live in lane group q=1
        const double s17 = s[1][1];                   // dim 17 lives in lane group q=0
        // ---- de-normalise + residual (dynamics.py:113,116), f64, no FMA, in place ----
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const f4 bv = *reinterpret_cast<const f4*>(Bl + L * HP + 16 * v + 4 * q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                if (d < S) {
                    const float dn = o[v][r] + bv[r];                  // BiasAdd (f32)
                    const double ud = __dadd_rn(__dmul_rn((double)dn, C[5 * 32 + d]), C[4 * 32 + d]);
                    s[v][r] = __dadd_rn(s[v][r], ud);
                }
            }
        }
        // ---- progress term + trajectory sum (cost_functions.py:28, :59-63) ----
        if (a.cost == BCMPC_COST_CHEETAH) {
            const double score = __dsub_rn(pen, __ddiv_rn(__dsub_rn(s[1][1], s17), 0.01));
            cost = __dadd_rn(cost, score);
        }
        if (a.traj && writer) {
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * v + 4 * q + r;
                    if (d < S) a.traj[((int64_t)(h + 1) * a.K + cand) * S + d] = s[v][r];
                }
        }
    }
    if (a.costs && writer && q == 0) a.costs[cand] = cost;
}

// ------------------------------------------------------------ launchers ----
template <int HP, int ACT, bool LN, int NW>
static hipError_t launch_grp_t(const RolloutArgs& a, hipStream_t st) {
    const size_t lds = (size_t)param_bytes(a.L, HP) + grp_slab_bytes<HP, NW>() + GRP_LDS_PAD;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)rollout_grp<HP, ACT, LN, NW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int64_t blocks = (a.K + 15) / 16;
    hipLaunchKernelGGL((rollout_grp<HP, ACT, LN, NW>), dim3((unsigned)blocks), dim3(64 * NW), lds, st, a);
    return hipGetLastError();
}

template <int HP, int NW>
static hipError_t launch_grp_act(const RolloutArgs& a, hipStream_t st) {
    if (a.ln) return a.act == BCMPC_ACT_RELU ? launch_grp_t<HP, BCMPC_ACT_RELU, true, NW>(a, st)
                                             : launch_grp_t<HP, BCMPC_ACT_TANH, true, NW>(a, st);
    return a.act == BCMPC_ACT_RELU ? launch_grp_t<HP, BCMPC_ACT_RELU, false, NW>(a, st)
                                   : launch_grp_t<HP, BCMPC_ACT_TANH, false, NW>(a, st);
}

template <int NW>
static hipError_t launch_grp_nw(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    switch (hidden_padded) {
        case 64:
            if constexpr (NW <= 4) return launch_grp_act<64, NW>(a, st);
            return hipErrorInvalidValue;
        case 128: return launch_grp_act<128, NW>(a, st);
        case 256: return launch_grp_act<256, NW>(a, st);
        case 512: return launch_grp_act<512, NW>(a, st);
        case 768:
            if constexpr (NW >= 4) return launch_grp_act<768, NW>(a, st);
            return hipErrorInvalidValue;
        case 1024:
            if constexpr (NW >= 4) return launch_grp_act<1024, NW>(a, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

size_t grp_lds_bytes(int hidden_padded, int n_layers, int nw) {
    const int T = hidden_padded / 16;
    return (size_t)param_bytes(n_layers, hidden_padded) + (size_t)grp_slab_tiles(T, nw) * 64 * 16 + 2 * nw * 16 * 4;
}

hipError_t launch_rollout_grp(const RolloutArgs& a, int hidden_padded, int nw, hipStream_t st) {
    switch (nw) {
        case 2: return launch_grp_nw<2>(a, hidden_padded, st);
        case 4: return launch_grp_nw<4>(a, hidden_padded, st);
        case 8: return launch_grp_nw<8>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace bcmpc
