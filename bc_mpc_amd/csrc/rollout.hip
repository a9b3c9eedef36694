// rollout.hip -- MI355X (gfx950) random-shooting MPC rollout kernels.
//
// One launch == one MPCcontroller.get_action (controllers.py:57-88) on this
// device's shard of the K candidates:
//   * per-candidate state fan-out (np.tile, controllers.py:63) into registers,
//   * H serial steps of NNDynamicsModel.predict (dynamics.py:106-119):
//       f64 normalise -> f32 cast (TF feed, dynamics.py:23-24) ->
//       dense/act[/LayerNorm] x L -> dense (dynamics.py:54-71) ->
//       f64 de-normalise + residual add,
//     with every dense layer on v_mfma_f32_16x16x4_f32 (exact f32 fma chain),
//   * the cheetah cost (cost_functions.py:10-30) accumulated per step in f64
//     registers in the reference's operation order (trajectory_cost_fn :59-63),
//   * np.argmin (controllers.py:82) in a second tiny kernel (first NaN, else
//     first minimum -> lowest index wins ties).
//
// Layout ("transposed" MLP, activations never leave the wave):
//   A wave owns 16 candidates (MFMA column j = lane & 15).  Each dense layer is
//   computed as D[neuron][cand] = W^T[neuron][k] * X[k][cand], weights as the
//   MFMA A operand, activations as the B operand.  The D fragment of a
//   16-neuron tile (lane (q=lane>>4, m) holds neurons 4q+r, r=0..3) is exactly
//   the B fragment of k-steps r=0..3 of the next layer when the weights are
//   pre-packed in that k order on the host -- so the x registers of one layer
//   feed the next with no lane movement.  Outputs of a layer are produced one
//   4-tile block at a time (runtime loop) and parked in a wave-private LDS
//   slab, then re-read into registers for the next layer.
//   State (f64) lives in the lanes that own the matching input/output rows:
//   row/dim d = 16v + 4q + r (v = 0,1).
//
// Weights are streamed from L2 (1 KiB per wave-instruction, float4 per lane,
// fragment order, see pack_layer in capi.cpp); all waves of a CU walk the
// same stream, so it is shared through the CU's L1.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "kernels.h"
#include "device_common.h"
#include "argmin_common.h"

namespace bcmpc {

// Streaming dense layer [TIN tiles in -> TOUT = NB*TB tiles out].  The packed
// weights [tb][u][j][lane] are ONE linear stream of 1-KiB fragments: u-step
// (tb, u) starts at byte (tb*TIN + u) * TB KiB.  A D-deep register ring holds
// the next D u-steps; each refill simply advances the stream position.  With
// EPI, block tb-1's bias+activation runs inside block tb's MFMA stream (VALU
// beside MFMA) and lands in the wave's LDS slab y (block -1 writes to a
// scratch tile past the end, branch-free).  Biases come from LDS (lgkmcnt),
// never through the vmcnt queue the weight ring lives on.
template <int TIN, int TOUT, int TB, int D, int ACT, bool EPI>
__device__ __forceinline__ void layer_stream(__amdgpu_buffer_rsrc_t rs, const float (&x)[TIN][4],
                                             const float* bias, f4* y, f4 (&out)[TB], int lane) {
    constexpr int NB = TOUT / TB;
    static_assert(NB * TB == TOUT, "TOUT must be a multiple of TB");
    // the ring slot of u-step u is u % D in EVERY block, so blocks must span whole ring turns
    static_assert(NB == 1 || TIN % D == 0, "TIN must be a multiple of the prefetch depth D");
    constexpr int STEPB = TB * 1024;              // bytes per u-step
    const int q = lane >> 4;
    const int voff = lane * 16;
    f4 ring[D][TB];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int j = 0; j < TB; ++j) ring[d][j] = wload(rs, voff, d * STEPB + j * 1024);
    f4 prev[TB];
#pragma unroll
    for (int j = 0; j < TB; ++j) prev[j] = (f4){0.f, 0.f, 0.f, 0.f};
    for (int tb = 0; tb < NB; ++tb) {
        const int base = tb * TIN * STEPB;
        const int dst = (tb == 0) ? TOUT : (tb - 1) * TB;         // scratch tile for the pseudo-block -1
        f4 acc[TB];
#pragma unroll
        for (int j = 0; j < TB; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < TIN; ++u) {
            const int slot = u % D;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < TB; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[slot][j][r], x[u][r], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TB; ++j) ring[slot][j] = wload(rs, voff, base + (u + D) * STEPB + j * 1024);
            if constexpr (EPI) {
                // spread the previous block's epilogue over this block's u-steps
                constexpr int GAP = TIN >= TB ? TIN / TB : 1;
#pragma unroll
                for (int e = 0; e < TB; ++e)
                    if ((TIN >= TB) ? (u == e * GAP + GAP / 2) : (u == TIN - 1)) {
                        y[(dst + e) * 64 + lane] = bias_act<ACT>(prev[e], bias, (dst + e) & (TOUT - 1), q);
                    }
            }
        }
#pragma unroll
        for (int j = 0; j < TB; ++j) prev[j] = acc[j];
    }
    if constexpr (EPI) {
        const int dst = (NB - 1) * TB;
#pragma unroll
        for (int e = 0; e < TB; ++e) y[(dst + e) * 64 + lane] = bias_act<ACT>(prev[e], bias, dst + e, q);
    }
#pragma unroll
    for (int j = 0; j < TB; ++j) out[j] = prev[j];
}

// tf.contrib.layers.layer_norm over the true hidden width (dynamics.py:68-69).
template <int T>
__device__ __forceinline__ void layer_norm(float (&x)[T][4], const float* __restrict__ g,
                                           const float* __restrict__ bta, int hidden, int lane) {
    const int q = lane >> 4;
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < T; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) sum += x[u][r];          // padded neurons are exactly 0
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float mean = sum / (float)hidden;
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < T; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float d = x[u][r] - mean;
            ss += (16 * u + 4 * q + r < hidden) ? d * d : 0.f;
        }
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    const float var = ss / (float)hidden;
    const float rs = 1.0f / sqrtf(var + 1e-12f);
#pragma unroll
    for (int u = 0; u < T; ++u) {
        const f4 gv = *reinterpret_cast<const f4*>(g + 16 * u + 4 * q);
        const f4 bv = *reinterpret_cast<const f4*>(bta + 16 * u + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float inv = rs * gv[r];
            x[u][r] = x[u][r] * inv + (bv[r] - mean * inv);   // nn.batch_normalization form
        }
    }
}

template <int T>
__device__ __forceinline__ void reload(float (&x)[T][4], const f4* y, int lane) {
#pragma unroll
    for (int u = 0; u < T; ++u) {
        const f4 v = y[u * 64 + lane];
        x[u][0] = v[0]; x[u][1] = v[1]; x[u][2] = v[2]; x[u][3] = v[3];
    }
}

// ------------------------------------------------------------ the kernel ---
#ifndef BCMPC_D
#define BCMPC_D 2
#endif
template <int HP, int ACT, bool LN>
__global__ __launch_bounds__(256) void rollout_fp32(const RolloutArgs a) {
    constexpr int T = HP / 16;     // hidden tiles
    constexpr int TB = 4;          // output tiles per streamed block (packing granule)
    constexpr int D = BCMPC_D;     // weight prefetch depth, u-steps
    static_assert(T % TB == 0, "hidden tiles must be a multiple of 4");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int q = lane >> 4;
    const int m = lane & 15;
    const int64_t cand = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wave) * 16 + m;
    const bool valid = cand < a.K;
    const int S = a.S, A = a.A, L = a.L;

    // ---- stage per-block parameters in LDS: consts (f64) + all biases ----
    double* C = reinterpret_cast<double*>(lds);                          // [8][32]
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < L; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i];
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bl[L * HP + i] = a.b[L][i];
    __syncthreads();
    f4* y = reinterpret_cast<f4*>(reinterpret_cast<char*>(lds) + param_bytes(L, HP)) + (size_t)wave * (T + TB) * 64;

    // state of candidate `cand`, dims d = 16v + 4q + r
    double s[2][4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int d = 16 * v + 4 * q + r;
            s[v][r] = (valid && d < S) ? (a.state_inline ? a.state_v[d] : a.state[cand * a.state_stride + d]) : 0.0;
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
    double cost = 0.0;   // trajectory_cost = 0 (cost_functions.py:60)
    const uint64_t gcand = (uint64_t)(a.cand_offset + cand);

    // actions of this lane's input rows i = 16v + 4q + r in [S, S+A): fetched
    // one step ahead so the step-start loads never stall the weight stream
    auto fetch_action = [&](int h, int i) -> double {
        const int j = i - S;
        if (!valid || i < S || j >= A) return 0.0;
        return a.actions ? a.actions[((int64_t)h * a.K + cand) * A + j]
                         : rng_action(a.seed, gcand, h, j, C[6 * 32 + j], C[7 * 32 + j]);
    };
    double act_next[2][4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) act_next[v][r] = fetch_action(0, 16 * v + 4 * q + r);

    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(a.w[0], a.wbytes[0]);
    const __amdgpu_buffer_rsrc_t rsL = layer_rsrc(a.w[L], a.wbytes[L]);

    for (int h = 0; h < a.H; ++h) {
        // ---- predict: normalise (dynamics.py:109-110), cast to f32 (TF feed) ----
        double act_cur[2][4];
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) act_cur[v][r] = act_next[v][r];
        if (h + 1 < a.H) {
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) act_next[v][r] = fetch_action(h + 1, 16 * v + 4 * q + r);
        }
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
                    xv = (float)__ddiv_rn(__dsub_rn(act_cur[v][r], C[2 * 32 + j]), C[3 * 32 + j]);
                }
                x0[v][r] = xv;
            }

        // ---- layer 0: [S+A -> h] ----
        float x[T][4];
        {
            f4 unused[TB];
            layer_stream<2, T, TB, 2, ACT, true>(rs0, x0, Bl, y, unused, lane);
            reload<T>(x, y, lane);
            if constexpr (LN) layer_norm<T>(x, a.lng[0], a.lnb[0], a.hidden, lane);
        }
        // ---- hidden layers 1..L-1: [h -> h], streamed, parked in LDS ----
        for (int l = 1; l < L; ++l) {
            f4 unused[TB];
            layer_stream<T, T, TB, D, ACT, true>(layer_rsrc(a.w[l], a.wbytes[l]), x, Bl + l * HP, y, unused, lane);
            reload<T>(x, y, lane);
            if constexpr (LN) layer_norm<T>(x, a.lng[l], a.lnb[l], a.hidden, lane);
        }
        // ---- output layer: [h -> S], no activation (dynamics.py:70) ----
        f4 o[2];
        layer_stream<T, 2, 2, D, ACT, false>(rsL, x, Bl, y, o, lane);

        // ---- de-normalise + residual (dynamics.py:113,116), f64, no FMA ----
        double sn[2][4];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const f4 bv = *reinterpret_cast<const f4*>(Bl + L * HP + 16 * v + 4 * q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                if (d < S) {
                    const float dn = o[v][r] + bv[r];                  // BiasAdd (f32)
                    const double ud = __dadd_rn(__dmul_rn((double)dn, C[5 * 32 + d]), C[4 * 32 + d]);
                    sn[v][r] = __dadd_rn(s[v][r], ud);
                } else {
                    sn[v][r] = 0.0;
                }
            }
        }

        // ---- cheetah cost (cost_functions.py:10-30), accumulated (:59-63) ----
        if (a.cost == BCMPC_COST_CHEETAH) {
            // dims 5,6,7 live in lane group q=1 (v=0, r=1..3); dim 17 in q=0 (v=1, r=1)
            double pen = 0.0;
            if (s[0][1] >= 0.2) pen += 10.0;
            if (s[0][2] >= 0.0) pen += 10.0;
            if (s[0][3] >= 0.0) pen += 10.0;
            pen = __shfl(pen, m + 16);
            const double score = __dsub_rn(pen, __ddiv_rn(__dsub_rn(sn[1][1], s[1][1]), 0.01));
            cost = __dadd_rn(cost, score);
        }
        if (a.traj && valid) {
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * v + 4 * q + r;
                    if (d < S) a.traj[((int64_t)(h + 1) * a.K + cand) * S + d] = sn[v][r];
                }
        }
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[v][r] = sn[v][r];
    }
    if (a.costs && valid && q == 0) a.costs[cand] = cost;
}

// ------------------------------------------------------------ argmin -------
// np.argmin (controllers.py:82) in two short launches: argmin_partial reduces
// contiguous chunks of the cost vector to one (cost, index) record per block,
// argmin_final reduces the records and writes the result (index, cost, first
// action).  better() is a total order (NaN first, then value, then lower index),
// so the grouping cannot change the answer.
__device__ __forceinline__ Best block_best(Best best, double* sc, int64_t* si) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
        if (better(o, best)) best = o;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) { sc[wave] = best.c; si[wave] = best.i; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            const Best o{sc[w], si[w]};
            if (better(o, best)) best = o;
        }
    return best;                                   // valid in thread 0
}

__global__ __launch_bounds__(256) void argmin_partial(const ArgminArgs a) {
    __shared__ double sc[4];
    __shared__ int64_t si[4];
    const int64_t chunk = (a.K + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * chunk;
    const int64_t i1 = i0 + chunk < a.K ? i0 + chunk : a.K;
    Best best{__builtin_inf(), INT64_MAX};
    for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const double v = a.costs[i];
        const Best c{a.maximize ? -v : v, i};      // argmax(x) == argmin(-x), NaN-first and ties alike
        if (better(c, best)) best = c;
    }
    best = block_best(best, sc, si);
    if (threadIdx.x == 0) { a.scratch_c[blockIdx.x] = best.c; a.scratch_i[blockIdx.x] = best.i; }
}

__global__ __launch_bounds__(256) void argmin_final(const ArgminArgs a) {
    __shared__ double sc[4];
    __shared__ int64_t si[4];
    Best best{__builtin_inf(), INT64_MAX};
    for (int b = threadIdx.x; b < a.nparts; b += blockDim.x) {
        const Best c{a.scratch_c[b], a.scratch_i[b]};
        if (better(c, best)) best = c;
    }
    best = block_best(best, sc, si);
    argmin_write_block(a, best, sc, si);
}

// argmin_partial + argmin_final in one block (nparts == 1)
__global__ __launch_bounds__(256) void argmin_single(const ArgminArgs a) {
    __shared__ double sc[4];
    __shared__ int64_t si[4];
    Best best{__builtin_inf(), INT64_MAX};
    for (int64_t i = threadIdx.x; i < a.K; i += blockDim.x) {
        const double v = a.costs[i];
        const Best c{a.maximize ? -v : v, i};
        if (better(c, best)) best = c;
    }
    best = block_best(best, sc, si);
    argmin_write_block(a, best, sc, si);
}

// ------------------------------------------------------------ launchers ----
static size_t slab_bytes(int HP) { return (size_t)(HP / 16 + 4) * 64 * sizeof(f4); }

int max_waves_per_block(int hidden_padded, int n_layers) {
    const size_t budget = 160 * 1024;
    for (int w : {4, 2, 1})
        if ((size_t)param_bytes(n_layers, hidden_padded) + w * slab_bytes(hidden_padded) <= budget) return w;
    return 0;
}

template <int HP, int ACT, bool LN>
static hipError_t launch_hp(const RolloutArgs& a, int waves_per_block, hipStream_t st) {
    const size_t lds = (size_t)param_bytes(a.L, HP) + waves_per_block * slab_bytes(HP);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)rollout_fp32<HP, ACT, LN>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int64_t waves = (a.K + 15) / 16;
    const int64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    hipLaunchKernelGGL((rollout_fp32<HP, ACT, LN>), dim3((unsigned)blocks), dim3(64 * waves_per_block), lds, st, a);
    return hipGetLastError();
}

template <int HP>
static hipError_t launch_act(const RolloutArgs& a, int wpb, hipStream_t st) {
    if (a.ln) return a.act == BCMPC_ACT_RELU ? launch_hp<HP, BCMPC_ACT_RELU, true>(a, wpb, st)
                                             : launch_hp<HP, BCMPC_ACT_TANH, true>(a, wpb, st);
    return a.act == BCMPC_ACT_RELU ? launch_hp<HP, BCMPC_ACT_RELU, false>(a, wpb, st)
                                   : launch_hp<HP, BCMPC_ACT_TANH, false>(a, wpb, st);
}

hipError_t launch_rollout(const RolloutArgs& a, int hidden_padded, int waves_per_block, hipStream_t st) {
    switch (hidden_padded) {
        case 64: return launch_act<64>(a, waves_per_block, st);
        case 128: return launch_act<128>(a, waves_per_block, st);
        case 256: return launch_act<256>(a, waves_per_block, st);
        case 512: return launch_act<512>(a, waves_per_block, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_argmin(const ArgminArgs& a, hipStream_t st) {
    if (a.nparts < 1 || a.nparts > kArgminParts) return hipErrorInvalidValue;
    if (a.nparts == 1) {                           // small K: one block scans and writes (one launch)
        hipLaunchKernelGGL(argmin_single, dim3(1), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(argmin_partial, dim3(a.nparts), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(argmin_final, dim3(1), dim3(256), 0, st, a);
    return hipGetLastError();
}

int argmin_parts(int64_t K) {
    if (K <= 4096) return 1;                       // one block: a launch saved beats the wider scan
    const int64_t p = (K + 511) / 512;             // >= 512 costs per block
    return (int)(p < 1 ? 1 : (p > kArgminParts ? kArgminParts : p));
}

}  // namespace bcmpc
