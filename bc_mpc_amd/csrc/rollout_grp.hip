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
constexpr int grp_waves_per_eu(int HP, int NW, int PHP = 0, bool RW = false) {
    return RW ? (NW == 8 ? 4 : 2)                      // reward net: 2 groups/CU (LDS), all resident
         : PHP > 0 ? (NW == 8 ? 4 : HP >= 512 ? 2 : 3)  // fused policy: more live state per wave
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
// dynamics.py:68-69): mean / variance over the true hidden width, across the
// SEGW waves of the wave's LN segment (SEGW = NW: one LayerNorm over the whole
// layer; SEGW = NW/2: the reward net's two heads, each normalised on its own,
// dynamics.py:160,165).  tile0 indexes gamma/beta, ltile0 is the tile index
// inside the segment (pad mask).
template <int TW, int NW, int SEGW = NW>
__device__ __forceinline__ void group_layer_norm(f4 (&v)[TW], int tile0, int ltile0, const float* __restrict__ g,
                                                 const float* __restrict__ bta, int hidden, float* red,
                                                 int w, int lane) {
    const int q = lane >> 4, m = lane & 15;
    const int seg0 = (w / SEGW) * SEGW;
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
    for (int k = 0; k < SEGW; ++k) tot += red[(seg0 + k) * 16 + m];
    const float mean = tot / (float)hidden;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float d = v[j][r] - mean;
            ss += (16 * (ltile0 + j) + 4 * q + r < hidden) ? d * d : 0.f;
        }
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    if (q == 0) red[(NW + w) * 16 + m] = ss;
    __syncthreads();
    float vs = 0.f;
#pragma unroll
    for (int k = 0; k < SEGW; ++k) vs += red[(NW + seg0 + k) * 16 + m];
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

// Layer 0 [S+A -> TW tiles] from registers: x0 holds the two input tiles
// (rows 16v+4q+r); ring holds u-step 0's fragments (prefetched by the caller).
template <int TW>
__device__ __forceinline__ void layer0_mfma(__amdgpu_buffer_rsrc_t rs0, f4 (&ring)[TW], const float (&x0)[2][4],
                                            f4 (&acc)[TW], int w, int lane) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < TW; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[j][r], x0[u][r], acc[j], 0, 0, 0);
        if (u == 0) {
#pragma unroll
            for (int j = 0; j < TW; ++j) ring[j] = wload(rs0, lane * 16, (w * 2 + 1) * TW * 1024 + j * 1024);
        }
    }
}

// Output layer [last hidden -> NOUT tiles], u (K) split over the group.  The
// K-split gives wave w exactly the u-steps of the hidden tiles it produced
// itself ([w*TW, (w+1)*TW)), so its B operands are its own activation
// registers x[] -- the last hidden layer never goes through the slab.  The NW
// partial tiles are then added in fixed wave order through the slab
// (deterministic), leaving the pre-bias result in every wave.  `ring` holds the
// first u-step's fragments (out_prefetch), issued before the epilogue.
template <int NOUT>
__device__ __forceinline__ void out_prefetch(__amdgpu_buffer_rsrc_t rs, f4 (&ring)[NOUT], int u0, int lane) {
#pragma unroll
    for (int k = 0; k < NOUT; ++k) ring[k] = wload(rs, lane * 16, (u0 * NOUT + k) * 1024);
}

template <int TW, int NW, int NOUT>
__device__ __forceinline__ void group_out(__amdgpu_buffer_rsrc_t rs, f4 (&ring)[NOUT], const f4 (&x)[TW],
                                          f4 (&o)[NOUT], f4* slab, int w, int lane) {
    f4 po[NOUT];
#pragma unroll
    for (int k = 0; k < NOUT; ++k) po[k] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        f4 nx[NOUT];
        if (j + 1 < TW) {
#pragma unroll
            for (int k = 0; k < NOUT; ++k) nx[k] = wload(rs, lane * 16, ((w * TW + j + 1) * NOUT + k) * 1024);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < NOUT; ++k)
                po[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[k][r], x[j][r], po[k], 0, 0, 0);
        if (j + 1 < TW) {
#pragma unroll
            for (int k = 0; k < NOUT; ++k) ring[k] = nx[k];
        }
    }
    if constexpr (!GRP_DIAG_NOBAR) __syncthreads();       // every wave is done reading the slab
#pragma unroll
    for (int k = 0; k < NOUT; ++k) slab[(NOUT * w + k) * 64 + lane] = po[k];
    if constexpr (!GRP_DIAG_NOBAR) __syncthreads();
#pragma unroll
    for (int k = 0; k < NOUT; ++k) o[k] = slab[k * 64 + lane];
#pragma unroll
    for (int g = 1; g < NW; ++g)                        // fixed summation order
#pragma unroll
        for (int k = 0; k < NOUT; ++k) o[k] += slab[(NOUT * g + k) * 64 + lane];
}

// One dense stack of the block, all layers fp32 MFMA.  Layer 0 reads its two
// input tiles from registers (x0); hidden layers read the shared slab; each
// wave owns TW = T/NW output tiles; the output layer (NOUT tiles) is K-split
// over the group and its partial tiles are summed in fixed wave order.
// Returns the pre-bias output tiles in every wave (tf.layers.dense adds the
// bias after the matmul; the caller does that in its own precision).
struct StackView {
    const f4* const* w;         // packed layers 0..L (global)
    const int32_t* wbytes;
    const float* bias;          // LDS: [L][HPAD] hidden biases (output bias handled by the caller)
    const float* const* lng;    // LN params (global, per hidden layer)
    const float* const* lnb;
    int L;
    int hidden;                 // true width (LN statistics)
};

template <int T, int NW, int NOUT, int ACT, bool LN>
__device__ __forceinline__ void group_mlp(const StackView& sv, f4 (&ring)[T / NW], const float (&x0)[2][4],
                                          f4 (&o)[NOUT], f4* slab, float* red, int w, int lane) {
    constexpr int TW = T / NW;          // output tiles per wave
    const int q = lane >> 4;
    const int tile0 = w * TW;
    // ---- layer 0 from registers: ring holds u-step 0 (prefetched by the caller) ----
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(sv.w[0], sv.wbytes[0]);
    f4 acc[TW];
#pragma unroll
    for (int j = 0; j < TW; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
    layer0_mfma<TW>(rs0, ring, x0, acc, w, lane);
    const __amdgpu_buffer_rsrc_t rso = layer_rsrc(sv.w[sv.L], sv.wbytes[sv.L]);
    f4 v[TW];
    for (int l = 0; l < sv.L; ++l) {
        if (l > 0) {
            // ---- hidden layer l: [h -> h] from the slab ----
#pragma unroll
            for (int j = 0; j < TW; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
            mm_slab<TW, (TW >= 16 ? 1 : 2)>(layer_rsrc(sv.w[l], sv.wbytes[l]), w * T * TW * 1024, 0, T, slab, acc,
                                           lane);
        }
        // bias + activation (+ LN) in registers
#pragma unroll
        for (int j = 0; j < TW; ++j) v[j] = bias_act<ACT>(acc[j], sv.bias + l * T * 16, tile0 + j, q);
        if constexpr (LN) group_layer_norm<TW, NW>(v, tile0, tile0, sv.lng[l], sv.lnb[l], sv.hidden, red, w, lane);
        if (l + 1 < sv.L) {                             // hand over through the slab
            if constexpr (!GRP_DIAG_NOBAR) __syncthreads();   // every wave is done reading the slab
#pragma unroll
            for (int j = 0; j < TW; ++j) slab[(tile0 + j) * 64 + lane] = v[j];
            if constexpr (!GRP_DIAG_NOBAR) __syncthreads();   // new activations visible
        }
    }
    // ---- output layer: [h -> NOUT tiles] from this wave's own tiles, K-split ----
    f4 oring[NOUT];
    out_prefetch<NOUT>(rso, oring, w * TW, lane);
    group_out<TW, NW, NOUT>(rso, oring, v, o, slab, w, lane);
}

// Reward net of NNDynamicsRewardModel.build_network (dynamics.py:150-177), same
// work split: trunk [S+A -> h] (T tiles) from registers; both heads' hidden
// layers as ONE [h -> 2h] layer (host-concatenated kernels dense_1 | dense_3,
// 2T tiles: waves [0, NW/2) own the delta head, [NW/2, NW) the reward head, each
// half LayerNorm'd on its own); then one block-diagonal [2h -> 32] output layer
// (rows 0..S-1 = dense_2 from the delta half, row S = dense_4 from the reward
// half), K-split over the group and fed from the head registers, so the 2h head
// activations never touch LDS.  Every head neuron is computed exactly once.
template <int T, int NW, bool LN>
__device__ __forceinline__ void group_mlp_rw(const StackView& sv, f4 (&ring)[T / NW], const float (&x0)[2][4],
                                             f4 (&o)[2], f4* slab, float* red, int w, int lane) {
    constexpr int TW = T / NW;          // trunk tiles per wave
    constexpr int TW2 = 2 * T / NW;     // head tiles per wave
    static_assert(NW % 2 == 0 && (2 * T) % NW == 0, "heads must split evenly over the group");
    const int q = lane >> 4;
    const int tile0 = w * TW;
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(sv.w[0], sv.wbytes[0]);
    {
        f4 acc[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
        layer0_mfma<TW>(rs0, ring, x0, acc, w, lane);
        f4 v[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) v[j] = bias_act<BCMPC_ACT_TANH>(acc[j], sv.bias, tile0 + j, q);
        if constexpr (LN) group_layer_norm<TW, NW>(v, tile0, tile0, sv.lng[0], sv.lnb[0], sv.hidden, red, w, lane);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TW; ++j) slab[(tile0 + j) * 64 + lane] = v[j];
        __syncthreads();
    }
    {
        const int htile0 = w * TW2;                     // first head tile of this wave (0..2T)
        f4 acc[TW2];
#pragma unroll
        for (int j = 0; j < TW2; ++j) acc[j] = (f4){0.f, 0.f, 0.f, 0.f};
        mm_slab<TW2, 1>(layer_rsrc(sv.w[1], sv.wbytes[1]), w * T * TW2 * 1024, 0, T, slab, acc,
                                          lane);
        f4 v[TW2];
#pragma unroll
        for (int j = 0; j < TW2; ++j) v[j] = bias_act<BCMPC_ACT_TANH>(acc[j], sv.bias + T * 16, htile0 + j, q);
        const __amdgpu_buffer_rsrc_t rso = layer_rsrc(sv.w[2], sv.wbytes[2]);
        f4 oring[2];
        out_prefetch<2>(rso, oring, htile0, lane);
        if constexpr (LN)
            group_layer_norm<TW2, NW, NW / 2>(v, htile0, htile0 - (w >= NW / 2 ? T : 0), sv.lng[1], sv.lnb[1],
                                              sv.hidden, red, w, lane);
        // ---- block-diagonal output [2h -> S+1] from this wave's own head tiles ----
        group_out<TW2, NW, 2>(rso, oring, v, o, slab, w, lane);
    }
}

template <int T, int NW>
__device__ __forceinline__ void prefetch_layer0(f4 (&ring)[T / NW], const f4* w0, int32_t bytes, int w, int lane) {
    constexpr int TW = T / NW;
    const __amdgpu_buffer_rsrc_t rs0 = layer_rsrc(w0, bytes);
#pragma unroll
    for (int j = 0; j < TW; ++j) ring[j] = wload(rs0, lane * 16, (w * 2 + 0) * TW * 1024 + j * 1024);
}

// Dynamics-net shape facts shared by the kernel and its launcher.
//   RW = false: NNDynamicsModel, L hidden layers of HP, output [HP -> S]
//   RW = true : NNDynamicsRewardModel, trunk HP + heads 2*HP, output [2HP -> S+1]
// bias rows (LB x HP floats, then 32 output-bias floats) and the widest slab layer.
__host__ __device__ constexpr int grp_bias_rows(int L, bool RW) { return RW ? 3 : L; }
__host__ __device__ constexpr int grp_widest_tiles(int HP, int PHP, bool) {
    return (HP > PHP ? HP : PHP) / 16;    // the reward heads (2*HP) stay in registers
}

template <int HP, int ACT, bool LN, int NW, int PHP, bool RW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(grp_waves_per_eu(HP, NW, PHP, RW), 8)))
void rollout_grp(const RolloutArgs a) {
    constexpr int T = HP / 16;          // hidden tiles of the dynamics MLP (reward net: of the trunk)
    constexpr int TW = T / NW;
    constexpr int TP = PHP / 16;        // hidden tiles of the fused policy MLP (0: none)
    constexpr int TPW = (TP > 0 ? TP : NW) / NW;
    constexpr int TMAX = grp_widest_tiles(HP, PHP, RW);
    static_assert(T % NW == 0 && (TP == 0 || TP % NW == 0), "hidden tiles must split evenly over the group");
    static_assert(!RW || ACT == BCMPC_ACT_TANH, "the reward net is tanh (dynamics.py:150)");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;
    const int m = lane & 15;
    const int64_t cand = (int64_t)blockIdx.x * 16 + m;
    const bool valid = cand < a.K;
    const int S = a.S, A = a.A, L = a.L;
    const int LB = grp_bias_rows(L, RW);

    // ---- per-block parameters in LDS: consts (f64), biases, policy params ----
    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    if constexpr (RW) {                                 // [trunk HP][heads 2HP][out 32]
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[i] = a.b[0][i];
        for (int i = threadIdx.x; i < 2 * HP; i += blockDim.x) Bl[HP + i] = a.b[1][i];
    } else {
        for (int l = 0; l < L; ++l)
            for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i];
    }
    float* const Bout = Bl + LB * HP;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bout[i] = a.b[RW ? 2 : L][i];
    float* Pb = Bout + 32;                              // policy: [PL][PHP] hidden biases, then params
    const int PL = a.pL;
    if constexpr (TP > 0) {
        for (int l = 0; l < PL; ++l)
            for (int i = threadIdx.x; i < PHP; i += blockDim.x) Pb[l * PHP + i] = a.pb[l][i];
        for (int i = threadIdx.x; i < kPolParams; i += blockDim.x) Pb[PL * PHP + i] = a.pparams[i];
    }
    f4* slab = reinterpret_cast<f4*>(reinterpret_cast<char*>(lds) + param_bytes(LB, HP) + pol_param_bytes(PL, PHP));
    float* red = reinterpret_cast<float*>(slab + grp_slab_tiles(TMAX, NW) * 64);
    for (int i = threadIdx.x; i < 64; i += blockDim.x) slab[TMAX * 64 + i] = (f4){0.f, 0.f, 0.f, 0.f};
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
            s[v][r] = (valid && d < S) ? (a.state_inline ? a.state_v[d] : a.state[cand * a.state_stride + d]) : 0.0;
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
    // cheetah: trajectory_cost = 0 (cost_functions.py:60); reward: the running
    // np.sum over steps of reward * gamma**i (controllers.py:139,150)
    double cost = 0.0;
    const uint64_t gcand = (uint64_t)(a.cand_offset + cand);
    // uniform draw j of step h: the caller's [H,K,A] array (np.random.uniform, controllers.py:53/191) or Philox
    auto fetch_uniform = [&](int h, int j) -> double {
        if (!valid) return 0.0;
        if (a.cem_mu)                                   // CEM iteration: clip(mu + sigma * z) (DESIGN.md "CEM")
            return cem_action(a.seed, gcand, h, j, a.cem_iter, a.cem_mu[h * A + j], a.cem_sigma[h * A + j],
                              C[6 * 32 + j], C[7 * 32 + j]);
        return a.actions ? a.actions[((int64_t)h * a.K + cand) * A + j]
                         : rng_action(a.seed, gcand, h, j, C[6 * 32 + j], C[7 * 32 + j]);
    };
    const StackView dyn{a.w, a.wbytes, Bl, a.lng, a.lnb, L, a.hidden};
    const StackView pol{a.pw, a.pwbytes, Pb, nullptr, nullptr, PL, PHP};

    for (int h = 0; h < a.H; ++h) {
        double pact[4];                                     // policy actions of rows 16+4q+r (tile 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) pact[r] = 0.0;
        if constexpr (TP > 0) {
            // ---- fused policy (ppo_bc_policy.py:54-88): obz = clip((f32(ob) - mean)/std, -5, 5) ----
            f4 pring[TPW];
            prefetch_layer0<TP, NW>(pring, a.pw[0], a.pwbytes[0], w, lane);
            const float* pm = Pb + PL * PHP;                // [obmean 32][obstd 32][logstd 16][out bias 16]
            float z0[2][4];
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * v + 4 * q + r;
                    float z = 0.f;
                    if (d < S) {
                        z = ((float)s[v][r] - pm[d]) / pm[32 + d];
                        z = fminf(fmaxf(z, -5.0f), 5.0f);
                    }
                    z0[v][r] = z;
                }
            f4 po[1];
            group_mlp<TP, NW, 1, BCMPC_ACT_TANH, false>(pol, pring, z0, po, slab, red, w, lane);
            // action rows i = S + j sit in tile 1 (host permutes the policy output rows there)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 + 4 * q + r;
                const int j = i - S;
                if (j >= 0 && j < A) {
                    const float mean = po[0][r] + pm[80 + (i - 16)];          // dense bias (f32)
                    if (a.pol_mode == BCMPC_POLICY_STOCHASTIC) {
                        const float sd = expf(pm[64 + j]);
                        pact[r] = (double)(mean + sd * rng_normal(a.seed ^ 0x9E3779B97F4A7C15ull, gcand, h, j));
                    } else {
                        // (1 - explore) * mean in f32 (NumPy keeps the f32 dtype), + explore * U in f64
                        const float t1 = (float)(1.0 - a.explore) * mean;
                        pact[r] = __dadd_rn((double)t1, __dmul_rn(a.explore, fetch_uniform(h, j)));
                    }
                }
            }
            if (a.act_out && h < a.act_out_steps && valid && w == 0) {   // action_paths (controllers.py:213)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 + 4 * q + r - S;
                    if (j >= 0 && j < A) a.act_out[((int64_t)h * a.K + cand) * A + j] = pact[r];
                }
            }
        }

        // ---- dynamics: layer-0 weights first (independent of the state) ----
        f4 ring[TW];
        prefetch_layer0<T, NW>(ring, a.w[0], a.wbytes[0], w, lane);
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
                    const double av = (TP > 0 && v == 1) ? pact[r] : fetch_uniform(h, j);
                    xv = (float)__ddiv_rn(__dsub_rn(av, C[2 * 32 + j]), C[3 * 32 + j]);
                }
                x0[v][r] = xv;
            }
        f4 o[2];
        if constexpr (RW) group_mlp_rw<T, NW, LN>(dyn, ring, x0, o, slab, red, w, lane);
        else group_mlp<T, NW, 2, ACT, LN>(dyn, ring, x0, o, slab, red, w, lane);

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
            const f4 bv = *reinterpret_cast<const f4*>(Bout + 16 * v + 4 * q);
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
        if constexpr (RW) {
            // ---- learned reward (dynamics.py:236) * gamma**h, running sum (controllers.py:139,150) ----
            float nr = 0.f;                                // output row S: tile S>>4, lane group (S&15)>>2, reg S&3
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (v == (S >> 4) && r == (S & 3)) nr = o[v][r];
            nr = __shfl(nr, m + 16 * ((S & 15) >> 2)) + Bout[S];
            const double rw = __dadd_rn(__dmul_rn((double)nr, a.std_reward), a.mean_reward);
            cost = __dadd_rn(cost, __dmul_rn(rw, a.gpow[h]));
        } else if (a.cost == BCMPC_COST_CHEETAH) {
            // ---- progress term + trajectory sum (cost_functions.py:28, :59-63) ----
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
template <int HP, int ACT, bool LN, int NW, int PHP, bool RW>
static hipError_t launch_grp_t(const RolloutArgs& a, hipStream_t st) {
    constexpr int TMAX = grp_widest_tiles(HP, PHP, RW);
    const size_t lds = (size_t)param_bytes(grp_bias_rows(a.L, RW), HP) + pol_param_bytes(a.pL, PHP) +
                       (size_t)grp_slab_tiles(TMAX, NW) * 64 * 16 + 2 * NW * 16 * 4 + GRP_LDS_PAD;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)rollout_grp<HP, ACT, LN, NW, PHP, RW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int64_t blocks = (a.K + 15) / 16;
    hipLaunchKernelGGL((rollout_grp<HP, ACT, LN, NW, PHP, RW>), dim3((unsigned)blocks), dim3(64 * NW), lds, st, a);
    return hipGetLastError();
}

template <int HP, int NW, int PHP>
static hipError_t launch_grp_act(const RolloutArgs& a, hipStream_t st) {
    if (a.model == BCMPC_MODEL_REWARD) {               // tanh two-head net (dynamics.py:150-177)
        if constexpr ((NW == 4 || NW == 8) && HP >= 128 && HP <= 512)
            return a.ln ? launch_grp_t<HP, BCMPC_ACT_TANH, true, NW, PHP, true>(a, st)
                        : launch_grp_t<HP, BCMPC_ACT_TANH, false, NW, PHP, true>(a, st);
        return hipErrorInvalidValue;
    }
    if (a.ln) return a.act == BCMPC_ACT_RELU ? launch_grp_t<HP, BCMPC_ACT_RELU, true, NW, PHP, false>(a, st)
                                             : launch_grp_t<HP, BCMPC_ACT_TANH, true, NW, PHP, false>(a, st);
    return a.act == BCMPC_ACT_RELU ? launch_grp_t<HP, BCMPC_ACT_RELU, false, NW, PHP, false>(a, st)
                                   : launch_grp_t<HP, BCMPC_ACT_TANH, false, NW, PHP, false>(a, st);
}

template <int NW>
static hipError_t launch_grp_nw(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    if (a.model == BCMPC_MODEL_REWARD) {               // trunk hidden padded to 128 / 256 / 512
        if constexpr (NW == 4 || NW == 8) {
            if (a.pL > 0 && a.phidden_padded != 128) return hipErrorInvalidValue;
            switch (hidden_padded) {
                case 128: return a.pL > 0 ? launch_grp_act<128, NW, 128>(a, st) : launch_grp_act<128, NW, 0>(a, st);
                case 256: return a.pL > 0 ? launch_grp_act<256, NW, 128>(a, st) : launch_grp_act<256, NW, 0>(a, st);
                case 512: return a.pL > 0 ? launch_grp_act<512, NW, 128>(a, st) : launch_grp_act<512, NW, 0>(a, st);
                default: return hipErrorInvalidValue;
            }
        }
        return hipErrorInvalidValue;
    }
    if (a.pL > 0) {   // fused policy: NW = 4 / 8, policy hidden padded to 128
        if constexpr (NW == 4 || NW == 8) {
            if (a.phidden_padded != 128) return hipErrorInvalidValue;
            switch (hidden_padded) {
                case 128: return launch_grp_act<128, NW, 128>(a, st);
                case 256: return launch_grp_act<256, NW, 128>(a, st);
                case 512: return launch_grp_act<512, NW, 128>(a, st);
                default: return hipErrorInvalidValue;
            }
        }
        return hipErrorInvalidValue;
    }
    switch (hidden_padded) {
        case 64:
            if constexpr (NW <= 4) return launch_grp_act<64, NW, 0>(a, st);
            return hipErrorInvalidValue;
        case 128: return launch_grp_act<128, NW, 0>(a, st);
        case 256: return launch_grp_act<256, NW, 0>(a, st);
        case 512: return launch_grp_act<512, NW, 0>(a, st);
        case 768:
            if constexpr (NW >= 4) return launch_grp_act<768, NW, 0>(a, st);
            return hipErrorInvalidValue;
        case 1024:
            if constexpr (NW >= 4) return launch_grp_act<1024, NW, 0>(a, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

size_t grp_lds_bytes(int hidden_padded, int n_layers, int nw, int policy_hidden_padded, int policy_layers,
                     int model) {
    const bool rw = model == BCMPC_MODEL_REWARD;
    const int tmax = grp_widest_tiles(hidden_padded, policy_hidden_padded, rw);
    return (size_t)param_bytes(grp_bias_rows(n_layers, rw), hidden_padded) +
           pol_param_bytes(policy_layers, policy_hidden_padded) + (size_t)grp_slab_tiles(tmax, nw) * 64 * 16 +
           2 * nw * 16 * 4;
}

hipError_t launch_rollout_grp(const RolloutArgs& a, int hidden_padded, int nw, hipStream_t st) {
    switch (nw) {
        case 4: return launch_grp_nw<4>(a, hidden_padded, st);
        case 8: return launch_grp_nw<8>(a, hidden_padded, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace bcmpc
