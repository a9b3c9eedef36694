// fit.hip -- NNDynamicsModel.fit (dynamics.py:81-104) on the GPU: Adam on the
// mean squared error of the normalised state deltas, the reference's TF1 graph
// (dynamics.py:44-52: tf.losses as reduce_mean(squared_difference), AdamOptimizer)
// restated as explicit forward / backward kernels in f32.
//
// One iteration (fit_iteration below), everything resident in HBM:
//   gather   : rows idx[b] of the device-resident data buffer -> normalised f32
//              inputs X0 = [ns, na] and targets T = n_delta (f64 normalise, f32 cast,
//              exactly the numpy -> placeholder path of dynamics.py:92-95)
//   forward  : Z_l = H_l W_l + b_l (gemm), A_l = act(Z_l), H_{l+1} = LN(A_l) or A_l
//              (row kernel: one wave per row, LN statistics over the true width)
//   loss     : L = mean((T - P)^2); dP = -((2 * (1/N)) * (T - P)) (TF's
//              SquaredDifference / Mean gradients, same f32 operation order)
//   backward : dW_l = H_l^T dZ_l, db_l = colsum(dZ_l), dH_l = dZ_l W_l^T (gemm),
//              LN backward (the autodiff of nn.moments + batch_normalization with the
//              stop_gradient on the mean inside the variance), act backward
//              (relu: dz = da [a > 0]; tanh: dz = da (1 - a^2))
//   adam     : TF1 ApplyAdam: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
//              w -= (m lr_t) / (sqrt(v) + eps), lr_t from the f32 beta powers (host)
//
// Shapes are small (batch 512, width <= 1024): the GEMM is a plain LDS-tiled f32
// FMA kernel, the iteration is launch-bound (~20 launches), not FLOP-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"

namespace bcmpc {

// ------------------------------------------------------------------ gemm ---
// C[M][N] = op(A) op(B) (+ bias[N]); op(A) is M x K (TA: A stored [K][M]),
// op(B) is K x N (TB: B stored [N][K]).  32 x 32 tile per 256-thread block,
// 2 x 2 outputs per thread, K staged through LDS 32 at a time; f32 fma.
// Split-K (gridDim.z > 1): block z covers K range [z*kc, (z+1)*kc) and writes its
// partial tile to C + z*M*ldc (scratch); gemm_reduce sums the partials in z order
// (deterministic) and adds the bias.
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32(const float* __restrict__ A, const float* __restrict__ B,
                                                float* __restrict__ C, const float* __restrict__ bias, int M,
                                                int N, int K, int lda, int ldb, int ldc, int kc) {
    __shared__ float As[32][32 + 1];
    __shared__ float Bs[32][32 + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
    const int kb = blockIdx.z * kc, ke = kb + kc < K ? kb + kc : K;
    float acc[2][2] = {};
    for (int k0 = kb; k0 < ke; k0 += 32) {
        for (int i = threadIdx.x; i < 32 * 32; i += 256) {
            const int kk = TA ? i / 32 : i % 32, mm = TA ? i % 32 : i / 32;   // coalesced along memory rows
            const int m = m0 + mm, k = k0 + kk;
            float va = 0.f;
            if (m < M && k < ke) va = TA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k];
            As[kk][mm] = va;
            const int kk2 = TB ? i % 32 : i / 32, nn = TB ? i / 32 : i % 32;
            const int n = n0 + nn, k2 = k0 + kk2;
            float vb = 0.f;
            if (n < N && k2 < ke) vb = TB ? B[(size_t)n * ldb + k2] : B[(size_t)k2 * ldb + n];
            Bs[kk2][nn] = vb;
        }
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
            const float a0 = As[kk][ty * 2], a1 = As[kk][ty * 2 + 1];
            const float b0 = Bs[kk][tx * 2], b1 = Bs[kk][tx * 2 + 1];
            acc[0][0] = __fmaf_rn(a0, b0, acc[0][0]);
            acc[0][1] = __fmaf_rn(a0, b1, acc[0][1]);
            acc[1][0] = __fmaf_rn(a1, b0, acc[1][0]);
            acc[1][1] = __fmaf_rn(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
    float* Cz = C + (size_t)blockIdx.z * M * ldc;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = m0 + ty * 2 + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + tx * 2 + j;
            if (n < N) Cz[(size_t)m * ldc + n] = (bias && gridDim.z == 1) ? acc[i][j] + bias[n] : acc[i][j];
        }
    }
}

// The same contract on the f32 matrix cores: one wave per 32 x 32 tile of C (2 x 2
// v_mfma_f32_16x16x4_f32 tiles), operands straight from global memory (L1/L2-resident at
// these sizes), K in steps of 4 with the next step's fragments in flight.  Fragment layouts:
// A 16x4: lane l holds A[l&15][l>>4]; B 4x16: B[l>>4][l&15]; D 16x16: D[4(l>>4)+r][l&15].
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool TA, bool TB>
__global__ __launch_bounds__(64) void gemm_mfma(const float* __restrict__ A, const float* __restrict__ B,
                                                float* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                int K, int lda, int ldb, int ldc, int kc) {
    const int lane = threadIdx.x;
    const int r16 = lane & 15, k4 = lane >> 4;
    const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
    const int kb = blockIdx.z * kc, ke = kb + kc < K ? kb + kc : K;
    auto lda_ = [&](int m, int k) -> float {
        if (m >= M || k >= ke) return 0.f;
        return TA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k];
    };
    auto ldb_ = [&](int k, int n) -> float {
        if (n >= N || k >= ke) return 0.f;
        return TB ? B[(size_t)n * ldb + k] : B[(size_t)k * ldb + n];
    };
    f4v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};
    // K in chunks of 8 steps (32): the next chunk's 32 fragments are loaded while this one's
    // 32 MFMAs run (one global-load latency per chunk, not per step)
    constexpr int CH = 8;
    float a0[CH], a1[CH], b0[CH], b1[CH];
    auto load = [&](int k) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < CH; ++s) {
            const int kk = k + 4 * s + k4;
            a0[s] = lda_(m0 + r16, kk);
            a1[s] = lda_(m0 + 16 + r16, kk);
            b0[s] = ldb_(kk, n0 + r16);
            b1[s] = ldb_(kk, n0 + 16 + r16);
        }
    };
    load(kb);
    for (int k = kb; k < ke; k += 4 * CH) {
        float c0[CH], c1[CH], d0[CH], d1[CH];
#pragma unroll
        for (int s = 0; s < CH; ++s) { c0[s] = a0[s]; c1[s] = a1[s]; d0[s] = b0[s]; d1[s] = b1[s]; }
        if (k + 4 * CH < ke) load(k + 4 * CH);
#pragma unroll
        for (int s = 0; s < CH; ++s) {
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(c0[s], d0[s], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(c0[s], d1[s], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(c1[s], d0[s], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(c1[s], d1[s], acc[1][1], 0, 0, 0);
        }
    }
    float* Cz = C + (size_t)blockIdx.z * M * ldc;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + 16 * j + r16;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 16 * i + 4 * k4 + r;
                if (m < M) Cz[(size_t)m * ldc + n] = (bias && gridDim.z == 1) ? acc[i][j][r] + bias[n] : acc[i][j][r];
            }
        }
}

#ifndef FIT_MFMA
#define FIT_MFMA 1
#endif

__global__ void gemm_reduce(const float* __restrict__ part, float* __restrict__ C, const float* __restrict__ bias,
                            int M, int N, int ldc, int nz) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int m = i / N, n = i % N;
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += part[(size_t)z * M * ldc + (size_t)m * ldc + n];
    C[(size_t)m * ldc + n] = bias ? s + bias[n] : s;
}

// split K when the output has few tiles and K is long (the weight gradients: K = batch)
template <bool TA, bool TB>
static hipError_t gemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                       int ldb, int ldc, hipStream_t st, float* scratch = nullptr, size_t scratch_floats = 0) {
    const int tiles = ((N + 31) / 32) * ((M + 31) / 32);
    int nz = 1;
    if (scratch)
        while (nz < 8 && tiles * nz < 256 && K / (nz * 2) >= 64 && (size_t)nz * 2 * M * ldc <= scratch_floats) nz *= 2;
    const int kc = ((K + nz - 1) / nz + 31) / 32 * 32;
    dim3 grid((N + 31) / 32, (M + 31) / 32, nz);
    if (FIT_MFMA)
        hipLaunchKernelGGL((gemm_mfma<TA, TB>), grid, dim3(64), 0, st, A, B, nz > 1 ? scratch : C, bias, M, N, K,
                           lda, ldb, ldc, kc);
    else
        hipLaunchKernelGGL((gemm_f32<TA, TB>), grid, dim3(256), 0, st, A, B, nz > 1 ? scratch : C, bias, M, N, K,
                           lda, ldb, ldc, kc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nz == 1) return e;
    hipLaunchKernelGGL(gemm_reduce, dim3((M * N + 255) / 256), dim3(256), 0, st, scratch, C, bias, M, N, ldc, nz);
    return hipGetLastError();
}

// ---------------------------------------------------------------- gather ---
// X0[b] = [(s - mean_obs)/(std_obs+1e-10), (a - mean_act)/(std_act+1e-10)] (f32),
// T[b] = (delta - mean_d)/(std_d+1e-10) (f32); f64 arithmetic as numpy (dynamics.py:73-75, 92-95)
// The batch of iteration *iter is idx_base[iter * stride ...] (stride 0: the caller offset the base),
// so one launch sequence serves every iteration of a graph.
__global__ void fit_gather(const double* __restrict__ st, const double* __restrict__ ac,
                           const double* __restrict__ de, const int64_t* __restrict__ idx_base, int stride,
                           const int32_t* __restrict__ iter, const double* __restrict__ nc,
                           float* __restrict__ X0, float* __restrict__ T, int B, int S, int A) {
    const int IN = S + A;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * (IN + S)) return;
    const int64_t* idx = idx_base + (int64_t)(*iter) * stride;
    const int b = i / (IN + S), c = i % (IN + S);
    const int64_t r = idx[b];
    if (c < S) {
        X0[b * IN + c] = (float)__ddiv_rn(__dsub_rn(st[r * S + c], nc[0 * 32 + c]), nc[1 * 32 + c]);
    } else if (c < IN) {
        const int j = c - S;
        X0[b * IN + c] = (float)__ddiv_rn(__dsub_rn(ac[r * A + j], nc[2 * 32 + j]), nc[3 * 32 + j]);
    } else {
        const int j = c - IN;
        T[b * S + j] = (float)__ddiv_rn(__dsub_rn(de[r * S + j], nc[4 * 32 + j]), nc[5 * 32 + j]);
    }
}

// NNDynamicsRewardModel: R[b] = (reward - mean_r) / (std_r + 1e-10) (f64, then f32: dynamics.py:203,
// :210's [-1, 1] column); nc rows 6 / 7 hold mean_r / std_r + 1e-10
__global__ void fit_gather_reward(const double* __restrict__ rw, const int64_t* __restrict__ idx_base, int stride,
                                  const int32_t* __restrict__ iter, const double* __restrict__ nc,
                                  float* __restrict__ R, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t r = (idx_base + (int64_t)(*iter) * stride)[b];
    R[b] = (float)__ddiv_rn(__dsub_rn(rw[r], nc[6 * 32]), nc[7 * 32]);
}

// dst += src (the trunk's gradient: the sum (AddN) of the two heads' data gradients)
__global__ void fit_add(float* __restrict__ dst, const float* __restrict__ src, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = dst[i] + src[i];
}

// ------------------------------------------------------------ row kernels ---
// one wave per row of width F (<= 1024): act in place Z -> A; with LN, H = LN(A)
// (tf.contrib.layers.layer_norm: nn.moments over the row, batch_normalization
// x*inv + (beta - mean*inv), inv = gamma * rsqrt(var + 1e-12))
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ void fit_act_fwd(float* __restrict__ Z, float* __restrict__ H, float* __restrict__ mean_out,
                            float* __restrict__ rs_out, const float* __restrict__ g, const float* __restrict__ be,
                            int B, int F, int act, int ln) {
    const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= B) return;
    float* z = Z + (size_t)row * F;
    float s = 0.f;
    for (int f = lane; f < F; f += 64) {
        float a = z[f];
        a = act == BCMPC_ACT_RELU ? fmaxf(a, 0.f) : tanhf(a);
        z[f] = a;
        s += a;
    }
    if (!ln) return;
    const float mean = wave_sum(s) / (float)F;
    float ss = 0.f;
    for (int f = lane; f < F; f += 64) {
        const float d = z[f] - mean;
        ss += d * d;
    }
    const float var = wave_sum(ss) / (float)F;
    const float rs = 1.0f / sqrtf(var + 1e-12f);
    float* h = H + (size_t)row * F;
    for (int f = lane; f < F; f += 64) {
        const float inv = rs * g[f];
        h[f] = z[f] * inv + (be[f] - mean * inv);
    }
    if (lane == 0) { mean_out[row] = mean; rs_out[row] = rs; }
}

// dH (in) -> dZ (out, may alias dH): LN backward then act backward, per row.
__global__ void fit_act_bwd(const float* __restrict__ dH, float* __restrict__ dZ, const float* __restrict__ Aact,
                            const float* __restrict__ mean_in, const float* __restrict__ rs_in,
                            const float* __restrict__ g, int B, int F, int act, int ln) {
    const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= B) return;
    const float* dh = dH + (size_t)row * F;
    const float* a = Aact + (size_t)row * F;
    float* dz = dZ + (size_t)row * F;
    float dmean = 0.f, drs = 0.f, mean = 0.f, rs = 0.f;
    if (ln) {
        mean = mean_in[row];
        rs = rs_in[row];
        float s1 = 0.f, s2 = 0.f;
        for (int f = lane; f < F; f += 64) {
            s1 += dh[f] * rs * g[f];                      // d(mean) = -sum dout * inv
            s2 += dh[f] * (a[f] - mean) * g[f];           // d(rs) = sum dout * (x - mean) * gamma
        }
        dmean = -wave_sum(s1);
        drs = wave_sum(s2);
    }
    // d(var) = drs * d rsqrt(var + eps) = drs * (-1/2) rs^3
    const float dvar = -0.5f * drs * rs * rs * rs;
    for (int f = lane; f < F; f += 64) {
        float da = dh[f];
        if (ln) da = dh[f] * rs * g[f] + dmean / (float)F + dvar * 2.0f * (a[f] - mean) / (float)F;
        const float av = a[f];
        dz[f] = act == BCMPC_ACT_RELU ? (av > 0.f ? da : 0.f) : da * (1.0f - av * av);
    }
}

// column sums: out[f] = sum_r X[r][f] (bias grads); with Aact: out2[f] = sum_r X[r][f] * xhat[r][f]
// where xhat = (A - mean_r) rs_r (LN gamma grads; out = beta grads).  Grid = 64-column blocks x RB
// row chunks (enough blocks to fill the chip at batch 512); block = 64 columns x 4 row groups.
// Each block leaves its chunk's partials in part[chunk][F]; the last block of a column block to
// finish (ticket counter) adds the chunks in chunk order: deterministic in one launch.
constexpr int kColChunks = 16;
__global__ __launch_bounds__(256) void fit_colsum(const float* __restrict__ X, float* __restrict__ out, int B, int F,
                                                  const float* __restrict__ Aact, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rs_in, float* __restrict__ out2,
                                                  float* __restrict__ part, unsigned* __restrict__ tickets) {
    __shared__ float p1[4][64], p2[4][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int f = blockIdx.x * 64 + c;
    const int nchunk = gridDim.y, chunk = blockIdx.y;
    const int r0 = (int)(((int64_t)B * chunk) / nchunk), r1 = (int)(((int64_t)B * (chunk + 1)) / nchunk);
    float s = 0.f, s2 = 0.f;
    if (f < F)
        for (int r = r0 + g; r < r1; r += 4) {
            const float x = X[(size_t)r * F + f];
            s += x;
            if (out2) s2 += x * (Aact[(size_t)r * F + f] - mean_in[r]) * rs_in[r];
        }
    p1[g][c] = s;
    p2[g][c] = s2;
    __syncthreads();
    if (g == 0 && f < F) {      // write-through (sc1) partials: no release fence needed
        __hip_atomic_store(&part[(size_t)chunk * 2 * F + f], p1[0][c] + p1[1][c] + p1[2][c] + p1[3][c],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&part[(size_t)chunk * 2 * F + F + f], p2[0][c] + p2[1][c] + p2[2][c] + p2[3][c],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // publish: stores complete, then the ticket (cdna_hip_programming.md "In-launch split-K
    // reduction", sc1 form); correct for any spread of the chunks over XCDs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(&tickets[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p1[0][0] = t == (unsigned)nchunk - 1 ? 1.f : 0.f;     // "last" through the existing LDS array
        if (t == (unsigned)nchunk - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (p1[0][0] == 0.f) return;
    if (g == 0 && f < F) {
        float t = 0.f, t2 = 0.f;
        for (int k = 0; k < nchunk; ++k) {
            t += part[(size_t)k * 2 * F + f];
            t2 += part[(size_t)k * 2 * F + F + f];
        }
        out[f] = t;
        if (out2) out2[f] = t2;
    }
    if (threadIdx.x == 0) tickets[blockIdx.x] = 0;       // ready for the next launch (stream order)
}

// loss = mean((T - P)^2) (one block), dP = -((2 * (1/N)) * (T - P)); tick: this call ends the
// iteration's losses (advances the counter and the beta powers) -- the reward model's reward loss
// runs first with tick = 0, its dynamics loss second
__global__ __launch_bounds__(1024) void fit_loss(const float* __restrict__ P, const float* __restrict__ T,
                                                 float* __restrict__ dP, float* __restrict__ loss_base,
                                                 int32_t* __restrict__ iter, float* __restrict__ bp, float b1,
                                                 float b2, int n, int tick = 1) {
    const int it = *iter;
    float* loss = loss_base + it;
    __shared__ float red[16];
    const float inv = 1.0f / (float)n;
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float d = T[i] - P[i];
        s += d * d;
        dP[i] = -((2.0f * inv) * d);
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        *loss = t * inv;
        if (!tick) return;
        // the previous iteration's end (TF1 _finish: beta powers *= beta), then the counter;
        // the iteration's Adam (after this kernel) reads bp = beta^(it+1)
        if (it > 0) {
            bp[0] = __fmul_rn(bp[0], b1);
            bp[1] = __fmul_rn(bp[1], b2);
        }
        *iter = it + 1;
    }
}

// TF1 ApplyAdam over the flat parameter vector; lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
// in f32 from the device beta powers bp[2] (correctly rounded, as the host expression)
__global__ void fit_adam(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                         const float* __restrict__ g, int64_t n, const float* __restrict__ bp, float lr, float b1,
                         float b2, float eps) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float lr_t = __fdiv_rn(__fmul_rn(lr, __fsqrt_rn(__fsub_rn(1.0f, bp[1]))), __fsub_rn(1.0f, bp[0]));
    const float gi = g[i];
    const float mi = m[i] + (gi - m[i]) * (1.0f - b1);
    const float vi = v[i] + (gi * gi - v[i]) * (1.0f - b2);
    m[i] = mi;
    v[i] = vi;
    w[i] = w[i] - (mi * lr_t) / (sqrtf(vi) + eps);
}


// ------------------------------------------------------------- fused step ---
// One Adam iteration in two launches (BCMPC_FIT_FUSED, default on):
//   fit_rows_kernel   one workgroup per 16 batch rows: gather, every forward layer (MFMA row-tile
//                     GEMM + act + LayerNorm in LDS), output, loss partial, dP, and every backward
//                     data gradient (dH_l = dZ_{l+1} W_{l+1}^T, LN / act backward -> dZ_l), plus the
//                     LayerNorm column partials of its 16 rows -- all row-local given the weights,
//                     so no workgroup waits for another;
//   fit_params_kernel one workgroup per 16 x 16 weight tile (the bias is the tile row k == in, fed
//                     by a column of ones: db = 1^T dZ on the same MFMAs) or per 64 LayerNorm
//                     columns: the batch reduction in a fixed order, then TF1 ApplyAdam in place.
// The kernel boundary is the only global synchronisation of the step.  Every global load after it
// comes from HBM / MALL (the previous launch wrote it on other XCDs), ~1-2 us per dependent trip, so
// the structure minimises dependent trips: all weights of a GEMM are requested before the first
// MFMA needs them, the backward GEMMs read a transposed weight copy (coalesced rows; the params
// kernel keeps it in step), LayerNorm parameters, activations and row statistics stay in LDS.
// Same row arithmetic as the per-op kernels above (fit_act_fwd / fit_act_bwd / fit_loss verbatim);
// only the GEMM and batch-sum orders differ.
constexpr int kFR = 16;                     // batch rows per row-block workgroup (one MFMA row tile)
constexpr int kFW = 16;                     // waves of the row-block workgroup
constexpr int kFK = 8;                      // k-steps (of 4) per weight chunk
constexpr int kFRing = 4;                   // weight chunks in flight per wave
constexpr int kPK = 32;                     // batch steps (of 4) per load batch of a weight-gradient tile

struct FitTile {                            // fit_params_kernel work item (one workgroup)
    int32_t kind;                           // 0: weight tile (+ bias row), 1: LayerNorm columns, 3: loss
    int32_t layer;
    int32_t k0, n0;                         // weight tile origin / first column
};

struct FusedArgs {
    const double* st; const double* ac; const double* de;
    const int64_t* idx_base; int32_t stride; int32_t* iter;
    const double* nc;
    float* w; float* wt; float* m; float* v;            // params, transposed kernel copy, Adam slots
    int32_t w_off[BCMPC_MAX_LAYERS + 1], b_off[BCMPC_MAX_LAYERS + 1];
    int32_t g_off[BCMPC_MAX_LAYERS], be_off[BCMPC_MAX_LAYERS];
    float* x0; float* t; float* p; float* dp;
    float* act; float* hln;                             // [L][Bmax][h]
    float* dzs;                                         // [L][Bmax][h]
    float* lnpart;                                      // [L][nblk][2][h] LayerNorm column partials
    float* loss_part; float* loss; float* bp;
    const FitTile* tiles; int32_t ntiles;
    int32_t B, Bmax, S, A, IN, L, h, act_kind, ln, ldw;
    float lr, b1, b2, eps;
};

// one chunk of kFK k-steps of the B operand through a buffer descriptor: one 32-bit lane offset
// (vo) for the whole GEMM, the chunk position in the scalar offset; rows past the matrix and the
// masked columns (vo beyond the range) read 0
__device__ __forceinline__ void rows_load(float* b, __amdgpu_buffer_rsrc_t rsrc, int vo, int kb, int kstride) {
#pragma unroll
    for (int s = 0; s < kFK; ++s)
        b[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, vo, (kb + 4 * s) * kstride, 0));
}

__device__ __forceinline__ f4v rows_mma(f4v acc, const float* b, const float* X, int kb, int K, int r16, int k4,
                                        int lds) {
#pragma unroll
    for (int s = 0; s < kFK; ++s) {
        const int k = kb + 4 * s + k4;
        const float x = k < K ? X[r16 * lds + k] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x, b[s], acc, 0, 0, 0);
    }
    return acc;
}

// Every weight load of a GEMM has been consumed by its end, but the compiler's wait analysis cannot
// see it through the conditional prefetches and keeps them "pending": the row phase after the GEMM
// then gets vmcnt(0) waits at register reuse -- which also wait for that phase's own global stores,
// a full HBM write trip (~2 us) per phase.  A real s_waitcnt vmcnt(0) here (nothing is in flight by
// then) clears the analysis.
__device__ __forceinline__ void rows_drained() {
    __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0), expcnt / lgkmcnt untouched (gfx9 encoding)
}

// acc += sum over k in [k0, k1) of X[r][k] W[k*ldw + n] for this lane's column n (a 16-wide tile),
// kFRing chunks of weights in flight
__device__ __forceinline__ f4v rows_tile(f4v acc, const float* X, int k0, int k1, __amdgpu_buffer_rsrc_t rsrc,
                                         int vo, int ldw, int r16, int k4, int lds) {
    constexpr int CK = 4 * kFK;
    float ring[kFRing][kFK];
#pragma unroll
    for (int j = 0; j < kFRing; ++j)
        if (k0 + j * CK < k1) rows_load(ring[j], rsrc, vo, k0 + j * CK, 4 * ldw);
    for (int kb = k0; kb < k1; kb += kFRing * CK) {
#pragma unroll
        for (int j = 0; j < kFRing; ++j) {
            const int kc = kb + j * CK;
            if (kc < k1) {
                acc = rows_mma(acc, ring[j], X, kc, k1, r16, k4, lds);
                if (kc + kFRing * CK < k1) rows_load(ring[j], rsrc, vo, kc + kFRing * CK, 4 * ldw);
            }
        }
    }
    return acc;
}

// C[r][n] = sum_k X[r][k] W[k*ldw + n] (+ bias[n]) for the 16 LDS rows X (stride lds), n < N, W row-major
// [K][ldw].  16-column tiles over the 16 waves; when there are fewer tiles than waves (the [h -> S]
// output layer) the K range is split over the idle waves and the partials (LDS, `kp`) are added in
// wave order.
__device__ __forceinline__ void rows_gemm(const float* X, int K, const float* __restrict__ W, int ldw, int N,
                          const float* __restrict__ bias, float* C, int lds, float* kp) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r16 = lane & 15, k4 = lane >> 4;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W), 0, K * ldw * 4, 0x00020000);
    const int nt = (N + 15) / 16;
    if (nt * 2 > kFW) {
        for (int n0 = 16 * wv; n0 < N; n0 += 16 * kFW) {
            const int n = n0 + r16;
            const int vo = n < N ? (k4 * ldw + n) * 4 : 0x40000000;
            const float bv = bias && n < N ? bias[n] : 0.f;          // requested before the weights
            f4v acc = rows_tile((f4v){0.f, 0.f, 0.f, 0.f}, X, 0, K, rsrc, vo, ldw, r16, k4, lds);
            rows_drained();
            if (n < N)
#pragma unroll
                for (int r = 0; r < 4; ++r) C[(4 * k4 + r) * lds + n] = bias ? acc[r] + bv : acc[r];
        }
        return;
    }
    // K split: wave wv takes tile wv % nt, K slice wv / nt of ks (whole 4-k-steps)
    const int ks = kFW / nt;
    const int t = wv % nt, q = wv / nt;
    const int n = 16 * t + r16;
    if (q < ks) {
        const int kq = ((K + 4 * ks - 1) / (4 * ks)) * 4;       // slice length, multiple of 4
        const int k0 = min(K, q * kq), k1 = min(K, k0 + kq);
        const int vo = n < N ? (k4 * ldw + n) * 4 : 0x40000000;
        f4v acc = (f4v){0.f, 0.f, 0.f, 0.f};
        if (k0 < k1) acc = rows_tile(acc, X, k0, k1, rsrc, vo, ldw, r16, k4, lds);
        rows_drained();
#pragma unroll
        for (int r = 0; r < 4; ++r) kp[(q * nt + t) * 256 + (4 * k4 + r) * 16 + r16] = acc[r];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 16 * nt * 16; i += 64 * kFW) {
        const int tt = i / 256, e = i % 256, r = e / 16, c = 16 * tt + e % 16;
        if (c < N) {
            float s = 0.f;
            for (int qq = 0; qq < ks; ++qq) s += kp[(qq * nt + tt) * 256 + e];
            C[r * lds + c] = bias ? s + bias[c] : s;
        }
    }
}

// wave sum without the LDS crossbar: DPP butterflies inside each 16-lane row (quad_perm xor 1, xor 2,
// row_ror 4, 8), then the four row totals in a fixed order (deterministic, wave-uniform)
template <int CTRL>
__device__ __forceinline__ float dpp_t(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_fast(float v) {
    v += dpp_t<0xB1>(v);                    // quad_perm [1,0,3,2]
    v += dpp_t<0x4E>(v);                    // quad_perm [2,3,0,1]
    v += dpp_t<0x124>(v);                   // row_ror 4
    v += dpp_t<0x128>(v);                   // row_ror 8
    const int b = __builtin_bit_cast(int, v);
    return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
           (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

__device__ __forceinline__ float adam_elem(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                           size_t i, float gi, float w0, float m0, float v0, float lr_t, float b1,
                                           float b2, float eps) {
    const float mi = m0 + (gi - m0) * (1.0f - b1);
    const float vi = v0 + (gi * gi - v0) * (1.0f - b2);
    const float wi = w0 - (mi * lr_t) / (sqrtf(vi) + eps);
    m[i] = mi;
    v[i] = vi;
    w[i] = wi;
    return wi;
}

__global__ __launch_bounds__(1024) void fit_rows_kernel(const FusedArgs a) {
    extern __shared__ float sm[];
    const int ld = a.ldw, S = a.S, IN = a.IN, L = a.L, h = a.h;
    float* bufA = sm;                       // [16][ld]: the current layer input / backward operand
    float* bufB = bufA + kFR * ld;          // [16][ld]: GEMM output
    float* bufC = bufB + kFR * ld;          // [16][ld]: dH * xhat (LayerNorm backward)
    float* tsm = bufC + kFR * ld;           // [16][32] targets
    float* red = tsm + kFR * 32;            // [kFW] loss partials per wave
    float* kp = red + kFW;                  // [kFW][256] K-split partials
    float* stat = kp + kFW * 256;           // [L][2][16] row mean / rs
    float* prm = stat + L * 2 * kFR;        // [L][2][h] LayerNorm gamma, beta (LN nets)
                                            // (every pointer the row phases read is LDS: no flat
                                            //  loads, whose waits would include the pending stores)
    float* acache = prm + 2 * L * h;        // [L][16][ld] activation rows A_l
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r0 = blockIdx.x * kFR;
    const int nr = min(kFR, a.B - r0);
    const int it = *a.iter;
    const int64_t* idx = a.idx_base + (int64_t)it * a.stride;
#ifdef BCMPC_FIT_STAMPS     // timing-only build: phase boundaries of workgroup 0, printed for iteration 5
    uint64_t stamps[40];
    int nst = 0;
    stamps[nst++] = __builtin_amdgcn_s_memrealtime();
#define FIT_STAMP() do { if (nst < 40) stamps[nst++] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define FIT_STAMP() do { } while (0)
#endif
    if (blockIdx.x == 0 && tid == 0 && it > 0) {          // (fit_loss: the previous iteration's finish)
        a.bp[0] = __fmul_rn(a.bp[0], a.b1);
        a.bp[1] = __fmul_rn(a.bp[1], a.b2);
    }
    // ---- gather (fit_gather), LayerNorm parameters into LDS ----
    if (a.ln)
        for (int i = tid; i < 2 * L * h; i += 64 * kFW) {
            const int l = i / (2 * h), j = i % (2 * h);
            prm[i] = j < h ? a.w[a.g_off[l] + j] : a.w[a.be_off[l] + j - h];
        }
    const double* nc = a.nc;
    for (int i = tid; i < kFR * (IN + S); i += 64 * kFW) {
        const int r = i / (IN + S), c = i % (IN + S);
        float val = 0.f;
        if (r < nr) {
            const int64_t row = idx[r0 + r];
            if (c < S) val = (float)__ddiv_rn(__dsub_rn(a.st[row * S + c], nc[0 * 32 + c]), nc[1 * 32 + c]);
            else if (c < IN) val = (float)__ddiv_rn(__dsub_rn(a.ac[row * a.A + c - S], nc[2 * 32 + c - S]), nc[3 * 32 + c - S]);
            else val = (float)__ddiv_rn(__dsub_rn(a.de[row * S + c - IN], nc[4 * 32 + c - IN]), nc[5 * 32 + c - IN]);
        }
        if (c < IN) {
            bufA[r * ld + c] = val;
            if (r < nr) a.x0[(size_t)(r0 + r) * IN + c] = val;
        } else {
            tsm[r * 32 + c - IN] = val;
            if (r < nr) a.t[(size_t)(r0 + r) * S + c - IN] = val;
        }
    }
    __syncthreads();
    FIT_STAMP();
    const size_t BH = (size_t)a.Bmax * h;
    // ---- forward (fit_act_fwd per row: one row per wave) ----
    for (int l = 0; l < L; ++l) {
        rows_gemm(bufA, l == 0 ? IN : h, a.w + a.w_off[l], h, h, a.w + a.b_off[l], bufB, ld, kp);
        __syncthreads();
        FIT_STAMP();
        {
            const int r = wv;
            float* z = bufB + r * ld;
            float* hx = bufA + r * ld;
            float* ac = acache + (l * kFR + r) * ld;
            const size_t go = (size_t)l * BH + (size_t)(r0 + r) * h;
            float s = 0.f;
#pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                float v = z[f];
                v = a.act_kind == BCMPC_ACT_RELU ? fmaxf(v, 0.f) : tanhf(v);
                z[f] = v;
                s += v;
                ac[f] = v;
                if (r < nr) a.act[go + f] = v;
            }
            if (!a.ln) {
                for (int f = lane; f < h; f += 64) hx[f] = z[f];
            } else {
                const float mean = wave_sum_fast(s) / (float)h;
                float ss = 0.f;
    #pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                    const float d = z[f] - mean;
                    ss += d * d;
                }
                const float var = wave_sum_fast(ss) / (float)h;
                const float rs = 1.0f / sqrtf(var + 1e-12f);
                const float* g = prm + 2 * l * h;
                const float* be = prm + 2 * l * h + h;
    #pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                    const float inv = rs * g[f];
                    const float hv = z[f] * inv + (be[f] - mean * inv);
                    hx[f] = hv;
                    if (r < nr) a.hln[go + f] = hv;
                }
                if (lane == 0) {
                    stat[(l * 2 + 0) * kFR + r] = mean;
                    stat[(l * 2 + 1) * kFR + r] = rs;
                }
            }
        }
        __syncthreads();
        FIT_STAMP();
    }
    // ---- output, loss partial, dP = -((2 * (1/N)) * (T - P)) (fit_loss) ----
    rows_gemm(bufA, h, a.w + a.w_off[L], S, S, a.w + a.b_off[L], bufB, ld, kp);
    __syncthreads();
    FIT_STAMP();
    const float inv = 1.0f / (float)(a.B * S);
    float sl = 0.f;
    for (int i = tid; i < kFR * S; i += 64 * kFW) {
        const int r = i / S, c = i % S;
        float g = 0.f;
        if (r < nr) {
            const float pv = bufB[r * ld + c];
            const float d = tsm[r * 32 + c] - pv;
            sl += d * d;
            g = -((2.0f * inv) * d);
            a.p[(size_t)(r0 + r) * S + c] = pv;
            a.dp[(size_t)(r0 + r) * S + c] = g;
        }
        bufA[r * ld + c] = g;
    }
    sl = wave_sum_fast(sl);
    if (lane == 0) red[wv] = sl;
    __syncthreads();
    FIT_STAMP();
    if (tid == 0) {
        float t = 0.f;
        for (int w = 0; w < kFW; ++w) t += red[w];
        a.loss_part[blockIdx.x] = t;
    }
    // ---- backward data gradients (fit_act_bwd per row), LayerNorm column partials ----
    const int nblk = (a.B + kFR - 1) / kFR;
    for (int l = L - 1; l >= 0; --l) {
        const int out = l + 1 == L ? S : h;                 // dZ_{l+1} width; W_{l+1}^T is [out][h]
        rows_gemm(bufA, out, a.wt + a.w_off[l + 1], h, h, nullptr, bufB, ld, kp);
        __syncthreads();
        FIT_STAMP();
        {
            const int r = wv;
            float* dh = bufB + r * ld;
            float* dz = bufA + r * ld;
            float* gx = bufC + r * ld;
            const size_t go = (size_t)l * BH + (size_t)(r0 + r) * h;
            if (r >= nr) {
    #pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                    dz[f] = 0.f;
                    dh[f] = 0.f;
                    gx[f] = 0.f;
                }
            } else {
                const float* av = acache + (l * kFR + r) * ld;
                const float* g = prm + 2 * l * h;
                float dmean = 0.f, drs = 0.f, mean = 0.f, rs = 0.f;
                if (a.ln) {
                    mean = stat[(l * 2 + 0) * kFR + r];
                    rs = stat[(l * 2 + 1) * kFR + r];
                    float s1 = 0.f, s2 = 0.f;
        #pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                        s1 += dh[f] * rs * g[f];
                        s2 += dh[f] * (av[f] - mean) * g[f];
                    }
                    dmean = -wave_sum_fast(s1);
                    drs = wave_sum_fast(s2);
                }
                const float dvar = -0.5f * drs * rs * rs * rs;
    #pragma unroll 4
            for (int f = lane; f < h; f += 64) {
                    float da = dh[f];
                    const float avv = av[f];
                    if (a.ln) {
                        da = dh[f] * rs * g[f] + dmean / (float)h + dvar * 2.0f * (avv - mean) / (float)h;
                        gx[f] = dh[f] * (avv - mean) * rs;            // (fit_colsum's gamma term)
                    }
                    const float dzv = a.act_kind == BCMPC_ACT_RELU ? (avv > 0.f ? da : 0.f) : da * (1.0f - avv * avv);
                    a.dzs[go + f] = dzv;
                    dz[f] = dzv;
                }
            }
        }
        __syncthreads();
        FIT_STAMP();
        if (a.ln) {                                       // this block's 16-row column sums, rows in order
            for (int f = tid; f < h; f += 64 * kFW) {
                float sb = 0.f, sg = 0.f;
                for (int r = 0; r < kFR; ++r) {
                    sb += bufB[r * ld + f];
                    sg += bufC[r * ld + f];
                }
                float* lp = a.lnpart + ((size_t)(l * nblk + blockIdx.x) * 2) * h;
                lp[f] = sb;
                lp[h + f] = sg;
            }
            __syncthreads();                              // (bufB is the next GEMM's output)
        }
    }
#ifdef BCMPC_FIT_STAMPS
    if (blockIdx.x == 0 && tid == 0 && it == 5) {
        for (int k = 1; k < nst; ++k) printf("stamp %d %.2f us\n", k, (double)(stamps[k] - stamps[0]) * 0.01);
    }
#endif
#undef FIT_STAMP
}

// one workgroup per task; its 4 waves take contiguous quarters of the batch (of the row blocks for
// LayerNorm columns) and their partials are added in wave order (deterministic)
__global__ __launch_bounds__(256) void fit_params_kernel(const FusedArgs a) {
    __shared__ float part[4][2][64];        // column-sum partials per wave
    __shared__ float tp[4][4][64];          // weight-tile partials per wave
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int B = a.B, S = a.S, IN = a.IN, L = a.L, h = a.h;
    const size_t BH = (size_t)a.Bmax * h;
    const FitTile tl = a.tiles[blockIdx.x];
    const int l = tl.layer;
    if (tl.kind == 3) {
        // the loss (fixed row-block order) and the iteration counter (fit_loss)
        if (threadIdx.x == 0) {
            const int it = *a.iter;
            float tot = 0.f;
            for (int k = 0; k < (B + kFR - 1) / kFR; ++k) tot += a.loss_part[k];
            a.loss[it] = tot * (1.0f / (float)(B * S));
            *a.iter = it + 1;
        }
        return;
    }
    const float lr_t = __fdiv_rn(__fmul_rn(a.lr, __fsqrt_rn(__fsub_rn(1.0f, a.bp[1]))), __fsub_rn(1.0f, a.bp[0]));
    if (tl.kind == 0) {
        // dW_l[k][n] = sum_b Hin[b][k] dZ[b][n], row k == in of the tile: the bias (Hin = 1)
        // (A = Hin^T: lane (k = r16, b = k4); B = dZ: (b = k4, n = r16))
        const int in = l == 0 ? IN : h, out = l == L ? S : h;
        const float* Hin = l == 0 ? a.x0 : (a.ln ? a.hln : a.act) + (size_t)(l - 1) * BH;
        const float* dZ = l == L ? a.dp : a.dzs + (size_t)l * BH;
        const int r16 = lane & 15, k4 = lane >> 4;
        const int k = tl.k0 + r16, n = tl.n0 + r16;
        // this lane's Adam operands (wave 0 updates), requested with the gradient operands
        float w0[4], m0[4], v0[4];
        size_t pi[4];
        if (wv == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int kk = tl.k0 + 4 * k4 + r;
                pi[r] = kk < in ? (size_t)a.w_off[l] + (size_t)kk * out + n : (size_t)a.b_off[l] + n;
                const bool ok = kk <= in && n < out;
                w0[r] = ok ? a.w[pi[r]] : 0.f;
                m0[r] = ok ? a.m[pi[r]] : 0.f;
                v0[r] = ok ? a.v[pi[r]] : 0.f;
            }
        const int q0 = (B * wv) / 4, q1 = (B * (wv + 1)) / 4;
        f4v acc = (f4v){0.f, 0.f, 0.f, 0.f};
        for (int bb = q0; bb < q1; bb += 4 * kPK) {
            float x[kPK], y[kPK];
#pragma unroll
            for (int s = 0; s < kPK; ++s) {
                const int b = bb + 4 * s + k4;
                x[s] = b < q1 ? (k < in ? Hin[(size_t)b * in + k] : (k == in ? 1.f : 0.f)) : 0.f;
                y[s] = (b < q1 && n < out) ? dZ[(size_t)b * out + n] : 0.f;
            }
#pragma unroll
            for (int s = 0; s < kPK; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], y[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) tp[wv][r][lane] = acc[r];
        __syncthreads();
        if (wv == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float gsum = ((tp[0][r][lane] + tp[1][r][lane]) + tp[2][r][lane]) + tp[3][r][lane];
                const int kk = tl.k0 + 4 * k4 + r;
                if (kk <= in && n < out) {
                    const float wn = adam_elem(a.w, a.m, a.v, pi[r], gsum, w0[r], m0[r], v0[r], lr_t, a.b1, a.b2, a.eps);
                    if (kk < in && l > 0) a.wt[(size_t)a.w_off[l] + (size_t)n * in + kk] = wn;   // W^T copy
                }
            }
        }
        return;
    }
    // LayerNorm columns: beta = colsum dH, gamma = colsum dH xhat over the row blocks' partials
    const int nblk = (B + kFR - 1) / kFR;
    const int q0 = (nblk * wv) / 4, q1 = (nblk * (wv + 1)) / 4;
    const int n = tl.n0 + lane;
    const bool ok = n < h;
    const size_t ib = (size_t)a.be_off[l] + n, ig = (size_t)a.g_off[l] + n;
    float wb = 0.f, mb = 0.f, vb = 0.f, wg = 0.f, mg = 0.f, vg = 0.f;
    if (wv == 0 && ok) {
        wb = a.w[ib]; mb = a.m[ib]; vb = a.v[ib];
        wg = a.w[ig]; mg = a.m[ig]; vg = a.v[ig];
    }
    float s1 = 0.f, s2 = 0.f;
    if (ok)
        for (int k = q0; k < q1; ++k) {
            const float* lp = a.lnpart + ((size_t)(l * nblk + k) * 2) * h;
            s1 += lp[n];
            s2 += lp[h + n];
        }
    part[wv][0][lane] = s1;
    part[wv][1][lane] = s2;
    __syncthreads();
    if (wv != 0 || !ok) return;
    const float t1 = ((part[0][0][lane] + part[1][0][lane]) + part[2][0][lane]) + part[3][0][lane];
    const float t2 = ((part[0][1][lane] + part[1][1][lane]) + part[2][1][lane]) + part[3][1][lane];
    adam_elem(a.w, a.m, a.v, ib, t1, wb, mb, vb, lr_t, a.b1, a.b2, a.eps);
    adam_elem(a.w, a.m, a.v, ig, t2, wg, mg, vg, lr_t, a.b1, a.b2, a.eps);
}

}  // namespace bcmpc

using namespace bcmpc;

// ------------------------------------------------------------------ C ABI ---
namespace {
thread_local std::string g_fit_error;
int ffail(int code, const std::string& msg) {
    g_fit_error = msg;
    return code;
}
}  // namespace

struct bcmpc_fitter {
    bcmpc_fit_config cfg{};
    hipStream_t stream = nullptr;
    int IN = 0, L = 0, h = 0, S = 0, A = 0, Bmax = 0;
    // flat parameters: per layer W_l [in][out], b_l [out]; then per hidden layer gamma, beta [h]
    std::vector<size_t> w_off, b_off, g_off, be_off;
    std::vector<int> lin, lout;                   // per dense layer: in / out width
    size_t n_params = 0;
    float *d_w = nullptr, *d_m = nullptr, *d_v = nullptr, *d_g = nullptr;
    // activations: X0 [B][IN], per hidden layer Z/A [B][h] and H (LN out) [B][h], mean/rs [B]; P/T/dP [B][S]
    float *d_x0 = nullptr, *d_t = nullptr, *d_p = nullptr, *d_dp = nullptr, *d_act = nullptr, *d_hln = nullptr;
    float *d_mean = nullptr, *d_rs = nullptr, *d_dh = nullptr, *d_dz = nullptr;
    float* d_loss = nullptr; int32_t loss_cap = 0;  // [iterations] losses of the last run
    float* d_split = nullptr; size_t split_floats = 0;  // split-K partials of the weight gradients
    double *d_st = nullptr, *d_ac = nullptr, *d_de = nullptr, *d_nc = nullptr;
    int64_t n_data = 0, data_cap = 0;
    int64_t* d_idx = nullptr; int64_t idx_cap = 0;
    float beta1_power = 0.f, beta2_power = 0.f;   // TF1 Adam accumulators (f32 variables), host mirror
    int32_t* d_iter = nullptr;                    // iteration counter of the running fit (device)
    float* d_bp = nullptr;                        // [beta1_power, beta2_power] (device)
    float* d_cpart = nullptr;                     // column-sum chunk partials [kColChunks][2][max width]
    unsigned* d_tickets = nullptr;                // column-sum completion tickets (one per 64 columns)
    // one captured graph of a whole uniform-batch run, reused while its shape and buffers match
    hipGraphExec_t graph = nullptr;
    int32_t graph_iters = 0, graph_b = 0;
    const void* graph_idx = nullptr;
    const void* graph_loss = nullptr;
    int64_t step = 0;
    bool has_weights = false;
    // the fused two-launch iteration (fit_rows_kernel + fit_params_kernel)
    bool fused = false;
    float *d_wt = nullptr;                        // transposed kernels (layers >= 1), kept by the Adam tiles
    float *d_dzs = nullptr, *d_lnpart = nullptr, *d_lpart = nullptr;   // [L][B][h], [L][nblk][2][h], [nblk]
    FitTile* d_tiles = nullptr;
    int32_t ntiles = 0, rows_ld = 0;
    size_t rows_lds = 0;
    // NNDynamicsRewardModel (cfg.model == BCMPC_MODEL_REWARD): parameters dense .. dense_4 (w/b_off[0..4]),
    // LayerNorm trunk / delta / reward (g/be_off[0..2]); activation slots 0 trunk, 1 delta head, 2 reward head
    bool rw = false;
    float *d_r = nullptr, *d_pr = nullptr, *d_dpr = nullptr, *d_dh2 = nullptr, *d_loss2 = nullptr;
    double* d_rwd = nullptr;                      // the buffer's rewards [n]
    int64_t rw_cap = 0;
    bool has_rewards = false;
    int32_t last_iters = 0;                       // iterations of the last run (its reward losses in d_loss2)
};

extern "C" {

const char* bcmpc_fit_last_error(void) { return g_fit_error.c_str(); }

int bcmpc_fit_create(const bcmpc_fit_config* c, bcmpc_fitter** out) {
    if (!c || !out) return ffail(BCMPC_ERR_ARG, "null argument");
    *out = nullptr;
    if (c->state_dim < 1 || c->state_dim > BCMPC_MAX_STATE || c->action_dim < 1 ||
        c->state_dim + c->action_dim > BCMPC_MAX_INPUT)
        return ffail(BCMPC_ERR_UNSUPPORTED, "state_dim / action_dim out of range");
    if (c->n_layers < 1 || c->n_layers > BCMPC_MAX_LAYERS || c->hidden < 1 || c->hidden > 1024)
        return ffail(BCMPC_ERR_UNSUPPORTED, "n_layers must be in [1, 8], hidden in [1, 1024]");
    if (c->activation != BCMPC_ACT_TANH && c->activation != BCMPC_ACT_RELU)
        return ffail(BCMPC_ERR_UNSUPPORTED, "activation must be tanh or relu");
    if (c->batch_size < 1) return ffail(BCMPC_ERR_ARG, "batch_size must be >= 1");
    if (c->model != BCMPC_MODEL_DELTA && c->model != BCMPC_MODEL_REWARD) return ffail(BCMPC_ERR_ARG, "unknown model");
    const bool rw = c->model == BCMPC_MODEL_REWARD;
    if (rw && (c->n_layers != 2 || c->activation != BCMPC_ACT_TANH))
        return ffail(BCMPC_ERR_UNSUPPORTED, "reward model: n_layers 2 (trunk + heads), tanh (dynamics.py:150-177)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || c->device < 0 || c->device >= ndev)
        return ffail(BCMPC_ERR_ARG, "device ordinal out of range");
    if (hipSetDevice(c->device) != hipSuccess) return ffail(BCMPC_ERR_HIP, "hipSetDevice failed");
    bcmpc_fitter* f = new bcmpc_fitter();
    f->cfg = *c;
    f->S = c->state_dim; f->A = c->action_dim; f->IN = f->S + f->A; f->L = c->n_layers; f->h = c->hidden;
    f->Bmax = c->batch_size;
    f->rw = rw;
    size_t off = 0;
    const int nk = rw ? 5 : f->L + 1, nln = rw ? 3 : f->L;
    for (int l = 0; l < nk; ++l) {
        int in = l == 0 ? f->IN : f->h, o = l == f->L ? f->S : f->h;
        if (rw) {                                         // dense, dense_1, dense_2, dense_3, dense_4
            const int ro[5] = {f->h, f->h, f->S, f->h, 1};
            o = ro[l];
        }
        f->w_off.push_back(off); off += (size_t)in * o;
        f->b_off.push_back(off); off += o;
        f->lin.push_back(in);
        f->lout.push_back(o);
    }
    for (int l = 0; l < nln; ++l) {
        f->g_off.push_back(off); off += f->h;
        f->be_off.push_back(off); off += f->h;
    }
    f->n_params = off;
    const size_t B = (size_t)f->Bmax, H = (size_t)f->h, L = (size_t)nln;   // (activation slots)
    auto al = [&](void** p, size_t bytes) { return hipMalloc(p, bytes > 0 ? bytes : 4) == hipSuccess; };
    bool ok = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) == hipSuccess &&
              al((void**)&f->d_w, off * 4) && al((void**)&f->d_m, off * 4) && al((void**)&f->d_v, off * 4) &&
              al((void**)&f->d_g, off * 4) && al((void**)&f->d_x0, B * f->IN * 4) && al((void**)&f->d_t, B * f->S * 4) &&
              al((void**)&f->d_p, B * f->S * 4) && al((void**)&f->d_dp, B * f->S * 4) &&
              al((void**)&f->d_act, L * B * H * 4) && al((void**)&f->d_hln, L * B * H * 4) &&
              al((void**)&f->d_mean, L * B * 4) && al((void**)&f->d_rs, L * B * 4) && al((void**)&f->d_dh, B * H * 4) &&
              al((void**)&f->d_dz, B * H * 4) &&
              al((void**)&f->d_split, (f->split_floats = 8 * (size_t)std::max(f->IN, f->h) * std::max(f->h, f->S)) * 4) &&
              al((void**)&f->d_nc, kConstRows * kConstCols * 8) && al((void**)&f->d_iter, 4) &&
              al((void**)&f->d_bp, 8) &&
              al((void**)&f->d_cpart, (size_t)kColChunks * 2 * std::max(f->h, f->S) * 4) &&
              al((void**)&f->d_tickets, 64 * 4) &&
              (!rw || (al((void**)&f->d_r, B * 4) && al((void**)&f->d_pr, B * 4) && al((void**)&f->d_dpr, B * 4) &&
                       al((void**)&f->d_dh2, B * H * 4)));
    if (!ok) { bcmpc_fit_destroy(f); return ffail(BCMPC_ERR_HIP, "device allocation failed"); }
    const char* fe = std::getenv("BCMPC_FIT_FUSED");
    f->fused = !(fe && fe[0] == '0') && !rw;          // (the reward model: the per-op kernels, one graph)
    if (f->fused) {
        // LDS of fit_rows_kernel: bufA/B/C, targets, loss partials, K-split partials, row statistics,
        // then (when it fits) LayerNorm parameters and every hidden layer's activation rows
        const int wmax = std::max(f->h, std::max(f->IN, f->S));
        f->rows_ld = (wmax + 3) / 4 * 4 + 4;
        const size_t base = (size_t)3 * kFR * f->rows_ld + kFR * 32 + kFW + kFW * 256 + 2 * kFR * f->L;
        const size_t cache = (size_t)2 * f->L * f->h + (size_t)f->L * kFR * f->rows_ld;
        constexpr size_t kLdsMax = 160 * 1024 / 4;
        f->rows_lds = (base + cache) * 4;
        f->fused = base + cache <= kLdsMax;               // (otherwise the per-op kernels)
    }
    if (f->fused) {
        std::vector<FitTile> tl;
        for (int l = 0; l <= f->L; ++l) {                 // weight tiles incl. the bias row k == in
            const int in = l == 0 ? f->IN : f->h, o = l == f->L ? f->S : f->h;
            for (int k0 = 0; k0 <= in; k0 += 16)
                for (int n0 = 0; n0 < o; n0 += 16) tl.push_back({0, l, k0, n0});
        }
        if (c->layer_norm)
            for (int l = 0; l < f->L; ++l)
                for (int n0 = 0; n0 < f->h; n0 += 64) tl.push_back({1, l, 0, n0});
        tl.push_back({3, 0, 0, 0});                       // loss + iteration counter
        f->ntiles = (int32_t)tl.size();
        const size_t nblk = (B + kFR - 1) / kFR;
        ok = al((void**)&f->d_wt, off * 4) && al((void**)&f->d_dzs, L * B * H * 4) &&
             al((void**)&f->d_lnpart, L * nblk * 2 * H * 4) && al((void**)&f->d_lpart, nblk * 4) &&
             al((void**)&f->d_tiles, tl.size() * sizeof(FitTile)) &&
             hipMemcpy(f->d_tiles, tl.data(), tl.size() * sizeof(FitTile), hipMemcpyHostToDevice) == hipSuccess &&
             (f->rows_lds <= 65536 ||
              hipFuncSetAttribute((const void*)fit_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)f->rows_lds) == hipSuccess);
        if (!ok) { bcmpc_fit_destroy(f); return ffail(BCMPC_ERR_HIP, "fused-step allocation failed"); }
    }
    (void)hipMemset(f->d_m, 0, off * 4);
    (void)hipMemset(f->d_v, 0, off * 4);
    (void)hipMemset(f->d_g, 0, off * 4);
    (void)hipMemset(f->d_tickets, 0, 64 * 4);     // (the LN slots of a net without LayerNorm stay 0: no update)
    f->beta1_power = c->beta1;
    f->beta2_power = c->beta2;
    *out = f;
    return BCMPC_OK;
}

int bcmpc_fit_destroy(bcmpc_fitter* f) {
    if (!f) return BCMPC_OK;
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    if (f->graph) (void)hipGraphExecDestroy(f->graph);
    for (void* p : {(void*)f->d_iter, (void*)f->d_bp, (void*)f->d_cpart, (void*)f->d_tickets, (void*)f->d_w, (void*)f->d_m, (void*)f->d_v, (void*)f->d_g, (void*)f->d_x0, (void*)f->d_t,
                    (void*)f->d_p, (void*)f->d_dp, (void*)f->d_act, (void*)f->d_hln, (void*)f->d_mean,
                    (void*)f->d_rs, (void*)f->d_dh, (void*)f->d_dz, (void*)f->d_loss, (void*)f->d_st,
                    (void*)f->d_ac, (void*)f->d_de, (void*)f->d_nc, (void*)f->d_idx, (void*)f->d_split,
                    (void*)f->d_wt, (void*)f->d_dzs, (void*)f->d_lnpart, (void*)f->d_lpart, (void*)f->d_tiles,
                    (void*)f->d_r, (void*)f->d_pr, (void*)f->d_dpr, (void*)f->d_dh2, (void*)f->d_loss2, (void*)f->d_rwd})
        if (p) (void)hipFree(p);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
    return BCMPC_OK;
}

int bcmpc_fit_set_params(bcmpc_fitter* f, const bcmpc_weights* w) {
    if (!f || !w || !w->kernels || !w->biases) return ffail(BCMPC_ERR_ARG, "null argument");
    if (f->cfg.layer_norm && (!w->ln_gamma || !w->ln_beta)) return ffail(BCMPC_ERR_ARG, "LayerNorm params missing");
    if (!w->mean_obs || !w->std_obs || !w->mean_action || !w->std_action || !w->mean_deltas || !w->std_deltas)
        return ffail(BCMPC_ERR_ARG, "normalization stats missing");
    if (f->rw && (!w->mean_reward || !w->std_reward)) return ffail(BCMPC_ERR_ARG, "mean_reward / std_reward missing");
    std::vector<float> hw(f->n_params, 0.f);
    const int nk = (int)f->w_off.size(), nln = (int)f->g_off.size();
    for (int l = 0; l < nk; ++l) {
        const size_t in = f->lin[l], o = f->lout[l];
        if (!w->kernels[l] || !w->biases[l]) return ffail(BCMPC_ERR_ARG, "null kernel / bias");
        std::copy(w->kernels[l], w->kernels[l] + in * o, hw.begin() + f->w_off[l]);
        std::copy(w->biases[l], w->biases[l] + o, hw.begin() + f->b_off[l]);
    }
    for (int l = 0; l < nln; ++l) {
        for (int i = 0; i < f->h; ++i) {
            hw[f->g_off[l] + i] = f->cfg.layer_norm ? w->ln_gamma[l][i] : 1.f;
            hw[f->be_off[l] + i] = f->cfg.layer_norm ? w->ln_beta[l][i] : 0.f;
        }
    }
    double nc[kConstRows * kConstCols] = {};
    for (int i = 0; i < kConstCols; ++i) {        // dynamics.py:73-75 normalize(x, std, mean) = (x - mean) / (std + 1e-10)
        nc[0 * 32 + i] = i < f->S ? w->mean_obs[i] : 0.0;
        nc[1 * 32 + i] = i < f->S ? w->std_obs[i] + 1e-10 : 1.0;
        nc[2 * 32 + i] = i < f->A ? w->mean_action[i] : 0.0;
        nc[3 * 32 + i] = i < f->A ? w->std_action[i] + 1e-10 : 1.0;
        nc[4 * 32 + i] = i < f->S ? w->mean_deltas[i] : 0.0;
        nc[5 * 32 + i] = i < f->S ? w->std_deltas[i] + 1e-10 : 1.0;
    }
    if (f->rw) {                                      // dynamics.py:203 normalize(reward, std_reward, mean_reward)
        nc[6 * 32] = w->mean_reward[0];
        nc[7 * 32] = w->std_reward[0] + 1e-10;
    }
    std::vector<float> hwt;
    if (f->fused) {                                   // W_l^T [out][in] at the same offsets (fit_rows_kernel)
        hwt.assign(f->n_params, 0.f);
        for (int l = 1; l <= f->L; ++l) {
            const int in = f->h, o = l == f->L ? f->S : f->h;
            for (int i = 0; i < in; ++i)
                for (int j = 0; j < o; ++j) hwt[f->w_off[l] + (size_t)j * in + i] = hw[f->w_off[l] + (size_t)i * o + j];
        }
    }
    if (hipSetDevice(f->cfg.device) != hipSuccess ||
        hipMemcpyAsync(f->d_w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
        (f->fused && hipMemcpyAsync(f->d_wt, hwt.data(), hwt.size() * 4, hipMemcpyHostToDevice, f->stream) != hipSuccess) ||
        hipMemcpyAsync(f->d_nc, nc, sizeof(nc), hipMemcpyHostToDevice, f->stream) != hipSuccess ||
        hipStreamSynchronize(f->stream) != hipSuccess)
        return ffail(BCMPC_ERR_HIP, "parameter upload failed");
    f->has_weights = true;
    return BCMPC_OK;
}

int bcmpc_fit_get_params(bcmpc_fitter* f, float* const* kernels, float* const* biases, float* const* ln_gamma,
                         float* const* ln_beta) {
    if (!f || !kernels || !biases) return ffail(BCMPC_ERR_ARG, "null argument");
    std::vector<float> hw(f->n_params);
    if (hipSetDevice(f->cfg.device) != hipSuccess ||
        hipMemcpyAsync(hw.data(), f->d_w, hw.size() * 4, hipMemcpyDeviceToHost, f->stream) != hipSuccess ||
        hipStreamSynchronize(f->stream) != hipSuccess)
        return ffail(BCMPC_ERR_HIP, "parameter download failed");
    const int nk = (int)f->w_off.size(), nln = (int)f->g_off.size();
    for (int l = 0; l < nk; ++l) {
        std::copy(hw.begin() + f->w_off[l], hw.begin() + f->w_off[l] + (size_t)f->lin[l] * f->lout[l], kernels[l]);
        std::copy(hw.begin() + f->b_off[l], hw.begin() + f->b_off[l] + f->lout[l], biases[l]);
    }
    if (f->cfg.layer_norm && ln_gamma && ln_beta)
        for (int l = 0; l < nln; ++l) {
            std::copy(hw.begin() + f->g_off[l], hw.begin() + f->g_off[l] + f->h, ln_gamma[l]);
            std::copy(hw.begin() + f->be_off[l], hw.begin() + f->be_off[l] + f->h, ln_beta[l]);
        }
    return BCMPC_OK;
}

int bcmpc_fit_set_data(bcmpc_fitter* f, const double* states, const double* actions, const double* deltas,
                       int64_t n) {
    if (!f || (n > 0 && (!states || !actions || !deltas)) || n < 0) return ffail(BCMPC_ERR_ARG, "bad argument");
    if (hipSetDevice(f->cfg.device) != hipSuccess) return ffail(BCMPC_ERR_HIP, "hipSetDevice failed");
    if (n > f->data_cap) {
        for (double** p : {&f->d_st, &f->d_ac, &f->d_de})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
        f->data_cap = 0;
        if (hipMalloc(&f->d_st, (size_t)n * f->S * 8) != hipSuccess ||
            hipMalloc(&f->d_ac, (size_t)n * f->A * 8) != hipSuccess ||
            hipMalloc(&f->d_de, (size_t)n * f->S * 8) != hipSuccess)
            return ffail(BCMPC_ERR_HIP, "data buffer allocation failed");
        f->data_cap = n;
    }
    if (n > 0 &&
        (hipMemcpyAsync(f->d_st, states, (size_t)n * f->S * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
         hipMemcpyAsync(f->d_ac, actions, (size_t)n * f->A * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
         hipMemcpyAsync(f->d_de, deltas, (size_t)n * f->S * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
         hipStreamSynchronize(f->stream) != hipSuccess))
        return ffail(BCMPC_ERR_HIP, "data upload failed");
    f->n_data = n;
    return BCMPC_OK;
}

// fused iteration: 2 launches (see fit_rows_kernel / fit_params_kernel)
static int fit_iteration_fused(bcmpc_fitter* f, const int64_t* d_idx, int stride, int B, float* d_loss) {
    FusedArgs a{};
    a.st = f->d_st; a.ac = f->d_ac; a.de = f->d_de;
    a.idx_base = d_idx; a.stride = stride; a.iter = f->d_iter; a.nc = f->d_nc;
    a.w = f->d_w; a.wt = f->d_wt; a.m = f->d_m; a.v = f->d_v;
    for (int l = 0; l <= f->L; ++l) { a.w_off[l] = (int32_t)f->w_off[l]; a.b_off[l] = (int32_t)f->b_off[l]; }
    for (int l = 0; l < f->L; ++l) { a.g_off[l] = (int32_t)f->g_off[l]; a.be_off[l] = (int32_t)f->be_off[l]; }
    a.x0 = f->d_x0; a.t = f->d_t; a.p = f->d_p; a.dp = f->d_dp;
    a.act = f->d_act; a.hln = f->d_hln;
    a.dzs = f->d_dzs; a.lnpart = f->d_lnpart;
    a.loss_part = f->d_lpart; a.loss = d_loss; a.bp = f->d_bp;
    a.tiles = f->d_tiles; a.ntiles = f->ntiles;
    a.B = B; a.Bmax = f->Bmax; a.S = f->S; a.A = f->A; a.IN = f->IN; a.L = f->L; a.h = f->h;
    a.act_kind = f->cfg.activation; a.ln = f->cfg.layer_norm ? 1 : 0; a.ldw = f->rows_ld;
    a.lr = f->cfg.learning_rate; a.b1 = f->cfg.beta1; a.b2 = f->cfg.beta2; a.eps = f->cfg.epsilon;
    hipLaunchKernelGGL(fit_rows_kernel, dim3((B + kFR - 1) / kFR), dim3(64 * kFW), f->rows_lds, f->stream, a);
    if (hipGetLastError() != hipSuccess) return ffail(BCMPC_ERR_HIP, "fit_rows_kernel launch failed");
    hipLaunchKernelGGL(fit_params_kernel, dim3(f->ntiles), dim3(256), 0, f->stream, a);
    if (hipGetLastError() != hipSuccess) return ffail(BCMPC_ERR_HIP, "fit_params_kernel launch failed");
    return BCMPC_OK;
}

// NNDynamicsRewardModel (dynamics.py:153-160, 195-219): loss_dynamic + loss_reward over the two-head net
// (dynamics.py:165-177), the same per-op kernels as the delta net; the run is one captured graph
//   forward : Z0 = X0 W0 + b0 -> tanh (+LN) = H0; per head: Z = H0 W + b -> tanh (+LN) = Hd / Hr;
//             Pd = Hd W2 + b2 [B][S], Pr = Hr W4 + b4 [B][1]
//   losses  : reward (tick 0, d_loss2) then dynamics (tick 1: ends the iteration)
//   backward: per head (output grads, dH = dP Wo^T, LN / tanh backward, head weight grads, its data
//             gradient into the trunk); dH0 = the delta head's + the reward head's (AddN); trunk
//   adam    : every parameter
static int fit_iteration_reward(bcmpc_fitter* f, const int64_t* d_idx, int stride, int B, float* d_loss) {
    hipStream_t st = f->stream;
    const int S = f->S, IN = f->IN, h = f->h, act = BCMPC_ACT_TANH, ln = f->cfg.layer_norm;
    const size_t BH = (size_t)f->Bmax * h;
    float* W = f->d_w;
    float* G = f->d_g;
#define FIT_TRY(x) do { if ((x) != hipSuccess) return ffail(BCMPC_ERR_HIP, #x); } while (0)
    const int ng = B * (IN + S);
    hipLaunchKernelGGL(fit_gather, dim3((ng + 255) / 256), dim3(256), 0, st, f->d_st, f->d_ac, f->d_de, d_idx,
                       stride, f->d_iter, f->d_nc, f->d_x0, f->d_t, B, S, f->A);
    FIT_TRY(hipGetLastError());
    hipLaunchKernelGGL(fit_gather_reward, dim3((B + 255) / 256), dim3(256), 0, st, f->d_rwd, d_idx, stride,
                       f->d_iter, f->d_nc, f->d_r, B);
    FIT_TRY(hipGetLastError());
    const dim3 rows((B + 3) / 4), rthreads(256);
    auto slot_a = [&](int s) { return f->d_act + (size_t)s * BH; };
    auto slot_h = [&](int s) { return ln ? f->d_hln + (size_t)s * BH : f->d_act + (size_t)s * BH; };
    auto mean_of = [&](int s) { return f->d_mean + (size_t)s * f->Bmax; };
    auto rs_of = [&](int s) { return f->d_rs + (size_t)s * f->Bmax; };
    // ---- forward: trunk (slot 0, dense / LayerNorm), heads (slot 1: dense_1 / LayerNorm_1, slot 2: dense_3 /
    //      LayerNorm_2) ----
    auto hidden_layer = [&](const float* Hin, int in, int l, int s) -> int {
        FIT_TRY((gemm<false, false>(Hin, W + f->w_off[l], slot_a(s), W + f->b_off[l], B, h, in, in, h, h, st)));
        hipLaunchKernelGGL(fit_act_fwd, rows, rthreads, 0, st, slot_a(s), f->d_hln + (size_t)s * BH, mean_of(s),
                           rs_of(s), W + f->g_off[s], W + f->be_off[s], B, h, act, ln);
        FIT_TRY(hipGetLastError());
        return BCMPC_OK;
    };
    if (int rc = hidden_layer(f->d_x0, IN, 0, 0)) return rc;
    if (int rc = hidden_layer(slot_h(0), h, 1, 1)) return rc;
    if (int rc = hidden_layer(slot_h(0), h, 3, 2)) return rc;
    FIT_TRY((gemm<false, false>(slot_h(1), W + f->w_off[2], f->d_p, W + f->b_off[2], B, S, h, h, S, S, st)));
    FIT_TRY((gemm<false, false>(slot_h(2), W + f->w_off[4], f->d_pr, W + f->b_off[4], B, 1, h, h, 1, 1, st)));
    hipLaunchKernelGGL(fit_loss, dim3(1), dim3(1024), 0, st, f->d_pr, f->d_r, f->d_dpr, f->d_loss2, f->d_iter, f->d_bp,
                       f->cfg.beta1, f->cfg.beta2, B, 0);
    FIT_TRY(hipGetLastError());
    hipLaunchKernelGGL(fit_loss, dim3(1), dim3(1024), 0, st, f->d_p, f->d_t, f->d_dp, d_loss, f->d_iter, f->d_bp,
                       f->cfg.beta1, f->cfg.beta2, B * S, 1);
    FIT_TRY(hipGetLastError());
    // ---- backward ----
    const int nch = std::max(1, std::min(kColChunks, B / 32));
    // one head: its output layer lo (width o, dP) and hidden layer lh on activation slot s; its data
    // gradient w.r.t. the trunk's output goes to dH0 (d_dh or d_dh2)
    auto head = [&](int lo, int o, const float* dP, int lh, int s, float* dH0) -> int {
        FIT_TRY((gemm<true, false>(slot_h(s), dP, G + f->w_off[lo], nullptr, h, o, B, h, o, o, st, f->d_split,
                                   f->split_floats)));
        hipLaunchKernelGGL(fit_colsum, dim3((o + 63) / 64, nch), dim3(256), 0, st, dP, G + f->b_off[lo], B, o, nullptr,
                           nullptr, nullptr, nullptr, f->d_cpart, f->d_tickets);
        FIT_TRY(hipGetLastError());
        FIT_TRY((gemm<false, true>(dP, W + f->w_off[lo], f->d_dh, nullptr, B, h, o, o, o, h, st)));
        if (ln)
            hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dh, G + f->be_off[s], B, h,
                               slot_a(s), mean_of(s), rs_of(s), G + f->g_off[s], f->d_cpart, f->d_tickets);
        hipLaunchKernelGGL(fit_act_bwd, rows, rthreads, 0, st, f->d_dh, f->d_dz, slot_a(s), mean_of(s), rs_of(s),
                           W + f->g_off[s], B, h, act, ln);
        FIT_TRY(hipGetLastError());
        FIT_TRY((gemm<true, false>(slot_h(0), f->d_dz, G + f->w_off[lh], nullptr, h, h, B, h, h, h, st, f->d_split,
                                   f->split_floats)));
        hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dz, G + f->b_off[lh], B, h,
                           nullptr, nullptr, nullptr, nullptr, f->d_cpart, f->d_tickets);
        FIT_TRY(hipGetLastError());
        FIT_TRY((gemm<false, true>(f->d_dz, W + f->w_off[lh], dH0, nullptr, B, h, h, h, h, h, st)));
        return BCMPC_OK;
    };
    if (int rc = head(2, S, f->d_dp, 1, 1, f->d_dh2)) return rc;     // delta head -> d_dh2
    // reward head -> d_dh: free once the head's own fit_act_bwd has consumed it (its last GEMM reads d_dz as
    // the A operand, so the result must not land in d_dz: the GEMM's tiles would overwrite rows that sibling
    // workgroups still read)
    if (int rc = head(4, 1, f->d_dpr, 3, 2, f->d_dh)) return rc;
    hipLaunchKernelGGL(fit_add, dim3((B * h + 255) / 256), dim3(256), 0, st, f->d_dh2, f->d_dh, B * h);
    FIT_TRY(hipGetLastError());
    // trunk: dH0 (d_dh2) -> LN / tanh backward -> dense's gradients
    if (ln)
        hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dh2, G + f->be_off[0], B, h,
                           slot_a(0), mean_of(0), rs_of(0), G + f->g_off[0], f->d_cpart, f->d_tickets);
    hipLaunchKernelGGL(fit_act_bwd, rows, rthreads, 0, st, f->d_dh2, f->d_dz, slot_a(0), mean_of(0), rs_of(0),
                       W + f->g_off[0], B, h, act, ln);
    FIT_TRY(hipGetLastError());
    FIT_TRY((gemm<true, false>(f->d_x0, f->d_dz, G + f->w_off[0], nullptr, IN, h, B, IN, h, h, st, f->d_split,
                               f->split_floats)));
    hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dz, G + f->b_off[0], B, h,
                       nullptr, nullptr, nullptr, nullptr, f->d_cpart, f->d_tickets);
    FIT_TRY(hipGetLastError());
    const int64_t n = (int64_t)f->n_params;
    hipLaunchKernelGGL(fit_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, f->d_m, f->d_v, G, n,
                       f->d_bp, f->cfg.learning_rate, f->cfg.beta1, f->cfg.beta2, f->cfg.epsilon);
    FIT_TRY(hipGetLastError());
#undef FIT_TRY
    return BCMPC_OK;
}

static int fit_iteration(bcmpc_fitter* f, const int64_t* d_idx, int stride, int B, float* d_loss) {
    if (f->rw) return fit_iteration_reward(f, d_idx, stride, B, d_loss);
    if (f->fused) return fit_iteration_fused(f, d_idx, stride, B, d_loss);
    hipStream_t st = f->stream;
    const int S = f->S, IN = f->IN, L = f->L, h = f->h, act = f->cfg.activation, ln = f->cfg.layer_norm;
    const size_t BH = (size_t)f->Bmax * h;
    float* W = f->d_w;
    float* G = f->d_g;
#define FIT_TRY(x) do { if ((x) != hipSuccess) return ffail(BCMPC_ERR_HIP, #x); } while (0)
    const int ng = B * (IN + S);
    hipLaunchKernelGGL(fit_gather, dim3((ng + 255) / 256), dim3(256), 0, st, f->d_st, f->d_ac, f->d_de, d_idx,
                       stride, f->d_iter, f->d_nc, f->d_x0, f->d_t, B, S, f->A);
    FIT_TRY(hipGetLastError());
    // ---- forward ----
    const dim3 rows((B + 3) / 4), rthreads(256);
    for (int l = 0; l < L; ++l) {
        const float* Hin = l == 0 ? f->d_x0 : (ln ? f->d_hln + (l - 1) * BH : f->d_act + (l - 1) * BH);
        const int in = l == 0 ? IN : h;
        float* Z = f->d_act + l * BH;
        FIT_TRY((gemm<false, false>(Hin, W + f->w_off[l], Z, W + f->b_off[l], B, h, in, in, h, h, st)));
        hipLaunchKernelGGL(fit_act_fwd, rows, rthreads, 0, st, Z, f->d_hln + l * BH, f->d_mean + l * f->Bmax,
                           f->d_rs + l * f->Bmax, W + f->g_off[l], W + f->be_off[l], B, h, act, ln);
        FIT_TRY(hipGetLastError());
    }
    const float* HL = ln ? f->d_hln + (L - 1) * BH : f->d_act + (L - 1) * BH;
    FIT_TRY((gemm<false, false>(HL, W + f->w_off[L], f->d_p, W + f->b_off[L], B, S, h, h, S, S, st)));
    hipLaunchKernelGGL(fit_loss, dim3(1), dim3(1024), 0, st, f->d_p, f->d_t, f->d_dp, d_loss, f->d_iter, f->d_bp,
                       f->cfg.beta1, f->cfg.beta2, B * S);
    FIT_TRY(hipGetLastError());
    // ---- backward ----
    // output layer: dW_L = H_L^T dP, db_L = colsum dP, dH = dP W_L^T
    FIT_TRY((gemm<true, false>(HL, f->d_dp, G + f->w_off[L], nullptr, h, S, B, h, S, S, st, f->d_split,
                               f->split_floats)));
    const int nch = std::max(1, std::min(kColChunks, B / 32));
    hipLaunchKernelGGL(fit_colsum, dim3((S + 63) / 64, nch), dim3(256), 0, st, f->d_dp, G + f->b_off[L], B, S, nullptr,
                       nullptr, nullptr, nullptr, f->d_cpart, f->d_tickets);
    FIT_TRY(hipGetLastError());
    FIT_TRY((gemm<false, true>(f->d_dp, W + f->w_off[L], f->d_dh, nullptr, B, h, S, S, S, h, st)));
    for (int l = L - 1; l >= 0; --l) {
        const float* Aact = f->d_act + l * BH;
        if (ln)   // LN grads: beta = colsum dH, gamma = colsum dH * xhat
            hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dh, G + f->be_off[l], B,
                               h, Aact, f->d_mean + l * f->Bmax, f->d_rs + l * f->Bmax, G + f->g_off[l], f->d_cpart,
                               f->d_tickets);
        hipLaunchKernelGGL(fit_act_bwd, rows, rthreads, 0, st, f->d_dh, f->d_dz, Aact, f->d_mean + l * f->Bmax,
                           f->d_rs + l * f->Bmax, W + f->g_off[l], B, h, act, ln);
        FIT_TRY(hipGetLastError());
        const float* Hin = l == 0 ? f->d_x0 : (ln ? f->d_hln + (l - 1) * BH : f->d_act + (l - 1) * BH);
        const int in = l == 0 ? IN : h;
        FIT_TRY((gemm<true, false>(Hin, f->d_dz, G + f->w_off[l], nullptr, in, h, B, in, h, h, st, f->d_split,
                                   f->split_floats)));
        hipLaunchKernelGGL(fit_colsum, dim3((h + 63) / 64, nch), dim3(256), 0, st, f->d_dz, G + f->b_off[l], B, h,
                           nullptr, nullptr, nullptr, nullptr, f->d_cpart, f->d_tickets);
        FIT_TRY(hipGetLastError());
        if (l > 0) FIT_TRY((gemm<false, true>(f->d_dz, W + f->w_off[l], f->d_dh, nullptr, B, in, h, h, h, in, st)));
    }
    // (without LayerNorm the LN slots of G are never written: zero since create, no update)
    // ---- Adam (TF1 ApplyAdam; beta powers are f32 variables updated after the step) ----
    const float b1 = f->cfg.beta1, b2 = f->cfg.beta2;
    const int64_t n = (int64_t)f->n_params;
    hipLaunchKernelGGL(fit_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, f->d_m, f->d_v, G, n,
                       f->d_bp, f->cfg.learning_rate, b1, b2, f->cfg.epsilon);
    FIT_TRY(hipGetLastError());

#undef FIT_TRY
    return BCMPC_OK;
}

int bcmpc_fit_run(bcmpc_fitter* f, const int64_t* indices, const int32_t* batch_sizes, int32_t iterations,
                  float* losses) {
    if (!f || !indices || !batch_sizes || iterations < 0) return ffail(BCMPC_ERR_ARG, "null argument");
    if (!f->has_weights) return ffail(BCMPC_ERR_STATE, "bcmpc_fit_set_params has not been called");
    if (f->rw && !f->has_rewards) return ffail(BCMPC_ERR_STATE, "reward model: bcmpc_fit_set_rewards has not been called");
    if (hipSetDevice(f->cfg.device) != hipSuccess) return ffail(BCMPC_ERR_HIP, "hipSetDevice failed");
    int64_t total = 0;
    for (int i = 0; i < iterations; ++i) {
        if (batch_sizes[i] < 1 || batch_sizes[i] > f->Bmax) return ffail(BCMPC_ERR_ARG, "batch size out of range");
        total += batch_sizes[i];
    }
    for (int64_t i = 0; i < total; ++i)
        if (indices[i] < 0 || indices[i] >= f->n_data) return ffail(BCMPC_ERR_ARG, "sample index out of range");
    if (total > f->idx_cap) {
        if (f->d_idx) (void)hipFree(f->d_idx);
        f->d_idx = nullptr;
        f->idx_cap = 0;
        if (hipMalloc(&f->d_idx, (size_t)std::max<int64_t>(total, 1) * 8) != hipSuccess)
            return ffail(BCMPC_ERR_HIP, "index buffer allocation failed");
        f->idx_cap = total;
    }
    if (total > 0 &&
        hipMemcpyAsync(f->d_idx, indices, (size_t)total * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess)
        return ffail(BCMPC_ERR_HIP, "index upload failed");
    if (iterations > f->loss_cap) {
        for (float** p : {&f->d_loss, &f->d_loss2})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
        f->loss_cap = 0;
        if (hipMalloc(&f->d_loss, (size_t)iterations * 4) != hipSuccess ||
            (f->rw && hipMalloc(&f->d_loss2, (size_t)iterations * 4) != hipSuccess))
            return ffail(BCMPC_ERR_HIP, "loss buffer allocation failed");
        f->loss_cap = iterations;
    }
    // device iteration state: counter 0, the host mirror's beta powers
    const float bp[2] = {f->beta1_power, f->beta2_power};
    if (hipMemsetAsync(f->d_iter, 0, 4, f->stream) != hipSuccess ||
        hipMemcpyAsync(f->d_bp, bp, 8, hipMemcpyHostToDevice, f->stream) != hipSuccess)
        return ffail(BCMPC_ERR_HIP, "iteration state upload failed");
    bool uniform = iterations > 0;
    for (int i = 1; i < iterations; ++i) uniform = uniform && batch_sizes[i] == batch_sizes[0];
    const char* ge = std::getenv("BCMPC_FIT_GRAPH");
    const bool use_graph = uniform && !(ge && ge[0] == '0');
    if (use_graph) {
        // the whole run as one graph (~20 launches per iteration otherwise dominate a 512-row step)
        if (!(f->graph && f->graph_iters == iterations && f->graph_b == batch_sizes[0] && f->graph_idx == f->d_idx &&
              f->graph_loss == f->d_loss)) {
            if (f->graph) (void)hipGraphExecDestroy(f->graph);
            f->graph = nullptr;
            if (hipStreamBeginCapture(f->stream, hipStreamCaptureModeThreadLocal) != hipSuccess)
                return ffail(BCMPC_ERR_HIP, "graph capture failed to start");
            int rc = BCMPC_OK;
            for (int i = 0; i < iterations && rc == BCMPC_OK; ++i)
                rc = fit_iteration(f, f->d_idx, batch_sizes[0], batch_sizes[0], f->d_loss);
            hipGraph_t g = nullptr;
            const hipError_t ec = hipStreamEndCapture(f->stream, &g);
            if (rc != BCMPC_OK || ec != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                return rc != BCMPC_OK ? rc : ffail(BCMPC_ERR_HIP, "graph capture failed");
            }
            const hipError_t ei = hipGraphInstantiate(&f->graph, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ei != hipSuccess) { f->graph = nullptr; return ffail(BCMPC_ERR_HIP, "graph instantiation failed"); }
            f->graph_iters = iterations;
            f->graph_b = batch_sizes[0];
            f->graph_idx = f->d_idx;
            f->graph_loss = f->d_loss;
        }
        if (hipGraphLaunch(f->graph, f->stream) != hipSuccess) return ffail(BCMPC_ERR_HIP, "graph launch failed");
    } else {
        int64_t pos = 0;
        for (int i = 0; i < iterations; ++i) {
            const int rc = fit_iteration(f, f->d_idx + pos, 0, batch_sizes[i], f->d_loss);
            if (rc != BCMPC_OK) return rc;
            pos += batch_sizes[i];
        }
    }
    for (int i = 0; i < iterations; ++i) {       // host mirror of the device beta powers (same f32 products)
        f->beta1_power *= f->cfg.beta1;
        f->beta2_power *= f->cfg.beta2;
        ++f->step;
    }
    if (losses && iterations > 0 &&
        hipMemcpyAsync(losses, f->d_loss, (size_t)iterations * 4, hipMemcpyDeviceToHost, f->stream) != hipSuccess)
        return ffail(BCMPC_ERR_HIP, "loss download failed");
    if (hipStreamSynchronize(f->stream) != hipSuccess) return ffail(BCMPC_ERR_HIP, "fit failed");
    f->last_iters = iterations;
    return BCMPC_OK;
}

int bcmpc_fit_set_rewards(bcmpc_fitter* f, const double* rewards, int64_t n) {
    if (!f || (n > 0 && !rewards) || n < 0) return ffail(BCMPC_ERR_ARG, "bad argument");
    if (!f->rw) return ffail(BCMPC_ERR_STATE, "the fitter was created for the delta model (config.model)");
    if (n != f->n_data) return ffail(BCMPC_ERR_ARG, "rewards: one per row of bcmpc_fit_set_data");
    if (hipSetDevice(f->cfg.device) != hipSuccess) return ffail(BCMPC_ERR_HIP, "hipSetDevice failed");
    if (n > f->rw_cap) {
        if (f->d_rwd) (void)hipFree(f->d_rwd);
        f->d_rwd = nullptr;
        f->rw_cap = 0;
        if (hipMalloc(&f->d_rwd, (size_t)std::max<int64_t>(n, 1) * 8) != hipSuccess)
            return ffail(BCMPC_ERR_HIP, "reward buffer allocation failed");
        f->rw_cap = n;
    }
    if (n > 0 && (hipMemcpyAsync(f->d_rwd, rewards, (size_t)n * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
                  hipStreamSynchronize(f->stream) != hipSuccess))
        return ffail(BCMPC_ERR_HIP, "reward upload failed");
    f->has_rewards = true;
    return BCMPC_OK;
}

int bcmpc_fit_reward_losses(bcmpc_fitter* f, float* losses) {
    if (!f || !losses) return ffail(BCMPC_ERR_ARG, "null argument");
    if (!f->rw) return ffail(BCMPC_ERR_STATE, "the fitter was created for the delta model (config.model)");
    if (f->last_iters > 0 &&
        (hipMemcpy(losses, f->d_loss2, (size_t)f->last_iters * 4, hipMemcpyDeviceToHost) != hipSuccess))
        return ffail(BCMPC_ERR_HIP, "loss download failed");
    return BCMPC_OK;
}

}  // extern "C"
