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

// loss = mean((T - P)^2) (one block), dP = -((2 * (1/N)) * (T - P))
__global__ __launch_bounds__(1024) void fit_loss(const float* __restrict__ P, const float* __restrict__ T,
                                                 float* __restrict__ dP, float* __restrict__ loss_base,
                                                 int32_t* __restrict__ iter, float* __restrict__ bp, float b1,
                                                 float b2, int n) {
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
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || c->device < 0 || c->device >= ndev)
        return ffail(BCMPC_ERR_ARG, "device ordinal out of range");
    if (hipSetDevice(c->device) != hipSuccess) return ffail(BCMPC_ERR_HIP, "hipSetDevice failed");
    bcmpc_fitter* f = new bcmpc_fitter();
    f->cfg = *c;
    f->S = c->state_dim; f->A = c->action_dim; f->IN = f->S + f->A; f->L = c->n_layers; f->h = c->hidden;
    f->Bmax = c->batch_size;
    size_t off = 0;
    for (int l = 0; l <= f->L; ++l) {
        const int in = l == 0 ? f->IN : f->h, o = l == f->L ? f->S : f->h;
        f->w_off.push_back(off); off += (size_t)in * o;
        f->b_off.push_back(off); off += o;
    }
    for (int l = 0; l < f->L; ++l) {
        f->g_off.push_back(off); off += f->h;
        f->be_off.push_back(off); off += f->h;
    }
    f->n_params = off;
    const size_t B = (size_t)f->Bmax, H = (size_t)f->h, L = (size_t)f->L;
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
              al((void**)&f->d_tickets, 64 * 4);
    if (!ok) { bcmpc_fit_destroy(f); return ffail(BCMPC_ERR_HIP, "device allocation failed"); }
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
                    (void*)f->d_ac, (void*)f->d_de, (void*)f->d_nc, (void*)f->d_idx, (void*)f->d_split})
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
    std::vector<float> hw(f->n_params, 0.f);
    for (int l = 0; l <= f->L; ++l) {
        const int in = l == 0 ? f->IN : f->h, o = l == f->L ? f->S : f->h;
        if (!w->kernels[l] || !w->biases[l]) return ffail(BCMPC_ERR_ARG, "null kernel / bias");
        std::copy(w->kernels[l], w->kernels[l] + (size_t)in * o, hw.begin() + f->w_off[l]);
        std::copy(w->biases[l], w->biases[l] + o, hw.begin() + f->b_off[l]);
    }
    for (int l = 0; l < f->L; ++l) {
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
    if (hipSetDevice(f->cfg.device) != hipSuccess ||
        hipMemcpyAsync(f->d_w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
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
    for (int l = 0; l <= f->L; ++l) {
        const int in = l == 0 ? f->IN : f->h, o = l == f->L ? f->S : f->h;
        std::copy(hw.begin() + f->w_off[l], hw.begin() + f->w_off[l] + (size_t)in * o, kernels[l]);
        std::copy(hw.begin() + f->b_off[l], hw.begin() + f->b_off[l] + o, biases[l]);
    }
    if (f->cfg.layer_norm && ln_gamma && ln_beta)
        for (int l = 0; l < f->L; ++l) {
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

static int fit_iteration(bcmpc_fitter* f, const int64_t* d_idx, int stride, int B, float* d_loss) {
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
        if (f->d_loss) (void)hipFree(f->d_loss);
        f->d_loss = nullptr;
        f->loss_cap = 0;
        if (hipMalloc(&f->d_loss, (size_t)iterations * 4) != hipSuccess)
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
    return BCMPC_OK;
}

}  // extern "C"
