// Microbenchmark: does f64 VALU (or f32 VALU / transcendental) on one wave of a SIMD slow down, or get
// slowed by, MFMAs of the other wave on the same SIMD?  512-thread workgroup, one per CU; waves w and
// w + 4 share a SIMD.  mode: 0 both MFMA-only-on-0-3 + idle 4-7; 1 VALU-only (waves 4-7) alone;
// 2 MFMA (0-3) beside VALU (4-7).  vkind: 0 f64 fma, 1 f32 fma, 2 exp/rcp (f32 trans).
// Prints per-group average cycles (s_memtime) of their loops.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void kern(int mode, int vkind, int iters, uint64_t* out, float* sink) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    float res = 0.f;
    if (w < 4) {
        if (mode == 0 || mode == 2) {
            h8 a = (h8)(_Float16)(0.001f * lane), b = (h8)(_Float16)0.002f;
            f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
            for (int i = 0; i < iters; ++i) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
            }
            res = c0[0] + c1[1] + c2[2] + c3[3];
        }
    } else {
        if (mode == 1 || mode == 2) {
            if (vkind == 0) {
                double x0 = 1.0 + lane, x1 = 2.0, x2 = 3.0, x3 = 4.0, y = 0.999999;
                for (int i = 0; i < iters; ++i) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        x0 = __builtin_fma(x0, y, 1e-9); x1 = __builtin_fma(x1, y, 1e-9);
                        x2 = __builtin_fma(x2, y, 1e-9); x3 = __builtin_fma(x3, y, 1e-9);
                    }
                }
                res = (float)(x0 + x1 + x2 + x3);
            } else if (vkind == 1) {
                float x0 = 1.0f + lane, x1 = 2.f, x2 = 3.f, x3 = 4.f, y = 0.9999f;
                for (int i = 0; i < iters; ++i) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        x0 = __builtin_fmaf(x0, y, 1e-9f); x1 = __builtin_fmaf(x1, y, 1e-9f);
                        x2 = __builtin_fmaf(x2, y, 1e-9f); x3 = __builtin_fmaf(x3, y, 1e-9f);
                    }
                }
                res = x0 + x1 + x2 + x3;
            } else {
                float x0 = 0.1f + 0.001f * lane, x1 = 0.2f, x2 = 0.3f, x3 = 0.4f;
                for (int i = 0; i < iters; ++i) {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        x0 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x0) + 1.f);
                        x1 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x1) + 1.f);
                        x2 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x2) + 1.f);
                        x3 = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x3) + 1.f);
                    }
                }
                res = x0 + x1 + x2 + x3;
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 8 + w] = t1 - t0;
    if (res == 12345.f) sink[threadIdx.x] = res;
}

int main() {
    const int blocks = 256, iters = 2000;
    uint64_t* d; float* sink;
    hipMalloc(&d, blocks * 8 * sizeof(uint64_t));
    hipMalloc(&sink, 512 * sizeof(float));
    uint64_t h[blocks * 8];
    const char* vk[3] = {"f64 fma", "f32 fma", "exp+add+rcp"};
    for (int vkind = 0; vkind < 3; ++vkind)
        for (int mode = 0; mode < 3; ++mode) {
            for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, mode, vkind, iters, d, sink);
            hipDeviceSynchronize();
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            double m0 = 0, m1 = 0;
            for (int b = 0; b < blocks; ++b)
                for (int w = 0; w < 8; ++w) (w < 4 ? m0 : m1) += (double)h[b * 8 + w];
            m0 /= blocks * 4; m1 /= blocks * 4;
            printf("valu=%-12s mode=%d (%s): mfma waves %.0f cycles (%.1f per mfma), valu waves %.0f cycles (%.2f per op)\n",
                   vk[vkind], mode, mode == 0 ? "mfma alone" : mode == 1 ? "valu alone" : "mfma beside valu", m0,
                   m0 / (iters * 4.0), m1, m1 / (iters * (vkind == 2 ? 8.0 * 2 : 16.0)));
        }
    return 0;
}
