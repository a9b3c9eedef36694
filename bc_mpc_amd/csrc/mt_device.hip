// mt_device.hip -- NumPy's legacy MT19937 draw of MPCcontroller.sample_random_actions
// (controllers.py:53: np.random.uniform(low, high, [H, K, A]) from the global RandomState) made
// on the GPU, bit for bit, continued from np.random.get_state() and handing back the state NumPy
// would hold after the same call.
//
// Stream.  Let y be the generator's raw words with y[0..623] = the caller's key block.  For every
// n >= 624, y[n] = y[n - 227] ^ mix(y[n - 624], y[n - 623]) (the twist of mt19937.c read as one
// linear recurrence), so 227 consecutive words can be produced in parallel from the 624 before
// them.  Draw word w is y[pos + w]; random_sample double d takes words 2d, 2d + 1:
// ((t(a) >> 5) * 2^26 + (t(b) >> 6)) / 2^53 (t = tempering), and the uniform is
// low[j] + (high[j] - low[j]) * d (mul, then add), j = d mod A.
//
// Parallel draw.  The draw is cut into chunks of consecutive words (MtChunk); chunk c starts
// from the 624-word window of block f = floor(s / 624): the key (f = 0), twist(key) (f = 1), or
// for f >= 2 the jump F^(624 (f - 1)) applied to block 1 = x[0..623].  By the jump-ahead
// identity F^J W = (x^J mod phi)(F) W (Haramoto et al. 2008; see mt_jump.cpp), block f's word m
// is XOR over the set coefficients i of g = x^(624 (f - 1)) mod phi of x[i + m], x = block 1's
// stream -- a GF(2) correlation of one 20.7k-word stream (generated once, mt_stream_kernel) with
// each chunk's polynomial (host-computed once per draw shape, mt_block_polys): mt_jump_kernel,
// one workgroup per (chunk, slice of the coefficients), partial windows XOR-combined by the
// generator.  mt_gen_kernel then runs each chunk's words from its window in LDS and stores them
// as uniforms straight into the shard's [H, K, A] f64 action array.
//
// All integer work (LDS + VALU/SALU); nothing here is a GEMM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace bcmpc {

namespace {

constexpr int kThreads = 256;
constexpr int kLag = 227;                 // 624 - 397: words producible in parallel
constexpr int kRing = 2048;               // generator ring (words), power of two

__device__ __forceinline__ uint32_t mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// one phase: ring words [n0, n0 + 227) from the 624 before them (all threads; one barrier after)
__device__ __forceinline__ void gen_phase(uint32_t* ring, int64_t n0) {
    const int t = threadIdx.x;
    if (t < kLag) {
        const int64_t n = n0 + t;
        ring[n & (kRing - 1)] = ring[(n - kLag) & (kRing - 1)] ^
                                mix(ring[(n - kMtN) & (kRing - 1)], ring[(n - kMtN + 1) & (kRing - 1)]);
    }
    __syncthreads();
}

// x[0 .. kMtStream) = y[624 ..): block 1 onwards, the stream every jump correlates with
__global__ __launch_bounds__(kThreads) void mt_stream_kernel(const uint32_t* __restrict__ in,
                                                             uint32_t* __restrict__ xs) {
    __shared__ uint32_t ring[kRing];
    for (int i = threadIdx.x; i < kMtN; i += kThreads) ring[i] = in[i];
    __syncthreads();
    for (int64_t n0 = kMtN; n0 < kMtN + kMtStream; n0 += kLag) {
        const int t = threadIdx.x;
        if (t < kLag) {
            const int64_t n = n0 + t;
            const uint32_t v = ring[(n - kLag) & (kRing - 1)] ^
                               mix(ring[(n - kMtN) & (kRing - 1)], ring[(n - kMtN + 1) & (kRing - 1)]);
            ring[n & (kRing - 1)] = v;
            if (n - kMtN < kMtStream) xs[n - kMtN] = v;
        }
        __syncthreads();
    }
}

// partial window of jump polynomial blockIdx.x / S over its coefficient words [w0, w1):
// part[m] = XOR_{i in [32 w0, 32 w1), g_i = 1} x[i + m], m in [0, 624)
__global__ __launch_bounds__(kThreads) void mt_jump_kernel(MtDrawArgs a) {
    extern __shared__ uint32_t seg[];     // x[32 w0 .. 32 w1 + 768)
    const int j = blockIdx.x / a.S, sp = blockIdx.x % a.S;
    const int w0 = sp * kMtPolyWords / a.S, w1 = (sp + 1) * kMtPolyWords / a.S;
    const int base = 32 * w0, len = 32 * (w1 - w0) + 768;
    for (int i = threadIdx.x; i < len; i += kThreads) seg[i] = a.xs[base + i];
    __syncthreads();
    const int t = threadIdx.x;
    const bool third = t < kMtN - 2 * kThreads;          // m = t + 512 exists for t < 112
    uint32_t acc0 = 0, acc1 = 0, acc2 = 0;
    const uint32_t* g = a.polys + (size_t)j * kMtPolyWords;
    for (int w = w0; w < w1; ++w) {
        uint32_t cw = __builtin_amdgcn_readfirstlane(g[w]);
        const int ib = 32 * (w - w0);
        while (cw) {                                      // uniform loop over the set coefficients
            const int i = ib + __builtin_ctz(cw);
            cw &= cw - 1;
            acc0 ^= seg[i + t];
            acc1 ^= seg[i + t + kThreads];
            if (third) acc2 ^= seg[i + t + 2 * kThreads];
        }
    }
    uint32_t* p = a.part + (size_t)blockIdx.x * kMtN;
    p[t] = acc0;
    p[t + kThreads] = acc1;
    if (third) p[t + 2 * kThreads] = acc2;
}

// one workgroup per chunk: window -> words [o, o + n) of the local stream -> uniforms
__global__ __launch_bounds__(kThreads) void mt_gen_kernel(MtDrawArgs a) {
    __shared__ uint32_t ring[kRing];
    const MtChunk ch = a.chunks[blockIdx.x];
    const int t = threadIdx.x;
    const int32_t pos = (int32_t)a.in[kMtN];
    // local stream index l: l = 0 is word 0 of the start window
    int f = ch.f;
    int64_t o = (int64_t)pos + ch.s - (int64_t)kMtN * f;   // local index of the chunk's first word
    if (f <= 1) {                                         // block 1 = the key block run forward
        o += (int64_t)kMtN * f;
        f = 0;
        for (int i = t; i < kMtN; i += kThreads) ring[i] = a.in[i];
    } else {
        const uint32_t* p = a.part + (size_t)ch.jidx * a.S * kMtN;
        for (int i = t; i < kMtN; i += kThreads) {
            uint32_t v = 0;
            for (int s = 0; s < a.S; ++s) v ^= p[(size_t)s * kMtN + i];
            ring[i] = v;
        }
    }
    __syncthreads();
    const int64_t nd = ch.n / 2;                          // doubles of this chunk
    const int A = a.A;
    const double* low = a.bounds;
    const double* high = a.bounds + A;
    int64_t avail = kMtN;                                 // local words [0, avail) generated
    int64_t e_done = 0;                                   // doubles emitted
    while (e_done < nd) {
        // generate up to 4 phases (908 words): the ring keeps 624 words of history + the batch
        // + at most one unemitted word
        const int64_t need = o + 2 * nd;
        for (int k = 0; k < 4 && avail < need; ++k, avail += kLag) gen_phase(ring, avail);
        // every double whose two words exist
        const int64_t e_avail = avail > o ? (avail - o) / 2 : 0;
        const int64_t e_end = e_avail < nd ? e_avail : nd;
        if (ch.out0 >= 0) {
            for (int64_t e = e_done + t; e < e_end; e += kThreads) {
                const int64_t l = o + 2 * e;
                const uint32_t wa = temper(ring[l & (kRing - 1)]) >> 5;
                const uint32_t wb = temper(ring[(l + 1) & (kRing - 1)]) >> 6;
                // (a * 2^26 + b) / 2^53: exact in f64 (< 2^53), as rk_double
                const double d = (double)(((uint64_t)wa << 26) | wb) * 0x1p-53;
                const int jj = (ch.j0 + (int)e) % A;
                const double lo = low[jj];
                a.out[ch.out0 + e] = __dadd_rn(lo, __dmul_rn(__dsub_rn(high[jj], lo), d));
            }
        }
        e_done = e_end;
        __syncthreads();
    }
    if (ch.final_) {
        // NumPy's state after the last word: the 624-word block holding it (complete) and the
        // position after it (rk_random twists lazily, so pos may be 624)
        const int64_t last = o + ch.n - 1;
        const int64_t b0 = (last / kMtN) * kMtN;
        while (avail < b0 + kMtN) {
            gen_phase(ring, avail);
            avail += kLag;
        }
        for (int i = t; i < kMtN; i += kThreads) a.final_state[i] = ring[(b0 + i) & (kRing - 1)];
        if (t == 0) a.final_state[kMtN] = (uint32_t)(last - b0 + 1);
    }
}

}  // namespace

hipError_t launch_mt_draw(const MtDrawArgs& a, hipStream_t st) {
    if (a.Cj > 0) {
        hipLaunchKernelGGL(mt_stream_kernel, dim3(1), dim3(kThreads), 0, st, a.in, a.xs);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        const int w_max = (kMtPolyWords + a.S - 1) / a.S + 1;
        const size_t lds = (size_t)(32 * w_max + 768) * sizeof(uint32_t);
        static size_t attr = 48 * 1024;                   // (set once per size above the default)
        if (lds > attr) {
            const hipError_t e = hipFuncSetAttribute((const void*)mt_jump_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            attr = lds;
        }
        hipLaunchKernelGGL(mt_jump_kernel, dim3(a.Cj * a.S), dim3(kThreads), lds, st, a);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(mt_gen_kernel, dim3(a.nchunks), dim3(kThreads), 0, st, a);
    return hipGetLastError();
}

}  // namespace bcmpc
