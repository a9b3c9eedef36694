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

constexpr int kWave = 64;                 // mt_jump_kernel: one wave per (chunk, coefficient slice)
constexpr int kGen = 256;                 // generators: 4 waves (a phase is 227 independent words)
constexpr int kLag = 227;                 // 624 - 397: words producible in parallel
constexpr int kRing = 4096;               // generator ring (words), power of two
constexpr int kBatch = 12;                // generator phases between emission passes
constexpr int kQ = 10;                    // jump: window words m per lane (64 x 10 >= 624)

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

// The register-chained generator.  Thread t < 227 owns word n = 624 + 227 P + t of every phase P
// (local stream index): it keeps its previous word y[n - 227] in a register and has the two older
// operands y[n - 624], y[n - 623] -- words of phases <= P - 1, i.e. published by the barrier that
// ended the previous interval -- fetched one interval ahead.  An interval is then one mix + XOR and
// one LDS store on the critical path, and one barrier per 227 words; the prefetch (and whatever work
// the caller puts in the interval) hides the LDS latency.  Ring slots written in phase P alias words
// >= 1400 older than anything read.
struct Chain {
    uint32_t prev = 0, a = 0, b = 0;
    int64_t n = 0;
    // ring words [0, 624) hold the start window
    __device__ __forceinline__ void init(const uint32_t* ring, int t) {
        n = kMtN + t;
        if (t < kLag) {
            prev = ring[kMtN - kLag + t];
            a = ring[t];
            b = ring[t + 1];
        }
    }
    // produce word n (threads < 227), store it, fetch the operands of the next phase
    __device__ __forceinline__ uint32_t step(uint32_t* ring, int t) {
        uint32_t v = 0;
        if (t < kLag) {
            v = prev ^ mix(a, b);
            ring[n & (kRing - 1)] = v;
            prev = v;
            a = ring[(n + kLag - kMtN) & (kRing - 1)];
            b = ring[(n + kLag - kMtN + 1) & (kRing - 1)];
        }
        n += kLag;
        return v;
    }
};

// x[0 .. kMtStream) = y[624 ..): block 1 onwards, the stream every jump correlates with
__global__ __launch_bounds__(kGen) void mt_stream_kernel(const uint32_t* __restrict__ in,
                                                         uint32_t* __restrict__ xs) {
    __shared__ uint32_t ring[kRing];
    const int t = threadIdx.x;
    for (int i = t; i < kMtN; i += kGen) ring[i] = in[i];
    __syncthreads();
    Chain ch;
    ch.init(ring, t);
    for (int64_t n0 = kMtN; n0 < kMtN + kMtStream; n0 += kLag) {
        const uint32_t v = ch.step(ring, t);
        if (t < kLag && n0 + t - kMtN < kMtStream) xs[n0 + t - kMtN] = v;
        __syncthreads();
    }
}

// partial window of jump polynomial blockIdx.x / S over its coefficient words [w0, w1):
// part[m] = XOR_{i in [32 w0, 32 w1), g_i = 1} x[i + m], m in [0, 624).  Lane l owns m = 10 l + q,
// q < 10: per coefficient word it reads the 41 stream words x[32 w + 10 l .. + 41) once into
// registers and XORs v[k + q] into acc[q] for every set bit k (a uniform branch per bit), i.e.
// ~4 LDS words per 32 x 10 (term, m) pairs instead of one per pair.
__global__ __launch_bounds__(kWave) void mt_jump_kernel(MtDrawArgs a) {
    extern __shared__ uint32_t seg[];     // x[32 w0 .. 32 w1 + 32 + kWave kQ)
    const int j = blockIdx.x / a.S, sp = blockIdx.x % a.S;
    const int w0 = sp * kMtPolyWords / a.S, w1 = (sp + 1) * kMtPolyWords / a.S;
    const int base = 32 * w0, len = 32 * (w1 - w0) + 32 + kWave * kQ;
    for (int i = threadIdx.x; i < len; i += kWave) seg[i] = a.xs[base + i];
    __syncthreads();
    const int l = threadIdx.x;
    uint32_t acc[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) acc[q] = 0;
    const uint32_t* g = a.polys + (size_t)j * kMtPolyWords;
    for (int w = w0; w < w1; ++w) {
        const uint32_t cw = __builtin_amdgcn_readfirstlane(g[w]);
        if (!cw) continue;
        const uint2* xp = reinterpret_cast<const uint2*>(seg + 32 * (w - w0) + kQ * l);   // 8-byte aligned
        uint32_t v[32 + kQ];
#pragma unroll
        for (int t = 0; t < (32 + kQ) / 2; ++t) {
            const uint2 p = xp[t];
            v[2 * t] = p.x;
            v[2 * t + 1] = p.y;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k)
            if (cw & (1u << k)) {
#pragma unroll
                for (int q = 0; q < kQ; ++q) acc[q] ^= v[k + q];
            }
    }
    uint32_t* p = a.part + (size_t)blockIdx.x * kMtN;
#pragma unroll
    for (int q = 0; q < kQ; ++q)
        if (kQ * l + q < kMtN) p[kQ * l + q] = acc[q];
}

// one workgroup per chunk: window -> words [o, o + n) of the local stream -> uniforms
__global__ __launch_bounds__(kGen) void mt_gen_kernel(MtDrawArgs a) {
    __shared__ uint32_t ring[kRing];
    const MtChunk ch = a.chunks[blockIdx.x];
    const int t = threadIdx.x;
    const int32_t pos = (int32_t)a.in[kMtN];
    // local stream index l: l = 0 is word 0 of the start window
    const int f = ch.f;
    int64_t o = (int64_t)pos + ch.s - (int64_t)kMtN * f;   // local index of the chunk's first word
    if (f <= 1) {                                         // block 1 = the key block run forward
        o += (int64_t)kMtN * f;
        for (int i = t; i < kMtN; i += kGen) ring[i] = a.in[i];
    } else {
        const uint32_t* p = a.part + (size_t)ch.jidx * a.S * kMtN;
        for (int i = t; i < kMtN; i += kGen) {
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
    const int64_t need = o + 2 * nd;                      // words the chunk reads
    Chain gen;
    gen.init(ring, t);
    while (e_done < nd) {
        // up to kBatch chain intervals (2724 words; the ring keeps them + 624 words of history +
        // one pending word), then one emission pass over every double whose two words exist: the
        // emission's latency chain (LDS, tempering, f64) overlaps across a thread's ~5 doubles
        // instead of sitting in every interval
        for (int k = 0; k < kBatch && avail < need; ++k) {
            (void)gen.step(ring, t);
            avail += kLag;
            __syncthreads();
        }
        const int64_t e_avail = avail > o ? (avail - o) / 2 : 0;
        const int64_t e_end = e_avail < nd ? e_avail : nd;
        if (ch.out0 >= 0) {
            int jj = (ch.j0 + (int)(e_done + t)) % A;      // action column, advanced by kGen per pass
            const int stride = kGen % A;
            for (int64_t e = e_done + t; e < e_end; e += kGen) {
                const int64_t l = o + 2 * e;
                const uint32_t wa = temper(ring[l & (kRing - 1)]) >> 5;
                const uint32_t wb = temper(ring[(l + 1) & (kRing - 1)]) >> 6;
                // (a * 2^26 + b) / 2^53: exact in f64 (< 2^53), as rk_double
                const double d = (double)(((uint64_t)wa << 26) | wb) * 0x1p-53;
                const double lo = low[jj];
                a.out[ch.out0 + e] = __dadd_rn(lo, __dmul_rn(__dsub_rn(high[jj], lo), d));
                jj += stride;
                if (jj >= A) jj -= A;
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
            (void)gen.step(ring, t);
            avail += kLag;
            __syncthreads();
        }
        for (int i = t; i < kMtN; i += kGen) a.final_state[i] = ring[(b0 + i) & (kRing - 1)];
        if (t == 0) a.final_state[kMtN] = (uint32_t)(last - b0 + 1);
    }
}

}  // namespace

hipError_t launch_mt_draw(const MtDrawArgs& a, hipStream_t st) {
    if (a.Cj > 0) {
        hipLaunchKernelGGL(mt_stream_kernel, dim3(1), dim3(kGen), 0, st, a.in, a.xs);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        const int w_max = (kMtPolyWords + a.S - 1) / a.S + 1;
        const size_t lds = (size_t)(32 * w_max + 32 + kWave * kQ) * sizeof(uint32_t);
        static size_t attr = 48 * 1024;                   // (set once per size above the default)
        if (lds > attr) {
            const hipError_t e = hipFuncSetAttribute((const void*)mt_jump_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            attr = lds;
        }
        hipLaunchKernelGGL(mt_jump_kernel, dim3(a.Cj * a.S), dim3(kWave), lds, st, a);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(mt_gen_kernel, dim3(a.nchunks), dim3(kGen), 0, st, a);
    return hipGetLastError();
}

}  // namespace bcmpc
