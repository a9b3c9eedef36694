// cem.hip -- CEM outer loop kernels (DESIGN.md "CEM"): elite selection and the
// mean / std refit.  The per-iteration rollout is the ordinary rollout kernel
// with CEM action sampling (cem_action, device_common.h).
//
// select_kernel: the n_elite smallest records under the total order
//   (orderable(cost), index) -- NaN after every number, ties to the lower index,
//   i.e. np.argsort(costs, kind="stable")[:E] -- by an 8-pass radix select on the
//   64-bit orderable cost (LDS histograms), then an index-ordered compaction
//   (block scans), so the output is in ascending index order whatever the input
//   sharding.  One 1024-thread block; the input (K or ranks*E records, <= a few MB)
//   is re-read from L2 per pass.
//
// refit_kernel: one wave per (h, j).  Lane l regenerates the actions of elites
//   l, l+64, ... (Philox, no stored action tensor) and sums them in that order; the
//   64 partials are combined by the xor butterfly (offsets 32..1); mean = sum / n.
//   Second pass the same for (a - mean)^2; std = sqrt(var / n) (np.std, ddof 0).
//   mu' = alpha*mu + (1-alpha)*mean, sigma' likewise.  f64, no FMA, fixed order
//   (restated by oracle.cem_refit).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"

namespace bcmpc {

// total order on f64 (NaN greatest, -0 == +0), as an unsigned key
__device__ __forceinline__ uint64_t orderable(double c) {
    if (c != c) return ~0ull;
    if (c == 0.0) c = 0.0;                             // -0 == +0, as np.argsort compares them
    const uint64_t b = __double_as_longlong(c);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// exclusive prefix sum of one flag per thread over the 1024-thread block, and the total
__device__ __forceinline__ int block_scan(int flag, int* wsum, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t bal = __ballot(flag);
    const int inwave = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int before = 0;
    total = 0;
    for (int k = 0; k < 16; ++k) {
        const int v = wsum[k];
        before += k < w ? v : 0;
        total += v;
    }
    __syncthreads();                                   // wsum is reused by the next call
    return before + inwave;
}

__global__ __launch_bounds__(1024) void select_kernel(const SelectArgs a) {
    __shared__ uint32_t hist[256];
    __shared__ int wsum[16];
    __shared__ uint64_t s_prefix;
    __shared__ int64_t s_remaining;
    __shared__ uint32_t s_valid;
    const int tid = threadIdx.x;

    auto rec = [&](int64_t i, uint64_t& key, int64_t& idx, double& cost) -> bool {
        if (a.pairs) {
            cost = a.pairs[i].cost;
            idx = a.pairs[i].index;
        } else {
            cost = a.costs[i];
            idx = a.index_base + i;
        }
        key = orderable(a.maximize ? -cost : cost);
        return idx >= 0;
    };

    if (tid == 0) { s_valid = 0; s_prefix = 0; }
    __syncthreads();
    {   // count valid records
        uint32_t n = 0;
        for (int64_t i = tid; i < a.m; i += blockDim.x) {
            uint64_t k; int64_t ix; double c;
            n += rec(i, k, ix, c) ? 1u : 0u;
        }
        atomicAdd(&s_valid, n);
    }
    __syncthreads();
    const int64_t E = a.n_elite < (int64_t)s_valid ? a.n_elite : (int64_t)s_valid;
    if (tid == 0) s_remaining = E;
    uint64_t mask = 0;
    for (int pass = 0; pass < 8 && E > 0; ++pass) {
        const int shift = 56 - 8 * pass;
        for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        const uint64_t prefix = s_prefix;
        for (int64_t i = tid; i < a.m; i += blockDim.x) {
            uint64_t k; int64_t ix; double c;
            if (rec(i, k, ix, c) && (k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid == 0) {                                // digit where the cumulative count reaches `remaining`
            int64_t rem = s_remaining, cum = 0;
            int d = 0;
            for (; d < 256; ++d) {
                if (cum + hist[d] >= rem) break;
                cum += hist[d];
            }
            s_remaining = rem - cum;
            s_prefix = prefix | ((uint64_t)d << shift);
        }
        mask |= 255ull << shift;
        __syncthreads();
    }
    // threshold key T; take every record below T and the first `need_eq` (by index) equal to T
    const uint64_t T = s_prefix;
    const int64_t need_eq = s_remaining;
    int64_t base = 0, eq_taken = 0;
    for (int64_t tile = 0; tile < a.m && E > 0; tile += blockDim.x) {
        const int64_t i = tile + tid;
        uint64_t k = 0; int64_t ix = -1; double c = 0.0;
        const bool v = i < a.m && rec(i, k, ix, c);
        const int is_eq = v && k == T;
        int tot_eq;
        const int eq_rank = block_scan(is_eq, wsum, tot_eq);
        const int sel = (v && k < T) || (is_eq && eq_taken + eq_rank < need_eq);
        int tot_sel;
        const int pos = block_scan(sel, wsum, tot_sel);
        if (sel) a.out[base + pos] = bcmpc_elite{c, ix};
        base += tot_sel;
        eq_taken += tot_eq;
    }
    for (int64_t i = E + tid; i < a.n_elite; i += blockDim.x) a.out[i] = bcmpc_elite{__builtin_nan(""), -1};
    if (tid == 0) *a.count = (int32_t)E;
}

__global__ __launch_bounds__(64) void refit_kernel(const RefitArgs a) {
    const int b = blockIdx.x;                          // b = h * A + j
    const int h = b / a.A, j = b - h * a.A;
    const int lane = threadIdx.x;
    const int n = *a.count;
    if (n <= 0) return;                                // nothing selected: distribution unchanged
    const double mu0 = a.mu[b], sd0 = a.sigma[b];
    const double lo = a.consts[6 * kConstCols + j], hi = a.consts[7 * kConstCols + j];
    double s = 0.0;
    for (int e = lane; e < n; e += 64)
        s = __dadd_rn(s, cem_action(a.seed, (uint64_t)a.elite[e].index, h, j, a.iter, mu0, sd0, lo, hi));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s = __dadd_rn(s, __shfl_xor(s, off));
    const double mean = __ddiv_rn(s, (double)n);
    double v = 0.0;
    for (int e = lane; e < n; e += 64) {
        const double d = __dsub_rn(cem_action(a.seed, (uint64_t)a.elite[e].index, h, j, a.iter, mu0, sd0, lo, hi),
                                   mean);
        v = __dadd_rn(v, __dmul_rn(d, d));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = __dadd_rn(v, __shfl_xor(v, off));
    const double sd = __dsqrt_rn(__ddiv_rn(v, (double)n));
    if (lane == 0) {
        const double beta = __dsub_rn(1.0, a.alpha);
        a.mu[b] = __dadd_rn(__dmul_rn(a.alpha, mu0), __dmul_rn(beta, mean));
        a.sigma[b] = __dadd_rn(__dmul_rn(a.alpha, sd0), __dmul_rn(beta, sd));
    }
}

hipError_t launch_select(const SelectArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(select_kernel, dim3(1), dim3(1024), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_refit(const RefitArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(refit_kernel, dim3((unsigned)(a.H * a.A)), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace bcmpc
