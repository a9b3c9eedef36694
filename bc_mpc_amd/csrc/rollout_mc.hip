// rollout_mc.hip -- multi-column team kernel: weights resident in registers across a team of CUs,
// several 16-candidate columns per team in flight (software-pipelined).
//
// Path: MPCcontroller.get_action on the shard (controllers.py:57-88) for the plain 2-layer tanh
// NNDynamicsModel (dynamics.py:54-71: [S+A -> h] tanh, [h -> h] tanh, [h -> S] linear; hidden 449..512)
// with the fused cheetah cost (cost_functions.py:9-30, 59-63).  Same arithmetic as rollout_team.hip's
// T = 4 layout (hi/lo f16 operands, three MFMA passes, f32 accumulate, f64 state and
// cost; the same summation orders), so its costs are bit-identical to the team kernel's -- a different
// schedule for mid-size K (BASELINE cfg2, K = 4096), where the one-column team does not fit the chip
// (one team of 4 CUs per column) and rollout_x3 streams the whole 1.18-MB net from L2 into every CU
// every step for 16 candidates.
//
//   * A team = T = 4 workgroups (one per CU, 4 waves each, one 512-register wave per SIMD).  Team wave
//     g = member * 4 + w owns hidden tiles [2g, 2g + 2) and output-layer k-step g: those weights live in
//     its registers for the whole launch (272 VGPRs).  Layer 0 is computed whole by every member (its
//     32 tiles split over the 4 waves) from an LDS copy of the layer-0 weights (64 KiB).
//   * The team owns NCOL columns.  Column-steps X_j = (column j mod NCOLP, step j div NCOLP) flow
//     through a pipeline of four stages, one barrier per interval; in interval k:
//       C  X_{k+1}: gather the T members' output partials of the column's previous step (granules
//                   published >= 1 interval earlier), de-normalise + residual + cheetah cost (f64),
//                   normalise the next input, column power of two, its hi/lo B fragment into LDS.
//                   Spread over the 4 waves by candidate (wave w: candidates 4w..4w+3), each member
//                   redundantly (every member needs the fragment); state in a global scratch.
//       L0 X_k:     layer 0 (this wave's 8 tiles) + tanh epilogue into slab[k & 1].
//       L1 X_{k-1}: the hidden layer (this wave's 2 tiles x 16 k-steps x 3 passes) from slab[(k-1) & 1],
//                   its epilogue, the output layer's k-step -> the wave's partial into LDS.
//       P  X_{k-2}: the member partial (4 waves in wave order) published as {epoch, f32} granules
//                   (rollout_team.hip's exchange format and buffer, data = flag).
//     L0 and L1 are independent within an interval, so their MFMAs and epilogues interleave; the
//     exchange of a column-step has >= NCOLP - 3 intervals to land (NCOLP >= 4: ghost columns pad a
//     team with fewer).  A member waits only in C, for granules published at least one interval
//     earlier by every member, so no member can block another's progress (all members resident).
//   * Give-up: a member that polls past its limit (~1 s) raises the mapped error word and tags its
//     granules "dead" (rollout_team.hip); the host reruns the call on the fallback engine.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"
#include "split_common.h"

namespace bcmpc {

// MC_STAMP 1 (timing diagnostic, variant builds only): per-phase s_memtime totals of every wave into
// a.stamps ([blocks][4][10]: 0 C loads + publish, 1 L0 + L1 MFMAs with the C computation, 2 C epoch check
// (and a late granule's poll), 3 C stores, 4 L1 epilogue + out, 5 barrier, 9 prologue)
#ifndef MC_STAMP
#define MC_STAMP 0
#endif
#if MC_STAMP && !defined(BCMPC_DIAG_VARIANT)
#error "MC_STAMP is a timing diagnostic: build it with tools/build_variants.sh"
#endif

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int kHP = 512, kNT = 32, kP = 16, kNWV = 4, kT = 4, kTPW = 2, kL0T = 8, kL0P = 4;
constexpr int kMcSpins = 1 << 20;            // polls before a member gives up (~1 s)
constexpr uint64_t kRowsWaitTicks = 20000000;

// LDS (bytes)
constexpr int kOffB = kConstRows * kConstCols * 8;                   // biases: layer 0, 1 (x 2 log2 e), out
constexpr int kOffW0 = param_bytes(2, kHP);                           // layer-0 image: tile t at t * 2048
constexpr int kOffSlab = kOffW0 + kNT * 2048;                         // [2][P][hi|lo][64] f4
constexpr int kOffB0 = kOffSlab + 2 * kP * 2048;                      // [2][hi|lo][64][8] f16
constexpr int kOffColf = kOffB0 + 2 * 2048;                           // [2][16] f32
constexpr int kOffParts = kOffColf + 2 * 16 * 4;                      // [2][4 waves][2 tiles][64] f4
constexpr int kOffDead = kOffParts + 2 * kNWV * 2 * 1024;
constexpr int kLds = kOffDead + 16;
static_assert(kLds <= 160 * 1024, "LDS");

__device__ __forceinline__ f4 mm(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mm3(h8 ah, h8 al, h8 bh, h8 bl, f4 c) {
    c = mm(ah, bh, c);
    c = mm(ah, bl, c);
    return mm(al, bh, c);
}
// LDS hand-offs only (rollout_team.hip): the global loads in flight are not drained
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void rollout_mc(const RolloutArgs a) {
    extern __shared__ __attribute__((aligned(16))) f4 lds[];
    char* const base = reinterpret_cast<char*>(lds);
    double* const C = reinterpret_cast<double*>(base);
    float* const Bl = reinterpret_cast<float*>(base + kOffB);
    const f4* const W0 = reinterpret_cast<const f4*>(base + kOffW0);
    int* const deadf = reinterpret_cast<int*>(base + kOffDead);

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, m = lane & 15;
    const int S = a.S, A = a.A, H = a.H;
    const int bx = blockIdx.x;
    const int team = ((bx >> 3) / kT) * 8 + (bx & 7);     // members of a team: blocks b, b + 8, ... (one XCD)
    const int tm = (bx >> 3) % kT;
    const int g = tm * kNWV + w;                           // team wave: hidden tiles [2g, 2g + 2)
    const int64_t ncol = (a.K + 15) / 16;
    const int ncol_t = a.mc_ncol;
    const int NCOLP = ncol_t < 4 ? 4 : ncol_t;             // pipeline columns (ghosts pad small teams)
    const int64_t c0 = (int64_t)team * ncol_t;
    const int J = NCOLP * (H + 1);
    const unsigned gen = __hip_atomic_load(a.team_ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ---- parameters and the layer-0 weights into LDS (every load in flight before the stores) ----
    {
        const int t = threadIdx.x;
        constexpr int NCn = (kConstRows * kConstCols + 255) / 256;
        double rc[NCn];
        float rb[2][2], rbo;
#pragma unroll
        for (int u = 0; u < NCn; ++u) rc[u] = a.consts[min(t + u * 256, kConstRows * kConstCols - 1)];
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
            for (int u = 0; u < 2; ++u) rb[l][u] = a.b[l][t + u * 256];
        rbo = a.b[2][min(t, 31)];
        constexpr int NW0 = kNT * 2048 / 16 / 256;          // 16 f4 per thread
        f4 rw[NW0];
        const f4* src = reinterpret_cast<const f4*>(a.w[0]);
#pragma unroll
        for (int u = 0; u < NW0; ++u) rw[u] = src[t + u * 256];
#pragma unroll
        for (int u = 0; u < NCn; ++u)
            if (t + u * 256 < kConstRows * kConstCols) C[t + u * 256] = rc[u];
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
            for (int u = 0; u < 2; ++u) Bl[l * kHP + t + u * 256] = rb[l][u] * kTanhK;
        if (t < 32) Bl[2 * kHP + t] = rbo;
        f4* const w0d = reinterpret_cast<f4*>(base + kOffW0);
#pragma unroll
        for (int u = 0; u < NW0; ++u) w0d[t + u * 256] = rw[u];
        if (t == 0) *deadf = 0;
    }
    if (a.rows_flag && threadIdx.x == 0) {
        // late pre-draw hit (capi.cpp; as rollout_team.hip): wait for the worker's last row
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(a.rows_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != a.rows_seq) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kRowsWaitTicks) {
                if (a.team_err) __hip_atomic_store(a.team_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();

    uint64_t ph_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tp_ = MC_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if constexpr (MC_STAMP) {
            const uint64_t t_ = __builtin_amdgcn_s_memtime();
            ph_[k] += t_ - tp_;
            tp_ = t_;
        }
    };
    // ---- this wave's resident weights: hidden tiles [2g, 2g + 2) over all k-steps, output k-step g ----
    const int voff = lane * 16;
    h8 w1h[kP][kTPW], w1l[kP][kTPW], woh[2], wol[2];
    {
        const __amdgpu_buffer_rsrc_t r1 = layer_rsrc(a.w[1], a.wbytes[1]);
#pragma unroll
        for (int p = 0; p < kP; ++p)
#pragma unroll
            for (int j = 0; j < kTPW; ++j) {
                w1h[p][j] = fload(r1, voff, ((g * kP + p) * kTPW + j) * 2048);
                w1l[p][j] = fload(r1, voff, ((g * kP + p) * kTPW + j) * 2048 + 1024);
            }
        const __amdgpu_buffer_rsrc_t r2 = layer_rsrc(a.w[2], a.wbytes[2]);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            woh[v] = fload(r2, voff, (g * 2 + v) * 2048);
            wol[v] = fload(r2, voff, (g * 2 + v) * 2048 + 1024);
        }
    }

    const float f1 = a.winv[1] * kTanhK, fo = a.winv[2];
    const float* const Bout = Bl + 2 * kHP;
    gu64* const gb = (gu64*)a.team_buf;
    const unsigned dep = (gen << 10) | 1023u;              // this launch's "dead" epoch (never a step's)
    const int spin_limit = a.team_spins > 0 ? a.team_spins : kMcSpins;
    bool dead = false;
    // C-stage lane roles: candidate cm of the column, state dims e and e + 16
    const int cm = 4 * w + (lane >> 4), e = lane & 15;
    const int d1 = e + 16;
    const int lb = 16 * (e >> 2) + cm;                     // the D-fragment lane holding rows e, e + 16 of cm
    auto slab = [&](int k) __attribute__((always_inline)) {
        return reinterpret_cast<f4*>(base + kOffSlab + (k & 1) * kP * 2048);
    };
    auto parts = [&](int k) __attribute__((always_inline)) {
        return reinterpret_cast<f4*>(base + kOffParts + (k & 1) * kNWV * 2 * 1024);
    };

    stamp(9);
    // C-stage lanes: the D-fragment granule rows of dims e (k8 = e & 3) and e + 16 (4 + (e & 3)), lane lb
    const int ka = (e & 3) * 64 + lb, kb = (4 + (e & 3)) * 64 + lb;
    for (int k = -1; k <= J; ++k) {
        // (an opaque zero keeps the per-interval LDS table reads in the loop instead of hoisted registers)
        int wz = 0;
        asm volatile("" : "+s"(wz));
        const double* const Cz = C + wz;

        // ======== C (X_{k+1}): its global loads first -- state scratch, the T members' partials of the
        //          column's previous step, the HBM action -- their latency passes under the MFMA block ========
        const int jc = k + 1;
        const bool c_act = jc >= 0 && jc < J;
        const int cci = c_act ? jc % NCOLP : 0, ch = c_act ? jc / NCOLP : 0;
        const int64_t ccol = c0 + cci;
        const bool c_real = c_act && cci < ncol_t && ccol < ncol;
        const int64_t lcol = c_real ? ccol : 0;                // (ghosts load a real column's memory, discarded)
        const int64_t cand = lcol * 16 + cm;
        const bool valid = c_real && cand < a.K;
        double* const stp = a.mc_state + ((((size_t)lcol * kT + tm) * kNWV + w) * 3) * 64 + lane;
        const gu64* const src = gb + ((size_t)lcol * 2 + ((ch - 1) & 1)) * kT * 512;
        const unsigned epw = (gen << 10) + (unsigned)ch;      // epoch of the partials of step ch - 1
        const bool gather = c_real && ch > 0;
        const bool need1 = d1 < S;
        unsigned long long xa[kT], xb[kT];
        double st0 = 0.0, st1 = 0.0, stc = 0.0, av = 0.0;
        const int aj = min(max(d1 - S, 0), A - 1);
        if (gather) {
            st0 = stp[0];
            st1 = stp[64];
            stc = stp[128];
        }
#pragma unroll
        for (int t = 0; t < kT; ++t) {
            xa[t] = __hip_atomic_load(src + t * 512 + ka, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            xb[t] = __hip_atomic_load(src + t * 512 + kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.actions && valid && ch < H && d1 >= S && d1 < S + A)
            av = a.actions[((int64_t)ch * a.K + cand) * A + aj];

        // ======== P: publish the member partial of X_{k-2} ========
        {
            const int jp = k - 2;
            if (jp >= 0 && jp < J) {
                const int ci = jp % NCOLP, h = jp / NCOLP;
                const int64_t col = c0 + ci;
                if (ci < ncol_t && col < ncol && h < H) {
                    const f4* const pr = parts(jp);
                    const int v = w >> 1;
                    f4 s4 = pr[(0 * 2 + v) * 64 + lane];
#pragma unroll
                    for (int x = 1; x < kNWV; ++x) s4 += pr[(x * 2 + v) * 64 + lane];   // wave order
                    const unsigned ep = (gen << 10) + (unsigned)h + 1u;
                    gu64* const mine = gb + (((size_t)col * 2 + (h & 1)) * kT + tm) * 512;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int rr = 2 * (w & 1) + i;
                        if (!dead && 16 * v + 4 * q + rr < S)
                            __hip_atomic_store(mine + (4 * v + rr) * 64 + lane,
                                               ((unsigned long long)ep << 32) | __float_as_uint(s4[rr]),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        }
        stamp(0);

        // ---- the C computation of X_{k+1} from the loaded values (branch-free, so it interleaves with the
        //      MFMAs below; garbage for ghosts and h == 0 is discarded by selects / guarded stores) ----
        double s0, s1, cost;
        float x0, x1;
        int sh;
        auto c_compute = [&]() __attribute__((always_inline)) {
            float oa = __uint_as_float((unsigned)xa[0]), ob = __uint_as_float((unsigned)xb[0]);
#pragma unroll
            for (int t = 1; t < kT; ++t) {                 // member order (the same bits in every member)
                oa += __uint_as_float((unsigned)xa[t]);
                ob += __uint_as_float((unsigned)xb[t]);
            }
            const int64_t sc0 = valid ? cand : 0;           // (per-candidate initial states: no read past K)
            const double i0 = e < S ? (a.state_inline ? a.state_v[e] : a.state[sc0 * a.state_stride + e]) : 0.0;
            const double i1 = d1 < S ? (a.state_inline ? a.state_v[min(d1, S - 1)]
                                                       : a.state[sc0 * a.state_stride + min(d1, S - 1)]) : 0.0;
            // cheetah penalties on the state before the step (cost_functions.py:16-26): dims 5..7
            const bool pen = (e == 5 && st0 >= 0.2) || ((e == 6 || e == 7) && st0 >= 0.0);
            const unsigned long long bal = __ballot(pen);
            const int npen = __popcll((bal >> (16 * (lane >> 4))) & 0xFFFFull);
            // de-normalise + residual (dynamics.py:113,116), f64, no FMA (dims >= S: padded constants, unread)
            const float dn0 = fmaf(oa, fo, Bout[e]);
            const double u0 = __dadd_rn(st0, __dadd_rn(__dmul_rn((double)dn0, Cz[5 * 32 + e]), Cz[4 * 32 + e]));
            const float dn1 = fmaf(ob, fo, Bout[d1]);
            const double u1 = __dadd_rn(st1, __dadd_rn(__dmul_rn((double)dn1, Cz[5 * 32 + d1]), Cz[4 * 32 + d1]));
            const double score = __dsub_rn(10.0 * (double)npen, div_rn(__dsub_rn(u1, st1), 0.01, 1.0 / 0.01));
            const double uc = a.cost == BCMPC_COST_CHEETAH ? __dadd_rn(stc, score) : stc;
            s0 = ch == 0 ? i0 : u0;
            s1 = ch == 0 ? i1 : u1;
            cost = ch == 0 ? 0.0 : uc;                       // trajectory_cost = 0 (cost_functions.py:60)
            // the next layer-0 input: normalised state (dynamics.py:109) and action (:110), f32 (the TF feed),
            // the candidate's power of two (max |x| -> [2^11, 2^12))
            const double act = a.actions ? av : rng_action(a.seed, (uint64_t)(a.cand_offset + cand), ch, aj,
                                                           Cz[6 * 32 + aj], Cz[7 * 32 + aj]);
            const float xs0 = (float)div_rn(__dsub_rn(s0, Cz[0 * 32 + e]), Cz[1 * 32 + e], Cz[8 * 32 + e]);
            const float xs1 = (float)div_rn(__dsub_rn(s1, Cz[0 * 32 + d1]), Cz[1 * 32 + d1], Cz[8 * 32 + d1]);
            const float xa1 = (float)div_rn(__dsub_rn(act, Cz[2 * 32 + aj]), Cz[3 * 32 + aj], Cz[9 * 32 + aj]);
            x0 = valid ? xs0 : 0.f;
            x1 = !valid ? 0.f : d1 < S ? xs1 : d1 < S + A ? xa1 : 0.f;
            float mx = fmaxf(fabsf(x0), fabsf(x1));
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
            int ex = 0;
            (void)frexpf(mx, &ex);
            sh = 12 - ex;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
        };

        // ======== L0 (X_k) and L1 (X_{k-1}): unconditional (pipeline fill / drain and ghost columns compute on
        //          stale LDS; their outputs are only read by stages that are inactive too) ========
        f4 acc1[kTPW], acc1b[kTPW];
        {
            const f4* const sr = slab(k - 1);
            f4* const sw = slab(k);
            const _Float16* const b0b = reinterpret_cast<const _Float16*>(base + kOffB0 + (k & 1) * 2048);
            const h8 bh0 = *reinterpret_cast<const h8*>(b0b + lane * 8);
            const h8 bl0 = *reinterpret_cast<const h8*>(b0b + 512 + lane * 8);
            const float cf = reinterpret_cast<const float*>(base + kOffColf)[(k & 1) * 16 + m];
#pragma unroll
            for (int j = 0; j < kTPW; ++j) acc1[j] = acc1b[j] = (f4){0.f, 0.f, 0.f, 0.f};
            f4 acc0[kL0T];
#pragma unroll
            for (int j = 0; j < kL0T; ++j) {
                const int t = kL0T * w + j;
                acc0[j] = mm3(sread(W0 + t * 128 + lane), sread(W0 + t * 128 + 64 + lane), bh0, bl0,
                              (f4){0.f, 0.f, 0.f, 0.f});
            }
#pragma unroll
            for (int p = 0; p < kP; ++p) {
                const h8 bh = sread(sr + (p * 2 + 0) * 64 + lane), bl = sread(sr + (p * 2 + 1) * 64 + lane);
#pragma unroll
                for (int j = 0; j < kTPW; ++j) {
                    if (p & 1) acc1b[j] = mm3(w1h[p][j], w1l[p][j], bh, bl, acc1b[j]);
                    else acc1[j] = mm3(w1h[p][j], w1l[p][j], bh, bl, acc1[j]);
                }
                if (p % 4 == 3) {                          // a layer-0 tile pair's epilogue every 4 k-steps
                    const int pp = p / 4;
                    h8 xh, xl;
                    epi_pair_tanh(acc0[2 * pp], acc0[2 * pp + 1], cf, Bl, kL0T * w + 2 * pp, q, xh, xl);
                    swrite(sw + ((kL0P * w + pp) * 2 + 0) * 64 + lane, xh);
                    swrite(sw + ((kL0P * w + pp) * 2 + 1) * 64 + lane, xl);
                }
                if (p == 9) c_compute();                   // (in the MFMA stream: its loads have landed by now)
            }
#pragma unroll
            for (int j = 0; j < kTPW; ++j) acc1[j] += acc1b[j];
        }
        stamp(1);

        // ======== C: the epoch check; a late granule (rare) -> poll, then recompute ========
        if (gather) {
            bool ok = true;
#pragma unroll
            for (int t = 0; t < kT; ++t)
                ok &= (unsigned)(xa[t] >> 32) == epw && (!need1 || (unsigned)(xb[t] >> 32) == epw);
            if (!__all(ok) && !dead) {
                for (int spins = 0;; ++spins) {
                    __builtin_amdgcn_s_sleep(1);
                    bool ok2 = true;
#pragma unroll
                    for (int t = 0; t < kT; ++t) {
                        xa[t] = __hip_atomic_load(src + t * 512 + ka, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        xb[t] = __hip_atomic_load(src + t * 512 + kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok2 &= (unsigned)(xa[t] >> 32) == epw && (!need1 || (unsigned)(xb[t] >> 32) == epw);
                    }
                    if (__all(ok2)) break;
                    bool gone = *reinterpret_cast<volatile int*>(deadf) != 0;
                    if ((spins & 31) == 31)
#pragma unroll
                        for (int t = 0; t < kT; ++t)
                            gone = gone || (unsigned)(__hip_atomic_load(src + t * 512 + lane, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) >> 32) == dep;
                    if (__any(gone) || spins >= spin_limit) {
                        // give up: the mapped error word (the host reruns the call on its fallback engine), this
                        // member's other waves (LDS), the team (dead tags in granule row 0 of both parities of
                        // every column of the team: every poller reads it)
                        dead = true;
                        *reinterpret_cast<volatile int*>(deadf) = 1;
                        if (lane == 0 && a.team_err)
                            __hip_atomic_store(a.team_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        for (int c2 = 0; c2 < ncol_t && c0 + c2 < ncol; ++c2)
                            for (int par = 0; par < 2; ++par)
                                __hip_atomic_store(gb + (((size_t)(c0 + c2) * 2 + par) * kT + tm) * 512 + lane,
                                                   (unsigned long long)dep << 32, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                c_compute();
            }
        }
        stamp(2);
        if (c_real) {
            const bool writer = tm == 0 && valid;
            if (writer && a.traj) {
                if (e < S) a.traj[((int64_t)ch * a.K + cand) * S + e] = s0;
                if (d1 < S) a.traj[((int64_t)ch * a.K + cand) * S + d1] = s1;
            }
            if (ch == H) {
                if (writer && e == 1 && a.costs) a.costs[cand] = cost;
            } else {
                const float sc = ldexpf(1.0f, sh);
                const float y0 = x0 * sc, y1 = x1 * sc;
                const _Float16 h0 = (_Float16)y0, h1 = (_Float16)y1;
                const _Float16 l0 = (_Float16)(y0 - (float)h0), l1 = (_Float16)(y1 - (float)h1);
                _Float16* const b0w = reinterpret_cast<_Float16*>(base + kOffB0 + (jc & 1) * 2048);
                b0w[lb * 8 + (e & 3)] = h0;
                b0w[lb * 8 + 4 + (e & 3)] = h1;
                b0w[512 + lb * 8 + (e & 3)] = l0;
                b0w[512 + lb * 8 + 4 + (e & 3)] = l1;
                if (e == 0)
                    reinterpret_cast<float*>(base + kOffColf)[(jc & 1) * 16 + cm] = ldexpf(a.winv[0], -sh) * kTanhK;
                stp[0] = s0;
                stp[64] = s1;
                stp[128] = cost;
            }
        }
        stamp(3);
        // ======== L1 (X_{k-1}): epilogue, output layer k-step, the wave's partial ========
        {
            h8 oh, ol;
            epi_pair_tanh(acc1[0], acc1[1], f1, Bl + kHP, kTPW * g, q, oh, ol);
            f4 po[2];
#pragma unroll
            for (int v = 0; v < 2; ++v) po[v] = mm3(woh[v], wol[v], oh, ol, (f4){0.f, 0.f, 0.f, 0.f});
            f4* const pw = parts(k - 1);
            pw[(w * 2 + 0) * 64 + lane] = po[0];
            pw[(w * 2 + 1) * 64 + lane] = po[1];
        }
        stamp(4);
        lds_barrier();
        dead = dead || *reinterpret_cast<volatile int*>(deadf) != 0;
        stamp(5);
    }
    if constexpr (MC_STAMP) {
        if (a.stamps && lane == 0)
            for (int k2 = 0; k2 < 10; ++k2) a.stamps[((size_t)blockIdx.x * 4 + w) * 10 + k2] = ph_[k2];
    }

    // the launch's last workgroup advances the generation (every workgroup read it at its start)
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(a.team_ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            __hip_atomic_store(a.team_ctl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.team_ctl + 1, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

bool mc_shape_ok(int hidden_padded, int n_layers, int state_dim, int action_dim, int horizon) {
    return hidden_padded == kHP && n_layers == 2 && state_dim >= 18 && state_dim + action_dim <= 32 &&
           action_dim >= 1 && horizon >= 1 && horizon <= 1022;
}
int mc_members() { return kT; }
int mc_teams(int64_t K, int n_cu) {
    const int64_t ncol = (K + 15) / 16;
    int teams = (n_cu / kT) / 8 * 8;                       // one workgroup per CU, a multiple of 8 teams
    if (teams < 8) return 0;
    const int64_t need = (ncol + 3) / 4;                   // at least 4 columns per team when K allows
    while (teams > 8 && (int64_t)(teams - 8) >= need) teams -= 8;
    return teams;
}
int mc_columns_per_team(int64_t K, int n_cu) {
    const int t = mc_teams(K, n_cu);
    return t ? (int)(((K + 15) / 16 + t - 1) / t) : 0;
}
size_t mc_state_bytes(int64_t K, int n_cu) {
    const int t = mc_teams(K, n_cu);
    return t ? (size_t)t * mc_columns_per_team(K, n_cu) * kT * kNWV * 3 * 64 * sizeof(double) : 0;
}

hipError_t launch_rollout_mc(const RolloutArgs& a, hipStream_t st) {
    static bool attr_set = false;
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void*)rollout_mc, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (!mc_shape_ok(kHP, a.L, a.S, a.A, a.H) || a.model != BCMPC_MODEL_DELTA || a.pL > 0 || a.ln ||
        a.act != BCMPC_ACT_TANH || a.f16_single || a.cem_mu || !a.team_buf || !a.team_ctl || !a.mc_state ||
        a.mc_nteam < 8 || a.mc_nteam % 8 || a.mc_ncol < 1 || (int64_t)a.mc_nteam * a.mc_ncol * 16 < a.K ||
        a.wbytes[0] < kNT * 2048)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(rollout_mc, dim3((unsigned)(a.mc_nteam * kT)), dim3(256), (size_t)kLds, st, a);
    return hipGetLastError();
}

}  // namespace bcmpc
