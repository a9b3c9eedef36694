// rollout_rr.hip -- "resident-column" split-f16 rollout kernel (BCMPC_KERNEL_SPLITR) for the
// headline net: NNDynamicsModel with two dense layers [S+A -> h] tanh, [h -> h] tanh and the
// linear [h -> S] output (dynamics.py:54-71), hidden padded to 64..512, no policy / reward
// net.  Same contract and arithmetic as rollout_x3 (one launch = one MPCcontroller.get_action on
// the shard, controllers.py:57-88; split-f16 operands, three MFMA passes, f64 state / cost), a
// different work split:
//
//   * Each wave owns one column of 16 candidates OUTRIGHT: the layer-1 input of its
//     candidates (hi + lo f16 B fragments of all HP/32 k-steps, 128 VGPRs at HP = 512) stays
//     in its registers, and the layer-1 output tiles are formed one at a time and folded
//     straight into the output layer (a tile pair's accumulators ARE one output-layer k-step's
//     B fragment).  No activation crosses LDS and no wave waits for another wave's epilogue:
//     the per-layer slab hand-off of rollout_x3 (lock-step, 52% MFMA-busy at cfg3) is gone.
//   * The weights are the only shared operand.  The host lays them out as one image of
//     NS = 2 + HP/16 "slots" per step (layer 0 in two halves, then one layer-1 tile per slot; the
//     slots also carry the output layer's fragments, see RrGeom).  A workgroup of RR_NWV waves
//     streams the image every step through a two-buffer LDS ring: each wave loads its share of
//     slot i+2 into registers (buffer_load) and writes slot i+1 into LDS (ds_write_b128) at the
//     barrier that opens slot i, and every wave reads its A fragments from LDS.
//   * Software pipeline: the tanh epilogue of layer-1 tile pair j and its output-layer MFMAs
//     run while tile pair j+1's MFMAs are in flight (independent instructions of one wave).
//
// Status: parity-green and opt-in (BCMPC_KERNEL_SPLITR).  At cfg3 it runs 2.03 ms
// against rollout_x3's 1.90 ms.  With one column per wave every wave reads every weight fragment
// from LDS (8 waves x 32 KiB per tile slot: the LDS array is busy ~90% of the slot), and with two
// columns per wave (RR_NCOL = 2, 512-register waves) the 256-register resident operand spills
// (3.06 ms).  An earlier LDS-DMA ring (global_load_lds_dwordx4) lost to ~100 cycles of issue per
// 1-KiB piece (s_memtime stamps: 21.7k of 126k cycles per step).
//
// Ring protocol: slot i's LDS image is complete when every wave has passed the barrier that opens
// slot i (each wave's ds_writes of it were issued before, and waited by the lgkmcnt(0) in front
// of the barrier); the same barrier proves slot i-1 read by every wave, so slot i+1 may overwrite
// its buffer.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"
#include "split_common.h"

namespace bcmpc {

namespace {

// slot geometry of the weight image (capi.cpp pack_rr_image): per step NS = 2 + T slots of
// 2P + 4 1-KiB pieces: slot 0 = layer-0 tiles [0, P) + the output layer's four fragments (tile 0
// hi, lo, tile 1 hi, lo) at k-step P-1; slot 1 = layer-0 tiles [P, 2P) + four zero pieces; slot
// 2 + t = layer-1 tile t (P k-steps, hi | lo) + output tile t & 1 (hi, lo) at k-step t/2 - 1
// (zero for t < 2) + two zero pieces.
template <int HP>
struct RrGeom {
    static constexpr int P = HP / 32;          // k-steps of a layer-1 tile
    static constexpr int T = HP / 16;          // tiles of a hidden layer
    static constexpr int SLOTP = 2 * P + 4;    // 1-KiB pieces per slot
    static constexpr int SLOTB = SLOTP * 1024;
    static constexpr int NS = 2 + T;           // slots per step
};

__device__ __forceinline__ void ring_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ f4 mm(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

__device__ __forceinline__ h8 lread(const char* p) { return *reinterpret_cast<const h8*>(p); }

}  // namespace

// timing-only diagnostics (results wrong), built by tools/rr_variants.sh only: 1 no ring waits /
// barriers, 2 no DMA issue (stale ring), 4 no layer-1 MFMAs, 8 A fragments not read from LDS,
// 16 no layer-0 epilogue; RR_STAMP 1: per-phase s_memtime totals per wave into a.stamps
// ([blocks][NWV][10]: 0 ring barrier, 1 layer-0 slots, 2 layer-1 slots, 3 step head / tail, 4 DMA
// vmcnt waits, 5 DMA issue); RR_DIAG 32 no vmcnt waits (barrier kept), 64 no barrier (waits kept)
#ifndef RR_STAMP
#define RR_STAMP 0
#endif
#ifndef RR_DIAG
#define RR_DIAG 0
#endif
#if (RR_DIAG || RR_STAMP) && !defined(BCMPC_DIAG_VARIANT)
#error "RR_DIAG is a timing-only diagnostic: build it with tools/rr_variants.sh"
#endif

#ifndef RR_PF
#define RR_PF 2                  // layer-1 A fragments in flight ahead of their MFMAs (k-steps)
#endif

// RR_NWV waves of 16 candidates per workgroup (8: one 128-candidate workgroup per CU, one weight
// stream per CU; 4: two 64-candidate workgroups per CU, independent phases, two weight streams)
#ifndef RR_NWV
#define RR_NWV 8
#endif
#ifndef RR_NCOL                  // 16-candidate columns per wave (2: 512-register waves, one per SIMD)
#define RR_NCOL 1
#endif
__host__ __device__ constexpr int rr_lds_bytes(int HP) { return param_bytes(2, HP) + 2 * (HP / 16 + 5) * 1024; }

template <int HP, int NWV, int NCOL>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NCOL == 1 ? 2 : 1, NCOL == 1 ? 2 : 1)))
void rollout_rr(const RolloutArgs a) {
    using G = RrGeom<HP>;
    constexpr int P = G::P, SLOTP = G::SLOTP, SLOTB = G::SLOTB, NS = G::NS;
    constexpr int SLOTB1 = SLOTB + 1024;                     // LDS buffer: the slot + one dummy piece
    constexpr int CB = 16 * NCOL * NWV;                      // candidates per workgroup
    constexpr int NPW = (SLOTP + NWV - 1) / NWV;             // pieces per slot of waves w < SLOTP % NWV
    static_assert(P % 2 == 0, "tile pairs alternate between two accumulator sets");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, m = lane & 15;
    const int S = a.S, A = a.A;

    double* C = reinterpret_cast<double*>(lds);
    float* Bl = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kConstRows * kConstCols * 8);
    for (int i = threadIdx.x; i < kConstRows * kConstCols; i += blockDim.x) C[i] = a.consts[i];
    for (int l = 0; l < 2; ++l)
        for (int i = threadIdx.x; i < HP; i += blockDim.x) Bl[l * HP + i] = a.b[l][i] * kTanhK;
    float* const Bout = Bl + 2 * HP;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) Bout[i] = a.b[2][i];
    char* const ring = reinterpret_cast<char*>(lds) + param_bytes(2, HP);

    // ---- weight ring: slot i of the launch = image slot i % NS in LDS buffer i % 2.  Each wave owns
    //      pieces k = w + u NWV of every slot and stages them through registers one slot ahead: at
    //      acquire(i) it writes slot i+1 (loaded at acquire(i-1)) and loads slot i+2.  Pieces past
    //      SLOTP read beyond the buffer's range (zeros) into a dummy piece of the LDS buffer. ----
    const __amdgpu_buffer_rsrc_t wrs = layer_rsrc(a.w[0], a.wbytes[0]);
    const int voff = lane * 16;
    h8 stg[NPW];
    int i_load = 0;
    auto load = [&]() __attribute__((always_inline)) {
        const int j = i_load % NS;
        ++i_load;
#pragma unroll
        for (int u = 0; u < NPW; ++u) {
            const int k = w + u * NWV;
            const int off = k < SLOTP ? j * SLOTB + k * 1024 : 0x7FFFF000;   // (beyond num_records: zeros)
            if constexpr (RR_DIAG & 2) stg[u] = (h8)(_Float16)0.0f;
            else stg[u] = fload(wrs, voff, off);
        }
    };
    auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < NPW; ++u) {
            const int k = w + u * NWV;
            *reinterpret_cast<h8*>(ring + buf * SLOTB1 + (k < SLOTP ? k : SLOTP) * 1024 + lane * 16) = stg[u];
        }
    };
    uint64_t ph_[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tp_ = RR_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if constexpr (RR_STAMP) {
            const uint64_t t_ = __builtin_amdgcn_s_memtime();
            ph_[k] += t_ - tp_;
            tp_ = t_;
        }
    };
    // acquire slot i of parity PAR (known at every call site): one barrier (slot i complete in
    // buffer PAR, slot i-1 read by every wave), then stage slot i+1 into buffer 1-PAR, load slot i+2
    auto acquire = [&](int ph, auto PARc) __attribute__((always_inline)) -> const char* {
        constexpr int PAR = decltype(PARc)::value;
        stamp(ph);
        if constexpr (!(RR_DIAG & 64)) ring_barrier();
        stamp(0);
        store(1 - PAR);
        load();
        stamp(5);
        return ring + PAR * SLOTB1;
    };
    load();
    store(0);
    load();

    // ---- per-candidate state: lane (q, m) holds dims 16 v + 4 q + r (v = 0, 1) of candidate m ----
    int64_t cand[NCOL];
    bool valid[NCOL];
    double s[NCOL][2][4];
    double cost[NCOL];                                          // trajectory_cost = 0 (cost_functions.py:60)
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
        cand[c] = (int64_t)blockIdx.x * CB + (w * NCOL + c) * 16 + m;
        valid[c] = cand[c] < a.K;
        cost[c] = 0.0;
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                s[c][v][r] = (valid[c] && d < S)
                                 ? (a.state_inline ? a.state_v[d] : a.state[cand[c] * a.state_stride + d]) : 0.0;
                if (a.traj && valid[c] && d < S) a.traj[cand[c] * S + d] = s[c][v][r];
            }
    }

    // ---- actions of step h, normalised (dynamics.py:110) and cast to f32 (the TF feed), in the
    //      lanes whose dims 16 v + 4 q + r are action dims: the caller's [H,K,A] array
    //      (np.random.uniform, controllers.py:53), Philox (rng_action), or the CEM sampler ----
    float xa[NCOL][2][4];
    auto act4 = [&](int h, int c, int v, float (&out)[4]) __attribute__((always_inline)) {
        const uint64_t gcand = (uint64_t)(a.cand_offset + cand[c]);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = 0.f;
        const int j0 = 16 * v + 4 * q - S;                       // action index of slot r = 0
        if (valid[c] && h < a.H && j0 + 3 >= 0 && j0 < A) {
            if (!a.actions && !a.cem_mu) {
                // Philox block j >> 1 yields actions 2 (j >> 1) and 2 (j >> 1) + 1 (rng_action)
                const int jb0 = j0 >> 1, nb = (S & 1) ? 3 : 2;
#pragma unroll
                for (int bb = 0; bb < 3; ++bb) {
                    const int jb = jb0 + bb;
                    if (bb < nb && 2 * jb + 1 >= 0 && 2 * jb < A) {
                        uint32_t ctr[4] = {(uint32_t)gcand, (uint32_t)(gcand >> 32), (uint32_t)h, (uint32_t)jb};
                        philox4x32_10(ctr, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int j = j0 + r;
                            if ((j >> 1) == jb && j >= 0 && j < A) {
                                const uint32_t x = (j & 1) ? ctr[2] : ctr[0], y = (j & 1) ? ctr[3] : ctr[1];
                                const double u =
                                    ((double)(x >> 5) * 67108864.0 + (double)(y >> 6)) / 9007199254740992.0;
                                const double lo = C[6 * 32 + j], hi = C[7 * 32 + j];
                                const double av = __dadd_rn(lo, __dmul_rn(__dsub_rn(hi, lo), u));
                                out[r] = (float)div_rn(__dsub_rn(av, C[2 * 32 + j]), C[3 * 32 + j], C[9 * 32 + j]);
                            }
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = j0 + r;
                    if (j >= 0 && j < A) {
                        const double av = a.cem_mu ? cem_action(a.seed, gcand, h, j, a.cem_iter, a.cem_mu[h * A + j],
                                                                a.cem_sigma[h * A + j], C[6 * 32 + j], C[7 * 32 + j])
                                                   : a.actions[((int64_t)h * a.K + cand[c]) * A + j];
                        out[r] = (float)div_rn(__dsub_rn(av, C[2 * 32 + j]), C[3 * 32 + j], C[9 * 32 + j]);
                    }
                }
            }
        }
    };
    auto actions = [&](int h) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
            act4(h, c, 0, xa[c][0]);
            act4(h, c, 1, xa[c][1]);
        }
    };

    const float f1 = a.winv[1] * kTanhK;                         // layer-1 result scale x 2 log2 e
    const float fo = a.winv[2];
    h8 xh[P][NCOL], xl[P][NCOL];                                 // layer-1 input of this wave's candidates
    f4 accA[2][NCOL], accB[2][NCOL];                             // tile pairs alternate between the two
    h8 ob[NCOL][2];                                              // layer-1 output pair (hi, lo) = output B fragment
    f4 po[2][NCOL];                                              // output layer [h -> S]: two 16-row tiles

    // one layer-1 tile from the slot's P k-steps (A fragments read RR_PF k-steps ahead of their
    // MFMAs; sched_barrier keeps the scheduler from sinking the reads next to their use under the
    // register pressure of the resident B operand)
    auto l1_tile = [&](const char* sl, f4 (&acc)[NCOL]) __attribute__((always_inline)) {
        const char* base = sl + lane * 16;
#pragma unroll
        for (int c = 0; c < NCOL; ++c) acc[c] = (f4){0.f, 0.f, 0.f, 0.f};
        h8 fh[RR_PF], fl[RR_PF];
#pragma unroll
        for (int p = 0; p < RR_PF && p < P; ++p) {
            fh[p] = lread(base + p * 2048);
            fl[p] = lread(base + p * 2048 + 1024);
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const h8 ah = fh[p % RR_PF], al = fl[p % RR_PF];
            if (p + RR_PF < P && !(RR_DIAG & 8)) {
                fh[p % RR_PF] = lread(base + (p + RR_PF) * 2048);
                fl[p % RR_PF] = lread(base + (p + RR_PF) * 2048 + 1024);
            }
#pragma unroll
            for (int c = 0; c < NCOL; ++c) {
                if constexpr (RR_DIAG & 4) {
                    acc[c] += (f4){(float)ah[0], (float)xh[p][c][0], (float)al[1], (float)xl[p][c][1]};
                } else {
                    acc[c] = mm(ah, xh[p][c], acc[c]);
                    acc[c] = mm(ah, xl[p][c], acc[c]);
                    acc[c] = mm(al, xh[p][c], acc[c]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // layer-1 pair pp's epilogue (tanh, split): the output layer's B fragment of k-step pp
    auto l1_epi = [&](const f4 (&acc)[2][NCOL], int pp) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NCOL; ++c) epi_pair_tanh(acc[0][c], acc[1][c], f1, Bl + HP, 2 * pp, q, ob[c][0], ob[c][1]);
    };
    // output tile v += its (hi, lo) fragment at the slot's piece pc x ob
    auto out_mm = [&](const char* sl, int pc, int v) __attribute__((always_inline)) {
        const h8 ah = lread(sl + (2 * P + pc) * 1024 + lane * 16), al = lread(sl + (2 * P + pc + 1) * 1024 + lane * 16);
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
            po[v][c] = mm(ah, ob[c][0], po[v][c]);
            po[v][c] = mm(ah, ob[c][1], po[v][c]);
            po[v][c] = mm(al, ob[c][0], po[v][c]);
        }
    };
    // one tile pair: slots of tiles 2pp (parity 0) and 2pp+1 (parity 1); the previous pair's
    // epilogue + output MFMAs (fragments carried by these two slots) run beside their MFMAs
    auto l1_pair = [&](int pp, f4 (&accN)[2][NCOL], const f4 (&accO)[2][NCOL]) __attribute__((always_inline)) {
        const char* sl = acquire(pp == 0 ? 1 : 2, std::integral_constant<int, 0>{});
        l1_tile(sl, accN[0]);
        if (pp > 0) {
            l1_epi(accO, pp - 1);
            out_mm(sl, 0, 0);
        }
        sl = acquire(2, std::integral_constant<int, 1>{});
        l1_tile(sl, accN[1]);
        if (pp > 0) out_mm(sl, 0, 1);
    };

    for (int h = 0;; ++h) {
        // ---- slot 0 of the step: layer-0 tiles [0, P) + the last pair's output fragments ----
        const char* s0 = acquire(h == 0 ? 3 : 2, std::integral_constant<int, 0>{});
        if (h > 0) {
            // ---- tail of step h-1: last pair's epilogue + output MFMAs, de-normalise + residual
            //      (dynamics.py:113,116; f64, no FMA), cheetah cost (cost_functions.py:12-28) ----
            l1_epi(accB, P - 1);
            out_mm(s0, 0, 0);
            out_mm(s0, 2, 1);
#pragma unroll
            for (int c = 0; c < NCOL; ++c) {
                // penalties on the current state: dims 5, 6, 7 live in lane row q = 1 (v = 0); the
                // reference adds 0 + 10 + 10 + 10 in order, exactly 10 * count
                const int npen =
                    partner_row16((s[c][0][1] >= 0.2) + (s[c][0][2] >= 0.0) + (s[c][0][3] >= 0.0));
                const double s17 = s[c][1][1];                    // dim 17: v = 1, row q = 0, r = 1
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const f4 bv = *reinterpret_cast<const f4*>(Bout + 16 * v + 4 * q);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * v + 4 * q + r;
                        if (d < S) {
                            const float dn = fmaf(po[v][c][r], fo, bv[r]);             // BiasAdd (f32)
                            const double ud = __dadd_rn(__dmul_rn((double)dn, C[5 * 32 + d]), C[4 * 32 + d]);
                            s[c][v][r] = __dadd_rn(s[c][v][r], ud);
                        }
                    }
                }
                if (a.cost == BCMPC_COST_CHEETAH) {
                    // score = pen - (s'17 - s17) / 0.01 (cost_functions.py:28), summed in step order (:59-63)
                    const double score =
                        __dsub_rn(10.0 * (double)npen, div_rn(__dsub_rn(s[c][1][1], s17), 0.01, 1.0 / 0.01));
                    cost[c] = __dadd_rn(cost[c], score);
                }
                if (a.traj && valid[c]) {
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int d = 16 * v + 4 * q + r;
                            if (d < S) a.traj[((int64_t)h * a.K + cand[c]) * S + d] = s[c][v][r];
                        }
                }
            }
        }
        if (h == a.H) break;
        actions(h);
        // ---- layer-0 input: normalised state (dynamics.py:109) and action, cast to f32; per
        //      candidate the power of two that puts max |x| in [2^11, 2^12) (undone in the epilogue) ----
        h8 b0h[NCOL], b0l[NCOL];
        float colf[NCOL];
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
            float x[8];
            float mx = 0.f;
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int d = 16 * v + 4 * q + r;
                    float xv = xa[c][v][r];
                    if (d < S)
                        xv = (float)div_rn(__dsub_rn(s[c][v][r], C[0 * 32 + d]), C[1 * 32 + d], C[8 * 32 + d]);
                    x[4 * v + r] = xv;
                    mx = fmaxf(mx, fabsf(xv));
                }
            mx = max_rows32(max_rows16(mx));
            int e = 0;
            (void)frexpf(mx, &e);                                // mx in [2^(e-1), 2^e)
            int sh = 12 - e;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
            const float sc = ldexpf(1.0f, sh);
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] *= sc;
            split8(x, b0h[c], b0l[c]);
            colf[c] = ldexpf(a.winv[0], -sh) * kTanhK;
        }
        // ---- layer 0 [S+A -> h]: T tiles of one k-step in two slots, pairs epilogued into the
        //      layer-1 input ----
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const char* sl = half == 0 ? s0 : acquire(1, std::integral_constant<int, 1>{});
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int t = half * P + u;
                const h8 ah = lread(sl + u * 2048 + lane * 16), al = lread(sl + u * 2048 + 1024 + lane * 16);
#pragma unroll
                for (int c = 0; c < NCOL; ++c) {
                    f4 acc = mm(ah, b0h[c], (f4){0.f, 0.f, 0.f, 0.f});
                    acc = mm(ah, b0l[c], acc);
                    accA[t & 1][c] = mm(al, b0h[c], acc);
                    if (t & 1) {
                        if constexpr (RR_DIAG & 16) {
                            xh[t >> 1][c] = __builtin_bit_cast(h8, accA[0][c]);
                            xl[t >> 1][c] = __builtin_bit_cast(h8, accA[1][c]);
                        } else {
                            epi_pair_tanh(accA[0][c], accA[1][c], colf[c], Bl, t - 1, q, xh[t >> 1][c], xl[t >> 1][c]);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NCOL; ++c) po[0][c] = po[1][c] = (f4){0.f, 0.f, 0.f, 0.f};
        // ---- layer 1 [h -> h], tile pairs alternating accumulator sets ----
        for (int pp = 0; pp < P; pp += 2) {
            l1_pair(pp, accA, accB);
            l1_pair(pp + 1, accB, accA);
        }
    }
    stamp(3);
    if constexpr (RR_STAMP) {
        if (a.stamps && lane == 0)
            for (int k = 0; k < 6; ++k) a.stamps[((size_t)blockIdx.x * NWV + w) * 10 + k] = ph_[k];
    }
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
        if (a.costs && valid[c] && q == 0) a.costs[cand[c]] = cost[c];
}

template <int HP>
static hipError_t launch_rr_t(const RolloutArgs& a, hipStream_t st) {
    constexpr int lds = rr_lds_bytes(HP);
    static_assert(lds <= 160 * 1024, "LDS: ring + parameters");
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)rollout_rr<HP, RR_NWV, RR_NCOL>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (a.L != 2 || a.act != BCMPC_ACT_TANH || a.ln || a.model != BCMPC_MODEL_DELTA || a.pL != 0 || a.S + a.A > 32 ||
        (a.cost == BCMPC_COST_CHEETAH && a.S < 18) ||
        (int64_t)a.wbytes[0] < (int64_t)RrGeom<HP>::NS * RrGeom<HP>::SLOTB)
        return hipErrorInvalidValue;
    constexpr int cb = 16 * RR_NCOL * RR_NWV;
    const int64_t blocks = (a.K + cb - 1) / cb;
    hipLaunchKernelGGL((rollout_rr<HP, RR_NWV, RR_NCOL>), dim3((unsigned)blocks), dim3(64 * RR_NWV), lds, st, a);
    return hipGetLastError();
}

int rr_candidates_per_block() { return 16 * RR_NCOL * RR_NWV; }

// image of the ring (capi.cpp pack_rr_image): slots per step x bytes per slot
size_t rr_image_bytes(int hidden_padded) {
    return (size_t)(2 + hidden_padded / 16) * (hidden_padded / 16 + 4) * 1024;
}

hipError_t launch_rollout_rr(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    switch (hidden_padded) {
        case 512: return launch_rr_t<512>(a, st);
        case 256: return launch_rr_t<256>(a, st);
        case 128: return launch_rr_t<128>(a, st);
        case 64: return launch_rr_t<64>(a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace bcmpc
