// rollout_team.hip -- small-K split-f16 rollout kernel (BCMPC_KERNEL_TEAM): weights resident in
// registers, one candidate column per team of workgroups.
//
// Path: MPCcontroller.get_action on the shard (controllers.py:57-88) for the 2-layer
// NNDynamicsModel (dynamics.py:54-71: [S+A -> h] act (+LN), [h -> h] act (+LN), [h -> S] linear)
// with the fused cheetah cost (cost_functions.py:9-30, 59-63).  Same arithmetic as rollout_x3
// (hi/lo f16 operands, three MFMA passes, f32 accumulate, f64 state / cost), a
// different work split for the reference's own small configurations (train_mpc_ppo.py:71,77:
// K = 400; BASELINE cfg1: K = 1000), where rollout_x3 leaves most CUs idle and each of its few
// workgroups re-streams the whole net from L2 every step ("small K").
//
//   * One 16-candidate column per TEAM of T workgroups (NWV waves each).  Global wave
//     g = member * NWV + w owns the layer-1 tiles [TPW g, TPW (g + 1)) and the matching
//     output-layer k-steps (K-split); every member computes ALL of layer 0 (its NWV waves split
//     the tiles), so the only cross-workgroup traffic of a step is the output layer's partial
//     sums.  Every weight fragment a wave ever uses is loaded ONCE, before the first step, into
//     its registers (HP = 512, T = 4: 336 VGPRs per wave, one wave per SIMD).
//   * Per step: f64 state -> layer-0 input (every wave, redundantly) -> layer 0 (this wave's
//     tiles) -> LDS slab -> barrier -> layer 1 (this wave's tiles, B fragments from the slab)
//     -> epilogue -> output partial (registers) -> LDS -> barrier -> member partial summed in
//     wave order -> (T > 1) exchange of member partials -> total summed in member order ->
//     de-normalise + residual + cost (f64, every wave, identical bits in every member).
//   * Exchange (T > 1; cdna_hip_programming.md Guideline 16, form R2: the data is the flag):
//     wave 0 of each member stores its partial as 8-byte {epoch, f32} granules with agent-scope
//     relaxed atomic stores and sweeps the other members' granules with agent-scope relaxed atomic
//     loads until every tag equals the step's epoch.  Two buffers by step parity: a member can
//     only be one step ahead of the slowest (it needs that member's partial to finish its own
//     step), so it never overwrites granules still unread.  Epoch = (gen << 10) + h + 1, gen a
//     per-engine launch counter advanced by the launch's last workgroup (ticket), so granules of
//     earlier launches never match and nothing has to be zeroed per call.  Spins are bounded:
//     a team that cannot meet (a member never became resident) sets *team_err and finishes.
//   * Co-residency: all T members of a team must run at once.  The host launches a team kernel
//     only when the whole grid fits one workgroup per CU (capi.cpp); members of a column are
//     numbered b, b + 8, ... so they share an XCD under round-robin dispatch (speed only).
//
// Numerics (same bar as rollout_x3): the output layer's partial sums are added in a fixed order
// (waves of a member, then members), identical in every member, so every member's f64 state is
// bit-identical and only member 0 writes costs / trajectories.  relu without LayerNorm: layer 0
// uses one power of two per candidate column (max over the member's waves, one LDS exchange), the
// layer-1 output one per wave, undone exactly on that wave's partial before the sums.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcmpc.h"
#include "device_common.h"
#include "kernels.h"
#include "split_common.h"
#include "argmin_common.h"

namespace bcmpc {

// TEAM_STAMP 1 (timing diagnostic, tools/team_variants.sh builds only): per-phase s_memtime totals of
// every wave into a.stamps ([blocks][NWV][10]: 0 tail, 1 action fill, 2 layer-0 input, 3 layer 0,
// 4 slab barrier, 5 layer-1 MFMAs, 6 layer-1 epilogue, 7 output + partials barrier, 8 member sums /
// exchange, 9 prologue); TEAM_STAMP 2: the prologue split instead (0 parameters, 1 first fill, 2 weight
// issue, 3 state set-up)
#ifndef TEAM_STAMP
#define TEAM_STAMP 0
#endif
#if TEAM_STAMP && !defined(BCMPC_DIAG_VARIANT)
#error "TEAM_STAMP is a timing diagnostic: build it with tools/team_variants.sh"
#endif

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int kTeamSpins = 1 << 20;      // exchange polls before a team gives up (~1 s)
constexpr uint64_t kRowsWaitTicks = 20000000;   // late pre-draw rows: give up after 0.2 s (100-MHz clock)
constexpr int kTeamNch = 16;             // steps of action inputs staged in LDS per fill
constexpr int kPolNch = 8;               // steps of the policy's draws (f64) staged per fill

// reward-net layout: TEAM_RW_NWV waves per member (4: one 512-register wave per SIMD, two head tiles
// per wave; 8: two 256-register waves per SIMD, one head tile each -- 68 spilled registers with the
// policy, measured slower)
#ifndef TEAM_RW_NWV
#define TEAM_RW_NWV 4
#endif
// hidden 256 (train_mpc_ppo.py's 2x256 net): 4 waves x 4 tiles (512-register waves) or 8 waves x 2 tiles
#ifndef TEAM_NWV256
#define TEAM_NWV256 4
#endif

__device__ __forceinline__ f4 mm(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// the split product hi*hi + hi*lo + lo*hi accumulated into c
__device__ __forceinline__ f4 mm3(h8 ah, h8 al, h8 bh, h8 bl, f4 c) {
    c = mm(ah, bh, c);
    c = mm(ah, bl, c);
    return mm(al, bh, c);
}

__device__ __forceinline__ float tanh4096(float z) {     // tanh(y) * 2^12 from z = 2 log2(e) y (rollout_x3)
    const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z) + 1.0f);
    return fmaf(-8192.0f, r, 4096.0f);
}

__host__ __device__ constexpr int team_wpe(int NWV) { return NWV >= 8 ? 2 : 1; }

// s[v] = p[(0 * 2 + v) * 64 + lane] + ... + p[((N - 1) * 2 + v) * 64 + lane] in that order (the same bits in
// every wave and member), both halves v together, the next term's parts requested before the current adds:
// one read at a time, each waited for, made 2 N dependent LDS round trips of it
template <int N>
__device__ __forceinline__ void ordered_sum2(const f4* p, int lane, f4 (&s)[2]) {
    s[0] = p[(0 * 2 + 0) * 64 + lane];
    s[1] = p[(0 * 2 + 1) * 64 + lane];
    if constexpr (N > 1) {
        f4 nx[2] = {p[(1 * 2 + 0) * 64 + lane], p[(1 * 2 + 1) * 64 + lane]};
#pragma unroll
        for (int t = 1; t < N; ++t) {
            const f4 c0 = nx[0], c1 = nx[1];
            if (t + 1 < N) {
                nx[0] = p[((t + 1) * 2 + 0) * 64 + lane];
                nx[1] = p[((t + 1) * 2 + 1) * 64 + lane];
            }
            s[0] += c0;
            s[1] += c1;
        }
    }
}

// The LDS constants table behind a compiler-opaque value, so the step loop re-reads it instead of hoisting
// it into registers: an opaque zero offset (keeps the LDS address space: ds_read), or (PTR) an opaque
// pointer (generic: flat loads; fewer live registers in the kernels that have none to spare)
template <bool PTR>
__device__ __forceinline__ const double* team_opaque_lds(const double* C) {
    if constexpr (PTR) {
        asm volatile("" : "+v"(C));
        return C;
    } else {
        int cz = 0;
        asm volatile("" : "+s"(cz));
        return C + cz;
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads (a __syncthreads() fence drains vmcnt too, which would hold every barrier of the
// first step behind the weight prologue's ~80 loads per wave).  Every hand-off between waves in
// this kernel goes through LDS; cross-workgroup data travels in atomic granules.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Chan et al.'s merge of the NWV waves' per-column (mean, M2) in wave order (xch: [NWV][16][2]; lane column m)
template <int NTL, int NWV, bool CLOSED>
__device__ __forceinline__ void ln_merge(const float* xch, int m, int hidden, float& mean, float& m2) {
    mean = 0.f;
    m2 = 0.f;
    if (hidden == 16 * NTL * NWV) {
        // every wave full (no padded rows): the merge weights nb / nn and n nb / nn are the same
        // f32 quotients as below, folded at compile time -- a chain of 2 NWV dependent divisions
        // per LayerNorm off the step's critical path (bit-identical)
#pragma unroll
        for (int v = 0; v < NWV; ++v) {
            const float nb = (float)(16 * NTL), n = (float)(16 * NTL * v), nn = n + nb;
            const f2 st = *reinterpret_cast<const f2*>(xch + (v * 16 + m) * 2);
            const float d = st[0] - mean;
            mean = mean + d * (nb / nn);
            m2 = m2 + st[1] + d * d * (n * nb / nn);
        }
    } else if constexpr (CLOSED) {
        // (padded rows: the merge weights from the closed form n_v = min(hidden, 16 NTL v) -- the same
        //  quotients as the running count gave, now independent of each other instead of a chain of
        //  2 NWV dependent divisions on the step's critical path)
        //  (an opaque copy of hidden keeps them in the step: hoisted, their registers spilled elsewhere)
        int hid = hidden;
        asm volatile("" : "+s"(hid));
        float wq0[NWV], wq1[NWV];
#pragma unroll
        for (int v = 0; v < NWV; ++v) {
            const float nb = (float)min(max(hid - 16 * NTL * v, 0), 16 * NTL);
            const float n = (float)min(max(hid, 0), 16 * NTL * v), nn = n + nb;
            wq0[v] = nb > 0.f ? nb / nn : 0.f;
            wq1[v] = nb > 0.f ? n * nb / nn : 0.f;
        }
#pragma unroll
        for (int v = 0; v < NWV; ++v) {
            if (hidden - 16 * NTL * v > 0) {
                const f2 st = *reinterpret_cast<const f2*>(xch + (v * 16 + m) * 2);
                const float d = st[0] - mean;
                mean = mean + d * wq0[v];
                m2 = m2 + st[1] + d * d * wq1[v];
            }
        }
    } else {
        // (the running count: kept where the closed form measured slower -- ppo_defaults +0.9 us
        //  although its rows are never padded)
        float n = 0.f;
#pragma unroll
        for (int v = 0; v < NWV; ++v) {
            const float nb = (float)min(max(hidden - 16 * NTL * v, 0), 16 * NTL);
            if (nb > 0.f) {
                const f2 st = *reinterpret_cast<const f2*>(xch + (v * 16 + m) * 2);
                const float nn = n + nb, d = st[0] - mean;
                mean = mean + d * (nb / nn);
                m2 = m2 + st[1] + d * d * (n * nb / nn);
                n = nn;
            }
        }
    }
}

// relu / LayerNorm epilogue of one wave's NTL tiles (tile x * NTL + j of the layer), one candidate
// column per lane column m: BiasAdd + activation in f32, then
//   XCH (LN, or relu's column max across the member): one exchange of per-column statistics
//     through LDS (xch: [NWV][16][2]) and a barrier, merged in wave order (Chan et al.; var =
//     M2 / hidden; x * inv + (beta - mean * inv), inv = rsqrt(var + eps) * gamma, x hsc);
//   !XCH (relu without LN, layer 1): this wave's own column max picks the power of two;
// then the split into the next layer's B fragments.  fcol: 2^-sh of relu's column scale.
//   DEFER (LN, the last hidden layer at T = 1): no barrier and no normalisation here -- the activations
//     are left centred on this wave's own column mean, the statistics published for the output layer's
//     partials barrier, and the normalisation applied to the summed output rows (rollout_team's DEFER)
template <int AK, int NTL, int NWV, bool XCH, bool CLOSED = false, bool DEFER = false>
__device__ __forceinline__ void epi_cols(f4 (&acc)[NTL], float f, const float* __restrict__ bias,
                                         const float* __restrict__ lg, const float* __restrict__ lb, float hsc,
                                         int hidden, float* xch, int x, int w, int lane, float& fcol) {
    constexpr bool RELU = (AK & 1) != 0, LNK = (AK & 2) != 0;
    const int q = lane >> 4, m = lane & 15;
#pragma unroll
    for (int j = 0; j < NTL; ++j) {
        const f4 b = *reinterpret_cast<const f4*>(bias + 16 * (x * NTL + j) + 4 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float z = fmaf(acc[j][r], f, b[r]);
            acc[j][r] = RELU ? fmaxf(z, 0.f) : tanh4096(z);              // pad rows: exactly 0
        }
    }
    const int nwr = min(max(hidden - 16 * NTL * x, 0), 16 * NTL);      // this wave's valid rows
    float s0 = 0.f, s1 = 0.f;
    if constexpr (LNK) {
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s0 += acc[j][r];
        s0 = add_rows(s0) * (nwr > 0 ? 1.0f / (float)nwr : 0.f);     // (loop-invariant reciprocal)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = acc[j][r] - s0;
                const bool in = 16 * (x * NTL + j) + 4 * q + r < hidden;
                s1 += in ? d * d : 0.f;
                if constexpr (DEFER) acc[j][r] = in ? d : 0.f;
            }
        s1 = add_rows(s1);
    } else {
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s0 = fmaxf(s0, acc[j][r]);
        s0 = max_rows32(max_rows16(s0));
    }
    if constexpr (XCH) {
        if (q == 0) *reinterpret_cast<f2*>(xch + (w * 16 + m) * 2) = (f2){s0, s1};
        if constexpr (DEFER) {
            // (published with the partials) the centred activations go into the split operands scaled by
            // this wave's column power of two, |d| max in [2^11, 2^12) as the relu path's below: the lo
            // half stays out of f16's subnormals (and hi below its overflow) whatever the weights' scale;
            // the wave's output partial is multiplied back by fcol = 2^-sh (exact) before the partials sum
            float mx = 0.f;
#pragma unroll
            for (int j = 0; j < NTL; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) mx = fmaxf(mx, fabsf(acc[j][r]));
            mx = max_rows32(max_rows16(mx));
            int e = 0;
            (void)frexpf(mx, &e);
            int sh = 12 - e;
            sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
            const float sc = ldexpf(1.0f, sh);
            fcol = ldexpf(1.0f, -sh);
#pragma unroll
            for (int j = 0; j < NTL; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[j][r] *= sc;
            return;
        }
        lds_barrier();                                                      // every wave's statistics published
    }
    if constexpr (LNK) {
        float mean = 0.f, m2 = 0.f;
        ln_merge<NTL, NWV, CLOSED>(xch, m, hidden, mean, m2);
        const float eps = RELU ? 1e-12f : 1e-12f * 16777216.0f;        // tanh: activations carry x 2^12
        const float rs = __builtin_amdgcn_rsqf(m2 * (1.0f / (float)hidden) + eps);    // v_rsq_f32 (~1 ulp)
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
            const f4 gv = *reinterpret_cast<const f4*>(lg + 16 * (x * NTL + j) + 4 * q);
            const f4 bv = *reinterpret_cast<const f4*>(lb + 16 * (x * NTL + j) + 4 * q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float inv = rs * gv[r];
                acc[j][r] = (acc[j][r] * inv + (bv[r] - mean * inv)) * hsc;
            }
        }
    } else {
        float mx = s0;
        if constexpr (XCH) {
            mx = 0.f;
#pragma unroll
            for (int v = 0; v < NWV; ++v) mx = fmaxf(mx, xch[(v * 16 + m) * 2]);
        }
        int e = 0;
        (void)frexpf(mx, &e);
        int sh = 12 - e;
        sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
        const float sc = ldexpf(1.0f, sh);
        fcol = ldexpf(1.0f, -sh);
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[j][r] *= sc;
    }
}

// activations of NTL tiles -> the next layer's B fragments (hi, lo): a tile pair is one 32-wide
// k-step (capi.cpp pack_x3_layer k order); a single tile fills the half of its k-step that its
// parity selects (odd: rows 16..31), the other half is zero
template <int NTL>
__device__ __forceinline__ void split_tiles(const f4 (&v)[NTL], int odd, h8 (&xh)[(NTL + 1) / 2],
                                            h8 (&xl)[(NTL + 1) / 2]) {
    if constexpr (NTL == 1) {
        float u[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            u[r] = odd ? 0.f : v[0][r];
            u[4 + r] = odd ? v[0][r] : 0.f;
        }
        split8(u, xh[0], xl[0]);
    } else {
#pragma unroll
        for (int pp = 0; pp < NTL / 2; ++pp) {
            const float u[8] = {v[2 * pp][0],     v[2 * pp][1],     v[2 * pp][2],     v[2 * pp][3],
                                v[2 * pp + 1][0], v[2 * pp + 1][1], v[2 * pp + 1][2], v[2 * pp + 1][3]};
            split8(u, xh[pp], xl[pp]);
        }
    }
}

}  // namespace

// LDS: consts | biases [2 or 3][HP] + 32 | LN gamma [2][HP], beta [2][HP] | slab [P][hi|lo][64] f4 |
// column exchange [2 layers][NWV][16][2] | output partials [NWV][2][64] f4 | members' partials [T][2][64] f4 +
// the team's "gave up" word (16 B) | (policy, T == 1) the policy's output partials [NWV][64] f4 | action inputs [kTeamNch][16][16] (no policy) | policy biases + params, policy hidden->hidden weights
// (PHP > 0; its first and output layers live in registers)
__host__ __device__ constexpr int team_lds_bytes(int HP, int NWV, int T, int AK, bool RW = false, int PHP = 0,
                                                 int PL = 0, int pw_bytes = 0) {
    return param_bytes(RW ? 3 : 2, HP) + ((AK & 2) ? 4 * HP * 4 : 0) + (HP / 32) * 2048 + (AK ? 2 * NWV * 16 * 2 * 4 : 0) +
           NWV * 2048 + (T > 1 ? T * 2048 + 16 : 0) + (PHP > 0 && T == 1 ? NWV * 1024 : 0) +
           (PHP > 0 ? pol_param_bytes(PL, PHP) + pw_bytes + kPolNch * 16 * 16 * 8 : kTeamNch * 16 * 16 * 4);
}

template <int HP, int NWV, int TPW, int T, int AK, int PHP = 0, bool RW = false>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(team_wpe(NWV), team_wpe(NWV))))
void rollout_team(const RolloutArgs a) {
    constexpr bool RELU = (AK & 1) != 0, LNK = (AK & 2) != 0, DYN = RELU && !LNK;
    constexpr float kAct = RELU ? 1.0f : kTanhK;        // folded into the epilogue factors / biases
    constexpr int NT = HP / 16, P = HP / 32;
    constexpr int L0T = NT / NWV, L0P = L0T / 2;        // layer-0 tiles / k-steps per wave (whole layer per member)
    constexpr int PPW = (TPW + 1) / 2;                  // output-layer k-steps per wave (TPW = 1: half of one)
    // a LayerNorm after layer 1 needs the whole layer in one workgroup -- except the reward net's heads,
    // whose per-member statistics ride along with the output partials (below)
    static_assert(!LNK || T == 1 || RW, "LayerNorm geometry");
    constexpr bool HLN = RW && LNK;                     // the reward net's LayerNorm heads (dynamics.py:165-177)
    // DEFER (relu + LayerNorm delta net at T = 1, TEAM_DEFER): the second LayerNorm moves behind the output
    // layer.  The output kernel is packed as dense_2 diag(gamma_1) (its bias + dense_2^T beta_1 in the bias
    // row, capi.cpp), each wave feeds it its activations centred on its own column mean, and after the
    // partials barrier -- which now also publishes the statistics -- the summed rows become
    // rsqrt(var + eps) (sum + sum_w (mean_w - mean) c_w), c_w = the wave's rows of the scaled, folded output
    // kernel summed (lnp + HP, [NWV][32]): one barrier and the normalisation pass fewer per step
    // (not with a fused policy: ppo_mpc_default's kernel spilled 8 VGPRs with it, +0.8 us)
    constexpr bool DEFER = TEAM_DEFER && T == 1 && AK == 3 && !RW && PHP == 0;     // (kernels.h)
    static_assert(!DEFER || NWV * 32 <= HP, "the deferred LayerNorm's per-wave row sums fit gamma_1's LDS slot");
    constexpr bool OPQ_PTR = RW || (PHP > 0 && HP > 256);   // (team_opaque_lds)
    // fused policy (MPCcontrollerPolicyNet, ppo_bc_policy.py:54-88): each wave owns one policy tile
    // pair; it shares the dynamics slab (free once the step's partials barrier has passed) and, when
    // a team barrier ends the step (T > 1), the partials buffer; at T == 1 waves may still be summing
    // the previous step's dynamics partials while the first ones publish their policy partials, so
    // those get a buffer of their own.  Any dynamics activation / LayerNorm (train_mpc_ppo.py's
    // 2x256 relu + LN net under the 2x128 tanh policy, :178, :198-216).
    // Reward net (NNDynamicsRewardModel): waves [0, NWV/2) hold delta-head tiles, waves [NWV/2, NWV)
    // reward-head tiles (TPW each), so every wave keeps one head's weights: NH waves per head.
    constexpr int PTW = PHP / 16 / NWV;                 // policy tiles per wave (1: half a k-step, 2: one)
    static_assert(PHP == 0 || PTW == 1 || PTW == 2, "policy geometry");
    static_assert(!RW || ((AK == 0 || AK == 2) && NWV % 2 == 0), "reward net: tanh (+ LayerNorm), delta / reward waves");
    constexpr int NB = RW ? 3 : 2;                      // hidden bias arrays (trunk, delta head, reward head)
    constexpr int NH = RW ? NWV / 2 : NWV;              // waves per head
    static_assert(HP == 16 * TPW * NH * T && (TPW == 1 || TPW % 2 == 0) && L0T % 2 == 0, "team geometry");
    extern __shared__ __attribute__((aligned(16))) f4 lds[];

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, m = lane & 15;
    const int S = a.S, A = a.A;
    const int bx = blockIdx.x;
    const int col = ((bx >> 3) / T) * 8 + (bx & 7);     // members of a column: blocks b, b + 8, ...
    const int tm = (bx >> 3) % T;                       // member
    const bool rw_wave = RW && w >= NH;                 // (reward net) this wave holds reward-head tiles
    const int g = tm * NH + (RW ? w % NH : w);          // team wave of its head: tiles [TPW g, TPW (g + 1))
    const int64_t ncol = (a.K + 15) / 16;
    uint64_t ph_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tp_ = TEAM_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    // TEAM_STAMP 2: the prologue's phases instead (slots 0 params, 1 first fill, 2 weight issue, 3 state)
    auto pstamp = [&](int k) __attribute__((always_inline)) {
        if constexpr (TEAM_STAMP == 2) {
            const uint64_t t_ = __builtin_amdgcn_s_memtime();
            ph_[k] += t_ - tp_;
            tp_ = t_;
        }
    };
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if constexpr (TEAM_STAMP == 1) {
            const uint64_t t_ = __builtin_amdgcn_s_memtime();
            ph_[k] += t_ - tp_;
            tp_ = t_;
        }
    };
    // TEAM_STAMP 3: s_memrealtime (100 MHz, one clock for the whole chip) at five points of the exchange of
    // steps H/2 and H/2 + 1 (slots 5 k + 0 partials done, 1 published, 2 this wave's members in, 3 every member
    // in, 4 totals): member skew and hand-off latency (BCMPC_STAMP_DUMP writes the raw records)
    auto rstamp = [&](int h, int k) __attribute__((always_inline)) {
        if constexpr (TEAM_STAMP == 3) {
            const int d = h - a.H / 2;
            if (d == 0 || d == 1) ph_[5 * d + k] = __builtin_amdgcn_s_memrealtime();
        }
    };
    unsigned gen = 0;
    if constexpr (T > 1) gen = __hip_atomic_load(a.team_ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    Best mybest{__builtin_inf(), INT64_MAX};              // (fused argmin) this workgroup's candidate
    if (col < ncol) {
        char* const base = reinterpret_cast<char*>(lds);
        double* C = reinterpret_cast<double*>(base);
        float* Bl = reinterpret_cast<float*>(base + kConstRows * kConstCols * 8);
        int off = param_bytes(NB, HP);
        float* const lnp = reinterpret_cast<float*>(base + off);
        off += LNK ? 4 * HP * 4 : 0;
        f4* const slab = reinterpret_cast<f4*>(base + off);
        off += P * 2048;
        float* const xch = reinterpret_cast<float*>(base + off);
        off += AK ? 2 * NWV * 16 * 2 * 4 : 0;                              // (as team_lds_bytes)
        f4* const parts = reinterpret_cast<f4*>(base + off);
        off += NWV * 2048;
        f4* const tot = reinterpret_cast<f4*>(base + off);
        int* const tdead = reinterpret_cast<int*>(base + off + T * 2048);   // (T > 1) this member gave up
        off += T > 1 ? T * 2048 + 16 : 0;
        f4* const pparts = PHP > 0 && T == 1 ? reinterpret_cast<f4*>(base + off) : parts;   // policy partials
        off += PHP > 0 && T == 1 ? NWV * 1024 : 0;
        float* const xas = reinterpret_cast<float*>(base + off);          // (no policy)
        float* const Pb = reinterpret_cast<float*>(base + off);           // (policy) biases [pL][PHP] + params
        const char* const plw = base + off + (PHP > 0 ? pol_param_bytes(a.pL, PHP) : 0);   // policy weights
        double* const pdraw = reinterpret_cast<double*>(const_cast<char*>(plw));  // (offset by pw_total below)

        // Parameters into LDS.  Every load is issued before the first LDS store (register batches with
        // compile-time trip counts): a load -> wait -> store loop per array paid one global round trip per
        // array and pass, ~3 us of the prologue at K = 400 (TEAM_STAMP 2, profiles/r02c_team_prologue_stamps.txt)
        // and one per 4-KB pass of the policy's hidden weights (16 at 2x128).  The loads are unconditional
        // (clamped indices: a load under the same test as its store was fused with it, load -> wait -> store)
        constexpr int BS = 64 * NWV;
        constexpr int NCn = (kConstRows * kConstCols + BS - 1) / BS, NHn = (HP + BS - 1) / BS;
        int pw_total = 0;                                 // policy: every layer's packed bytes, copied once
        if constexpr (PHP > 0) {
            for (int l = 1; l < a.pL; ++l) pw_total += a.pwbytes[l];
            // the policy's hidden layers 1..pL-1 (contiguous, capi.cpp pw_off): 16 f4 per thread in flight
            const f4* src = a.pw[1];
            f4* const dst = reinterpret_cast<f4*>(const_cast<char*>(plw));
            const int n4 = pw_total / 16;
            for (int i0 = threadIdx.x; i0 < n4; i0 += 16 * BS) {
                f4 r[16];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (i0 + u * BS < n4) r[u] = src[i0 + u * BS];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (i0 + u * BS < n4) dst[i0 + u * BS] = r[u];
            }
        }
        {
            const int t = threadIdx.x;
            double rc[NCn];
            float rb[NB][NHn], rbo = 0.f;
#pragma unroll
            for (int u = 0; u < NCn; ++u)
                rc[u] = a.consts[min(t + u * BS, kConstRows * kConstCols - 1)];
#pragma unroll
            for (int l = 0; l < NB; ++l)
#pragma unroll
                for (int u = 0; u < NHn; ++u)
                    rb[l][u] = a.b[l][min(t + u * BS, HP - 1)];
            rbo = a.b[NB][min(t, 31)];
            // (LayerNorm: gamma / beta of the trunk, and of layer 1 without the reward net's heads)
            constexpr int NLN = LNK ? (HLN ? 1 : 2) : 0;
            float rg[NLN > 0 ? NLN : 1][NHn], rbt[NLN > 0 ? NLN : 1][NHn];
#pragma unroll
            for (int l = 0; l < NLN; ++l)
#pragma unroll
                for (int u = 0; u < NHn; ++u)
                {
                        rg[l][u] = a.lng[l][min(t + u * BS, HP - 1)];
                        rbt[l][u] = a.lnb[l][min(t + u * BS, HP - 1)];
                    }
            // (policy: biases of its pL <= 3 layers and its parameters)
            constexpr int NPn = PHP > 0 ? (PHP + BS - 1) / BS : 1, NQn = (kPolParams + BS - 1) / BS;
            float rpb[3][NPn], rpp[NQn];
            if constexpr (PHP > 0) {
#pragma unroll
                for (int l = 0; l < 3; ++l)
#pragma unroll
                    for (int u = 0; u < NPn; ++u)
                        rpb[l][u] = a.pb[min(l, a.pL - 1)][min(t + u * BS, PHP - 1)];
#pragma unroll
                for (int u = 0; u < NQn; ++u)
                    rpp[u] = a.pparams[min(t + u * BS, kPolParams - 1)];
            }
            constexpr int NRn = (T * 32 + BS - 1) / BS;
            float rrs[NRn];
            if constexpr (HLN)
#pragma unroll
                for (int u = 0; u < NRn; ++u)
                    rrs[u] = a.head_rs[min(t + u * BS, T * 32 - 1)];
            // ---- the stores ----
#pragma unroll
            for (int u = 0; u < NCn; ++u)
                if (t + u * BS < kConstRows * kConstCols) C[t + u * BS] = rc[u];
#pragma unroll
            for (int l = 0; l < NB; ++l)
#pragma unroll
                for (int u = 0; u < NHn; ++u)
                    if (t + u * BS < HP) Bl[l * HP + t + u * BS] = rb[l][u] * kAct;
            if (t < 32) Bl[NB * HP + t] = rbo;
            if constexpr (PHP > 0) {
#pragma unroll
                for (int l = 0; l < 3; ++l)
#pragma unroll
                    for (int u = 0; u < NPn; ++u)
                        if (l < a.pL && t + u * BS < PHP) Pb[l * PHP + t + u * BS] = rpb[l][u] * kTanhK;
#pragma unroll
                for (int u = 0; u < NQn; ++u)
                    if (t + u * BS < kPolParams) Pb[a.pL * PHP + t + u * BS] = rpp[u];
            }
            if constexpr (HLN) {
                // the trunk's gamma / beta at [0, HP) / [2 HP, 3 HP); [HP, ..): the heads' centring table
                // head_rs [T][32], then Chan's merge weights (nb / nn, n nb / nn) of the T members in order
#pragma unroll
                for (int u = 0; u < NHn; ++u)
                    if (t + u * BS < HP) {
                        lnp[t + u * BS] = rg[0][u];
                        lnp[2 * HP + t + u * BS] = rbt[0][u];
                    }
#pragma unroll
                for (int u = 0; u < NRn; ++u)
                    if (t + u * BS < T * 32) lnp[HP + t + u * BS] = rrs[u];
                if (t == 0) {
                    float n = 0.f;
                    for (int tt = 0; tt < T; ++tt) {
                        const float nb = (float)min(max(a.hidden - 16 * TPW * NH * tt, 0), 16 * TPW * NH), nn = n + nb;
                        lnp[HP + T * 32 + 2 * tt] = nb > 0.f ? nb / nn : 0.f;
                        lnp[HP + T * 32 + 2 * tt + 1] = nb > 0.f ? n * nb / nn : 0.f;
                        n = nn;
                    }
                }
            } else if constexpr (LNK) {
#pragma unroll
                for (int l = 0; l < 2; ++l)
#pragma unroll
                    for (int u = 0; u < NHn; ++u)
                        if (t + u * BS < HP) {
                            lnp[l * HP + t + u * BS] = rg[l][u];
                            lnp[(2 + l) * HP + t + u * BS] = rbt[l][u];
                        }
            }
        }

        if constexpr (T > 1)
            if (threadIdx.x == 0) *tdead = 0;
        if constexpr (PHP == 0)
            for (int i = threadIdx.x; i < kTeamNch * 16 * 16; i += blockDim.x)
                if ((i & 15) >= A) xas[i] = 0.f;            // action slots past A stay zero (fill writes j < A)
        if (a.rows_flag && threadIdx.x == 0) {
            // late pre-draw hit (capi.cpp): the host worker publishes the rows' sequence number after its
            // last row; its stores are ordered, so a system-scope acquire of the word makes every row visible
            // (fine-grained host memory: no GPU cache holds an older copy).  A worker that never publishes
            // gives up after ~0.2 s (100-MHz real-time clock): the team's error word makes the host rerun
            // the call on its fallback engine with a fresh draw
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
        __syncthreads();                                  // parameters in LDS (and the rows published)
        pstamp(0);
        // ---- actions, normalised (dynamics.py:110) and cast to f32 (the TF feed), staged in LDS for
        //      kTeamNch steps at a time by the whole workgroup (one action per thread and pass, not per
        //      lane in the step loop): the caller's [H,K,A] array (np.random.uniform,
        //      controllers.py:53), Philox (rng_action), or the CEM sampler ----
        // the policy's draws for kPolNch steps, by the whole workgroup: N(0,1) of the stochastic policy
        // (rng_normal, f32, exact in the f64 slot) or the explore uniforms U (the caller's array,
        // controllers.py:191, or Philox) -- none depends on the state, so no step waits for them
        double* const pdr = pdraw + (PHP > 0 ? pw_total / 8 : 0);
        auto fill_draws = [&](int h0) {
            const int nh = min(kPolNch, a.H - h0), n = nh * 16 * A;
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int hh = i / (16 * A), rem = i - hh * 16 * A, mm = rem / A, j = rem - mm * A;
                const int64_t c = (int64_t)col * 16 + mm;
                double v = 0.0;
                if (c < a.K) {
                    const int h = h0 + hh;
                    const uint64_t gc = (uint64_t)(a.cand_offset + c);
                    v = a.pol_mode == BCMPC_POLICY_STOCHASTIC
                            ? (double)rng_normal(a.seed ^ 0x9E3779B97F4A7C15ull, gc, h, j)
                        : a.actions ? a.actions[((int64_t)h * a.K + c) * A + j]
                                    : rng_action(a.seed, gc, h, j, C[6 * 32 + j], C[7 * 32 + j]);
                }
                pdr[(hh * 16 + mm) * 16 + j] = v;
            }
        };
        auto fill_actions = [&](int h0) {
            if constexpr (PHP > 0) {                      // (the policy makes the actions)
                if (h0 % kPolNch == 0) fill_draws(h0);
                return;
            }
            const int nh = min(kTeamNch, a.H - h0);
            if (!a.cem_mu && !a.actions) {
                // device Philox: one block feeds actions 2p and 2p + 1 (half the blocks per pass)
                const int AP = (A + 1) >> 1, n = nh * 16 * AP;
                for (int i = threadIdx.x; i < n; i += blockDim.x) {
                    const int hh = i / (16 * AP), rem = i - hh * 16 * AP, mm = rem / AP, p = rem - mm * AP;
                    const int j0 = 2 * p, j1 = min(2 * p + 1, A - 1);
                    const int64_t c = (int64_t)col * 16 + mm;
                    float x0 = 0.f, x1 = 0.f;
                    if (c < a.K) {
                        double v0, v1;
                        rng_action_pair(a.seed, (uint64_t)(a.cand_offset + c), h0 + hh, p, C[6 * 32 + j0],
                                        C[7 * 32 + j0], C[6 * 32 + j1], C[7 * 32 + j1], v0, v1);
                        x0 = (float)div_rn(__dsub_rn(v0, C[2 * 32 + j0]), C[3 * 32 + j0], C[9 * 32 + j0]);
                        x1 = (float)div_rn(__dsub_rn(v1, C[2 * 32 + j1]), C[3 * 32 + j1], C[9 * 32 + j1]);
                    }
                    float* const dst = xas + (hh * 16 + mm) * 16;
                    dst[j0] = x0;
                    if (2 * p + 1 < A) dst[j1] = x1;
                }
                return;
            }
            const int n = nh * 16 * A;
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int hh = i / (16 * A), rem = i - hh * 16 * A, mm = rem / A, j = rem - mm * A;
                const int64_t c = (int64_t)col * 16 + mm;
                float xv = 0.f;
                if (c < a.K) {
                    const int h = h0 + hh;
                    const uint64_t gc = (uint64_t)(a.cand_offset + c);
                    const double av = a.cem_mu ? cem_action(a.seed, gc, h, j, a.cem_iter, a.cem_mu[h * A + j],
                                                            a.cem_sigma[h * A + j], C[6 * 32 + j], C[7 * 32 + j])
                                      : a.actions ? a.actions[((int64_t)h * a.K + c) * A + j]
                                                  : rng_action(a.seed, gc, h, j, C[6 * 32 + j], C[7 * 32 + j]);
                    xv = (float)div_rn(__dsub_rn(av, C[2 * 32 + j]), C[3 * 32 + j], C[9 * 32 + j]);
                }
                xas[(hh * 16 + mm) * 16 + j] = xv;
            }
        };

        fill_actions(0);                                  // (before the weight loads: its global loads
        lds_barrier();                                    //  would otherwise wait behind them)
        pstamp(1);
        // ---- every weight fragment this wave uses, once (issued after the parameter barrier so the
        //      loads stay in flight through the first step's LDS barriers) (capi.cpp: layer 0 packed with TWp = L0T,
        //      layer 1 with TWp = TPW, the output layer [0][k-step][tile]) ----
        const int voff = lane * 16;
        h8 w0h[L0T], w0l[L0T], w1h[P][TPW], w1l[P][TPW], woh[PPW][2], wol[PPW][2];
        // fused policy: its first layer's tiles and its output layer's k-step stay in registers
        constexpr int PA = PHP > 0 ? PTW : 1;
        h8 p0h[PA], p0l[PA], pwoh, pwol;
        if constexpr (PHP > 0) {
            const __amdgpu_buffer_rsrc_t q0 = layer_rsrc(a.pw[0], a.pwbytes[0]);
#pragma unroll
            for (int j = 0; j < PTW; ++j) {
                p0h[j] = fload(q0, voff, (w * PTW + j) * 2048);
                p0l[j] = fload(q0, voff, (w * PTW + j) * 2048 + 1024);
            }
            const __amdgpu_buffer_rsrc_t qo = layer_rsrc(a.pw[a.pL], a.pwbytes[a.pL]);
            const int kp = PTW == 2 ? w : w >> 1;         // this wave's k-step of the output layer
            pwoh = fload(qo, voff, kp * 2048);
            pwol = fload(qo, voff, kp * 2048 + 1024);
        }
        {
            if constexpr (!RW) {                          // (reward net: streamed per step, below)
                const __amdgpu_buffer_rsrc_t r0 = layer_rsrc(a.w[0], a.wbytes[0]);
#pragma unroll
                for (int j = 0; j < L0T; ++j) {
                    w0h[j] = fload(r0, voff, (w * L0T + j) * 2048);
                    w0l[j] = fload(r0, voff, (w * L0T + j) * 2048 + 1024);
                }
            }
            const int lh = rw_wave ? 3 : 1;               // this wave's head (dense_1 or dense_3)
            const __amdgpu_buffer_rsrc_t r1 = layer_rsrc(a.w[lh], a.wbytes[lh]);
#pragma unroll
            for (int p = 0; p < P; ++p)
#pragma unroll
                for (int j = 0; j < TPW; ++j) {
                    w1h[p][j] = fload(r1, voff, ((g * P + p) * TPW + j) * 2048);
                    w1l[p][j] = fload(r1, voff, ((g * P + p) * TPW + j) * 2048 + 1024);
                }
            // (reward-head waves: tile 0 zero, tile 1 = dense_4 packed as one 16-row tile whose row S-16
            //  feeds output row S -- capi.cpp split reward layout; the delta output weights there are 0)
            const __amdgpu_buffer_rsrc_t r2 = layer_rsrc(a.w[rw_wave ? 4 : 2], a.wbytes[rw_wave ? 4 : 2]);
#pragma unroll
            for (int pp = 0; pp < PPW; ++pp)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const int p = TPW == 1 ? g >> 1 : g * PPW + pp;
                    const int o = rw_wave ? (v == 0 ? 0x7FFFF000 : p * 2048) : (p * 2 + v) * 2048;  // (beyond range: 0)
                    woh[pp][v] = fload(r2, voff, o);
                    wol[pp][v] = fload(r2, voff, o + 1024);
                }
        }

        pstamp(2);
        // ---- per-candidate state: lane (q, m) holds dims 16 v + 4 q + r (v = 0, 1) of candidate m,
        //      in every wave of every member ----
        const int64_t cand = (int64_t)col * 16 + m;
        const bool valid = cand < a.K;
        const bool writer = tm == 0 && w == 0;            // costs / trajectories: member 0, wave 0
        double s[2][4];
        double cost = 0.0;                                // trajectory_cost = 0 (cost_functions.py:60)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int d = 16 * v + 4 * q + r;
                s[v][r] = (valid && d < S) ? (a.state_inline ? a.state_v[d] : a.state[cand * a.state_stride + d]) : 0.0;
                if (writer && a.traj && valid && d < S) a.traj[cand * S + d] = s[v][r];
            }

        const float f1base = a.winv[1] * kAct;
        const float fo = a.winv[2];
        float* const Bout = Bl + NB * HP;
        const int qc = RW ? (S - 16) >> 2 : 0;           // lane row holding the cost: dim 17 / reward row S
        gu64* const gb = (gu64*)a.team_buf;           // (global address space: never flat)
        bool dead = false;                                // the team cannot meet: finish without waiting
        const int spin_limit = a.team_spins > 0 ? a.team_spins : kTeamSpins;
        f4 ot[2];                                         // the step's summed output layer (rows 16 v + 4 q + r)
        double gp = 0.0;                                  // (reward net) gamma**(h-1) for this step's tail

        pstamp(3);
        stamp(9);
        for (int h = 0;; ++h) {
            if constexpr (RW) {
                // reward net: the registers hold both heads' tiles, so the trunk's fragments (8 KB per
                // wave) are re-read from L2 every step, requested here -- their latency passes under the
                // tail, the policy and the layer-0 input (an opaque offset keeps them in the loop)
                int vo = voff;
                asm volatile("" : "+v"(vo));
                const __amdgpu_buffer_rsrc_t r0 = layer_rsrc(a.w[0], a.wbytes[0]);
#pragma unroll
                for (int j = 0; j < L0T; ++j) {
                    w0h[j] = fload(r0, vo, (w * L0T + j) * 2048);
                    w0l[j] = fload(r0, vo, (w * L0T + j) * 2048 + 1024);
                }
            }
            if (h > 0) {
                // ---- de-normalise + residual (dynamics.py:113,116; f64, no FMA), cheetah cost
                //      (cost_functions.py:12-28), in step order (:59-63) ----
                const int npen = partner_row16((s[0][1] >= 0.2) + (s[0][2] >= 0.0) + (s[0][3] >= 0.0));
                const double s17 = s[1][1];               // dim 17: v = 1, row q = 0, r = 1
                // (branch-free: dims >= S carry the padded constants -- mean 0, std 0 -- and are never read)
                f4 bv[2];
                double c4[2][4], c5[2][4];
                // (the constants are re-read from LDS every step: an opaque offset keeps the compiler from
                //  hoisting 40 doubles per lane out of the step loop, registers the resident weights need.
                //  An offset, not an opaque pointer: that lost the LDS address space -- flat loads)
                //  (Kept an opaque pointer in the 512-wide policy / reward-net kernels: the LDS-addressed
                //  form spilled 9-12 more registers there, run.sh recipe +12.6 us)
                const double* Cs = team_opaque_lds<OPQ_PTR>(C);
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    bv[v] = *reinterpret_cast<const f4*>(Bout + 16 * v + 4 * q);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        c4[v][r] = Cs[4 * 32 + 16 * v + 4 * q + r];
                        c5[v][r] = Cs[5 * 32 + 16 * v + 4 * q + r];
                    }
                }
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float dn = fmaf(ot[v][r], fo, bv[v][r]);                 // BiasAdd (f32)
                        const double ud = __dadd_rn(__dmul_rn((double)dn, c5[v][r]), c4[v][r]);
                        s[v][r] = __dadd_rn(s[v][r], ud);
                    }
                if constexpr (RW) {
                    // learned reward (dynamics.py:236) x gamma**h, running sum (controllers.py:139,150):
                    // output row S = tile 1, lane row (S - 16) >> 2, register (S - 16) & 3
                    if (q == qc) {
                        float o_s = 0.f;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (r == ((S - 16) & 3)) o_s = ot[1][r];
                        const float nr = fmaf(o_s, fo, Bout[S]);                      // BiasAdd (f32)
                        const double rw = __dadd_rn(__dmul_rn((double)nr, a.std_reward), a.mean_reward);
                        cost = __dadd_rn(cost, __dmul_rn(rw, gp));
                    }
                }
                if (a.cost == BCMPC_COST_CHEETAH) {
                    const double score =
                        __dsub_rn(10.0 * (double)npen, div_rn(__dsub_rn(s[1][1], s17), 0.01, 1.0 / 0.01));
                    cost = __dadd_rn(cost, score);
                }
                if (writer && a.traj && valid) {
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int d = 16 * v + 4 * q + r;
                            if (d < S) a.traj[((int64_t)h * a.K + cand) * S + d] = s[v][r];
                        }
                }
            }
            if constexpr (RW) gp = h < a.H ? a.gpow[h] : 0.0;   // gamma**h for the next tail (requested early)
            stamp(0);
            if (h == a.H) break;
            if (h > 0 && h % (PHP > 0 ? kPolNch : kTeamNch) == 0) {
                fill_actions(h);
                lds_barrier();                               // the chunk's action inputs (the previous chunk's
            }                                             // last reads were before the partials barrier)
            stamp(1);

            // ---- fused policy (MlpPolicy.act, ppo_bc_policy.py:54-88; mixing controllers.py:196-206),
            //      computed by every member (the same bits everywhere): obz = clip((f32(ob) - mean) / std,
            //      -5, 5) x 2^11 in this lane's dims (one k-step B fragment, no exchange), tanh hidden
            //      layers x 2^12 (wave w: tile pair = k-step w of the next layer, through the slab), the
            //      output tile (action j at row S - 16 + j) K-split over the waves, partials summed in
            //      wave order in every wave; pact = the actions of this lane's v = 1 dims ----
            double pact[4] = {0.0, 0.0, 0.0, 0.0};
            if constexpr (PHP > 0) {
                constexpr int PPn = PHP / 32;
                const float* const pm = Pb + a.pL * PHP;   // [obmean 32][obstd 32][logstd 16][out bias 16]
                h8 zh, zl;
                {
                    float z[8];
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int d = 16 * v + 4 * q + r;
                            float vv = ((float)s[v][r] - pm[d]) / pm[32 + d];
                            vv = fminf(fmaxf(vv, -5.0f), 5.0f);
                            z[4 * v + r] = d < S ? vv * 2048.0f : 0.f;
                        }
                    split8(z, zh, zl);
                }
                auto lread = [&](int byte_off) __attribute__((always_inline)) {
                    return *reinterpret_cast<const h8*>(plw + byte_off + lane * 16);
                };
                typedef _Float16 h4 __attribute__((ext_vector_type(4)));
                // this wave's policy tiles [PTW w, PTW (w + 1)) of every hidden layer; their epilogue
                // is the B fragment of k-step w (PTW = 2) or half w & 1 of k-step w >> 1 (PTW = 1)
                f4 pa[PTW];
                h8 xh, xl;
                auto pepi = [&](float f, const float* bias) __attribute__((always_inline)) {
                    if constexpr (PTW == 2) {
                        epi_pair_tanh(pa[0], pa[1], f, bias, 2 * w, q, xh, xl);
                    } else {
                        const f4 b = *reinterpret_cast<const f4*>(bias + 16 * w + 4 * q);
#pragma unroll
                        for (int r = 0; r < 4; ++r) pa[0][r] = tanh4096(fmaf(pa[0][r], f, b[r]));
                        split_tiles<1>(pa, w & 1, *reinterpret_cast<h8(*)[1]>(&xh), *reinterpret_cast<h8(*)[1]>(&xl));
                    }
                };
#pragma unroll
                for (int j = 0; j < PTW; ++j) pa[j] = mm3(p0h[j], p0l[j], zh, zl, (f4){0.f, 0.f, 0.f, 0.f});
                pepi(a.pwinv[0] * kTanhK, Pb);
                int lbase = 0, buf = 0;                   // (LDS: hidden layers 1..pL-1 only)
                for (int l = 1; l < a.pL; ++l) {
                    if constexpr (PTW == 2) {
                        swrite(slab + ((buf * PPn + w) * 2 + 0) * 64 + lane, xh);
                        swrite(slab + ((buf * PPn + w) * 2 + 1) * 64 + lane, xl);
                    } else {
                        const h4 hh4 = {xh[4 * (w & 1)], xh[4 * (w & 1) + 1], xh[4 * (w & 1) + 2], xh[4 * (w & 1) + 3]};
                        const h4 ll4 = {xl[4 * (w & 1)], xl[4 * (w & 1) + 1], xl[4 * (w & 1) + 2], xl[4 * (w & 1) + 3]};
                        reinterpret_cast<h4*>(slab + ((buf * PPn + (w >> 1)) * 2 + 0) * 64 + lane)[w & 1] = hh4;
                        reinterpret_cast<h4*>(slab + ((buf * PPn + (w >> 1)) * 2 + 1) * 64 + lane)[w & 1] = ll4;
                    }
                    lds_barrier();                        // the layer's input complete
#pragma unroll
                    for (int j = 0; j < PTW; ++j) pa[j] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int pq = 0; pq < PPn; ++pq) {
                        const h8 bh = sread(slab + ((buf * PPn + pq) * 2 + 0) * 64 + lane);
                        const h8 bl = sread(slab + ((buf * PPn + pq) * 2 + 1) * 64 + lane);
#pragma unroll
                        for (int j = 0; j < PTW; ++j) {
                            const int o = lbase + ((PTW * w + j) * PPn + pq) * 2048;     // [tile][k-step][hi|lo]
                            pa[j] = mm3(lread(o), lread(o + 1024), bh, bl, pa[j]);
                        }
                    }
                    pepi(a.pwinv[l] * kTanhK, Pb + l * PHP);
                    lbase += a.pwbytes[l];
                    buf ^= 1;                             // (double-buffered: no barrier before the writes)
                }
                // output layer [PHP -> one 16-row tile], K-split: this wave's (half) k-step, from registers
                const f4 po_ = mm3(pwoh, pwol, xh, xl, (f4){0.f, 0.f, 0.f, 0.f});
                pparts[w * 64 + lane] = po_;
                lds_barrier();                            // the output layer's partials
                f4 o = pparts[0 * 64 + lane];
#pragma unroll
                for (int x = 1; x < NWV; ++x) o += pparts[x * 64 + lane];   // fixed summation order
                const float fo_p = a.pwinv[a.pL];
                const double* const dr = pdr + ((h % kPolNch) * 16 + m) * 16;
                // (branch-free over the 4 rows: every row's LDS operands requested first -- the action index
                //  clamped -- and rows outside [S, S + A) drop their value after; per-row branches issued each
                //  row's reads and waited for them before the next row's)
                float pb_[4], ls_[4];
                double dr_[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int jc = min(max(16 + 4 * q + r - S, 0), A - 1);
                    pb_[r] = pm[80 + 4 * q + r];
                    ls_[r] = pm[64 + jc];
                    dr_[r] = dr[jc];
                }
                double pv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float mean = o[r] * fo_p + pb_[r];                    // dense bias (f32)
                    if (a.pol_mode == BCMPC_POLICY_STOCHASTIC) {
                        pv[r] = (double)(mean + expf(ls_[r]) * (float)dr_[r]);
                    } else {
                        // (1 - explore) * mean in f32 (NumPy keeps the f32 dtype), + explore * U in f64
                        const float t1 = (float)(1.0 - a.explore) * mean;
                        pv[r] = __dadd_rn((double)t1, __dmul_rn(a.explore, dr_[r]));
                    }
                    asm volatile("" : "+v"(pv[r]));
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 + 4 * q + r - S;
                    const bool in = j >= 0 && j < A;
                    pact[r] = in ? pv[r] : 0.0;
                    if (in && writer && a.act_out && h < a.act_out_steps && valid)   // action_paths (controllers.py:213)
                        __hip_atomic_store(&a.act_out[((int64_t)h * a.K + cand) * A + j], pact[r], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }

            // ---- layer-0 input: normalised state (dynamics.py:109) and action, cast to f32, scaled by
            //      the power of two that puts the column's max |x| in [2^11, 2^12) ----
            h8 b0h, b0l;
            float colf;
            {
                float x[8];
                float mx = 0.f;
                const float* const xr = xas + ((h % kTeamNch) * 16 + m) * 16;
                double c0[2][4], c1[2][4], c8[2][4];
                float av[2][4];
                const double* Cs = team_opaque_lds<OPQ_PTR>(C);     // (as in the tail)
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * v + 4 * q + r;
                        c0[v][r] = Cs[0 * 32 + d];
                        c1[v][r] = Cs[1 * 32 + d];
                        c8[v][r] = Cs[8 * 32 + d];
                        if constexpr (PHP > 0 && !OPQ_PTR) {  // the policy's action (dynamics.py:110)
                            // (computed in every lane and kept only in the action rows: a per-row branch
                            //  waited for each row's LDS constants before the next row's)
                            const int j = min(max(d - S, 0), A - 1);
                            float an = (float)div_rn(__dsub_rn(pact[r], Cs[2 * 32 + j]), Cs[3 * 32 + j], Cs[9 * 32 + j]);
                            asm volatile("" : "+v"(an));
                            av[v][r] = v == 1 && d >= S && d < S + A ? an : 0.f;
                        } else if constexpr (PHP > 0) {       // (the 512-wide kernels: no registers to spare)
                            const int j = min(max(d - S, 0), A - 1);
                            av[v][r] = v == 1 && d >= S && d < S + A
                                           ? (float)div_rn(__dsub_rn(pact[r], C[2 * 32 + j]), C[3 * 32 + j], C[9 * 32 + j])
                                           : 0.f;
                        } else {
                            av[v][r] = xr[min(max(d - S, 0), 15)];     // (slots >= A hold zeros)
                        }
                    }
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int d = 16 * v + 4 * q + r;
                        const float xs_ = (float)div_rn(__dsub_rn(s[v][r], c0[v][r]), c1[v][r], c8[v][r]);
                        const float xv = d < S ? xs_ : av[v][r];
                        x[4 * v + r] = xv;
                        mx = fmaxf(mx, fabsf(xv));
                    }
                mx = max_rows32(max_rows16(mx));
                int e = 0;
                (void)frexpf(mx, &e);
                int sh = 12 - e;
                sh = mx > 0.f ? (sh < -100 ? -100 : (sh > 100 ? 100 : sh)) : 0;
                const float sc = ldexpf(1.0f, sh);
#pragma unroll
                for (int k = 0; k < 8; ++k) x[k] *= sc;
                split8(x, b0h, b0l);
                colf = ldexpf(a.winv[0], -sh) * kAct;
            }

            stamp(2);
            // ---- layer 0 [S+A -> h]: this wave's L0T tiles, into the slab ----
            float fcol0 = 1.f;
            {
                f4 acc0[L0T];
#pragma unroll
                for (int j = 0; j < L0T; ++j) acc0[j] = mm3(w0h[j], w0l[j], b0h, b0l, (f4){0.f, 0.f, 0.f, 0.f});
                h8 xh[L0P], xl[L0P];
                if constexpr (AK == 0) {
#pragma unroll
                    for (int pp = 0; pp < L0P; ++pp)
                        epi_pair_tanh(acc0[2 * pp], acc0[2 * pp + 1], colf, Bl, w * L0T + 2 * pp, q, xh[pp], xl[pp]);
                } else {
                    epi_cols<AK, L0T, NWV, true, RW>(acc0, colf, Bl, lnp, lnp + 2 * HP, a.hsc[0], a.hidden, xch, w, w,
                                                 lane, fcol0);
                    split_tiles<L0T>(acc0, 0, xh, xl);
                }
#pragma unroll
                for (int pp = 0; pp < L0P; ++pp) {
                    swrite(slab + ((w * L0P + pp) * 2 + 0) * 64 + lane, xh[pp]);
                    swrite(slab + ((w * L0P + pp) * 2 + 1) * 64 + lane, xl[pp]);
                }
            }
            stamp(3);
            lds_barrier();                                   // layer-1 input complete
            stamp(4);

            // ---- layer 1 [h -> h]: this wave's TPW tiles over all P k-steps ----
            // (TPW <= 2: even / odd k-steps in separate accumulators, four independent MFMA chains)
            constexpr int KS = TPW <= 2 ? 2 : 1;
            f4 acc1[TPW], acc1b[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc1[j] = acc1b[j] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const h8 bh = sread(slab + (p * 2 + 0) * 64 + lane), bl = sread(slab + (p * 2 + 1) * 64 + lane);
#pragma unroll
                for (int j = 0; j < TPW; ++j) {
                    if (KS == 2 && (p & 1)) acc1b[j] = mm3(w1h[p][j], w1l[p][j], bh, bl, acc1b[j]);
                    else acc1[j] = mm3(w1h[p][j], w1l[p][j], bh, bl, acc1[j]);
                }
            }
            if constexpr (KS == 2)
#pragma unroll
                for (int j = 0; j < TPW; ++j) acc1[j] += acc1b[j];
            stamp(5);
            // (reward-head waves: dense_3's scale and biases)
            const float f1 = rw_wave ? a.winv[3] * kTanhK : DYN ? f1base * fcol0 : f1base;
            const float* const Bh = Bl + (rw_wave ? 2 : 1) * HP;
            h8 oh[PPW], ol[PPW];
            float fcol1 = 1.f;
            float hst[4] = {0.f, 0.f, 0.f, 0.f};          // (HLN) the member's (mean, M2) of both heads
            if constexpr (HLN) {
                // LayerNorm over a head split across the team (dynamics.py:171, :177; TF1 layer_norm, eps
                // 1e-12): tanh x 2^12, this wave's (mean, M2) over its valid rows, merged with its head's
                // other waves in wave order (Chan) into the MEMBER's statistics; the output layer then sees
                // h - mean_member (gamma is folded into the output weights, beta into their bias: capi.cpp),
                // and the team's exact (h - mean) sums are rebuilt after the exchange from the members'
                // statistics: sum_t P_t + sum_t (mean_t - mean) rs_t, times rsqrt(var + eps)
                const int nwr = min(max(a.hidden - 16 * TPW * g, 0), 16 * TPW);
                float s0 = 0.f, s1 = 0.f;
#pragma unroll
                for (int j = 0; j < TPW; ++j) {
                    const f4 b = *reinterpret_cast<const f4*>(Bh + 16 * (TPW * g + j) + 4 * q);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        acc1[j][r] = tanh4096(fmaf(acc1[j][r], f1, b[r]));     // pad rows: exactly 0
                        s0 += acc1[j][r];
                    }
                }
                s0 = add_rows(s0) * (nwr > 0 ? 1.0f / (float)nwr : 0.f);
#pragma unroll
                for (int j = 0; j < TPW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float d = acc1[j][r] - s0;
                        s1 += (16 * (TPW * g + j) + 4 * q + r < a.hidden) ? d * d : 0.f;
                    }
                s1 = add_rows(s1);
                float* const hx = xch + NWV * 32;
                if (q == 0) *reinterpret_cast<f2*>(hx + (w * 16 + m) * 2) = (f2){s0, s1};
                lds_barrier();                               // every wave's head statistics
#pragma unroll
                for (int hd = 0; hd < 2; ++hd) {
                    float mean = 0.f, m2 = 0.f, n = 0.f;
#pragma unroll
                    for (int v = 0; v < NH; ++v) {
                        const float nb = (float)min(max(a.hidden - 16 * TPW * (tm * NH + v), 0), 16 * TPW);
                        if (nb > 0.f) {
                            const f2 st = *reinterpret_cast<const f2*>(hx + ((hd * NH + v) * 16 + m) * 2);
                            const float nn = n + nb, d = st[0] - mean;
                            mean = mean + d * (nb / nn);
                            m2 = m2 + st[1] + d * d * (n * nb / nn);
                            n = nn;
                        }
                    }
                    hst[2 * hd] = mean;
                    hst[2 * hd + 1] = m2;
                }
                const float mc = rw_wave ? hst[2] : hst[0];
#pragma unroll
                for (int j = 0; j < TPW; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc1[j][r] -= mc;        // (pad rows: zero output weights)
                split_tiles<TPW>(acc1, g & 1, oh, ol);
            } else if constexpr (AK == 0 && TPW >= 2) {
#pragma unroll
                for (int pp = 0; pp < PPW; ++pp)
                    epi_pair_tanh(acc1[2 * pp], acc1[2 * pp + 1], f1, Bh, TPW * g + 2 * pp, q, oh[pp], ol[pp]);
            } else {
                if constexpr (AK == 0) {
                    const f4 b = *reinterpret_cast<const f4*>(Bh + 16 * g + 4 * q);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc1[0][r] = tanh4096(fmaf(acc1[0][r], f1, b[r]));
                } else if constexpr (DYN) {
                    epi_cols<AK, TPW, NWV, false>(acc1, f1, Bl + HP, lnp, lnp, 1.f, a.hidden, nullptr, g, w, lane,
                                                  fcol1);
                } else {
                    epi_cols<AK, TPW, NWV, true, false, DEFER>(acc1, f1, Bl + HP, lnp + HP, lnp + 3 * HP, a.hsc[1], a.hidden,
                                                 xch + NWV * 32, g, w, lane, fcol1);
                }
                split_tiles<TPW>(acc1, g & 1, oh, ol);
            }

            stamp(6);
            // ---- output layer [h -> S] (2 tiles), K-split: this wave's k-steps; partials summed in
            //      wave order, then member order ----
            f4 po[2] = {(f4){0.f, 0.f, 0.f, 0.f}, (f4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int pp = 0; pp < PPW; ++pp)
#pragma unroll
                for (int v = 0; v < 2; ++v) po[v] = mm3(woh[pp][v], wol[pp][v], oh[pp], ol[pp], po[v]);
            if constexpr (DYN || DEFER) {
                po[0] *= fcol1;                           // exact: undo this wave's column power of two
                po[1] *= fcol1;
            }
            parts[(w * 2 + 0) * 64 + lane] = po[0];
            parts[(w * 2 + 1) * 64 + lane] = po[1];
            lds_barrier();                                   // partials complete; every wave is done with the slab
            stamp(7);
            rstamp(h, 0);
            if constexpr (T == 1) {
                // (one term at a time here: the pipelined ordered_sum2 measured +1.5 us at ppo_defaults)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    ot[v] = parts[(0 * 2 + v) * 64 + lane];
#pragma unroll
                    for (int x = 1; x < NWV; ++x) ot[v] += parts[(x * 2 + v) * 64 + lane];
                }
                if constexpr (DEFER) {
                    // the deferred LayerNorm of the last hidden layer (its statistics published before the
                    // partials barrier): rows 16 v + 4 q + r of this lane's candidate
                    const float* const hx = xch + NWV * 32;
                    float mean, m2;
                    ln_merge<TPW, NWV, false>(hx, m, a.hidden, mean, m2);
                    const float rs = __builtin_amdgcn_rsqf(m2 * (1.0f / (float)a.hidden) + 1e-12f);
                    const float* const cw = lnp + HP;
                    f4 corr[2] = {(f4){0.f, 0.f, 0.f, 0.f}, (f4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int x = 0; x < NWV; ++x) {
                        const float dm = hx[(x * 16 + m) * 2] - mean;
#pragma unroll
                        for (int v = 0; v < 2; ++v) {
                            const f4 c4 = *reinterpret_cast<const f4*>(cw + x * 32 + 16 * v + 4 * q);
#pragma unroll
                            for (int r = 0; r < 4; ++r) corr[v][r] = fmaf(dm, c4[r], corr[v][r]);
                        }
                    }
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) ot[v][r] = rs * (ot[v][r] + corr[v][r]);
                }
            } else {
                // member partial: every wave sums the parts in wave order (the same bits in each)
                f4 mp[2];
                ordered_sum2<NWV>(parts, lane, mp);
                // exchange (rows < S, + row S for the reward net): wave 0 publishes this member's partial
                // as granules {epoch, f32} at k * 64 + lane (k = 4 v + r); member (tm + o) % T's are
                // collected by wave o % NWV; every partial lands in the LDS slot of its member
                const unsigned ep = (gen << 10) + (unsigned)h + 1u;
                // a member that gave up tags its granules of both parities with this launch's "dead" epoch
                // (h + 1 <= H <= 1022 never reaches 1023), so its partners -- and a member that only becomes
                // resident later -- give up at their next poll instead of spinning to their own limit
                const unsigned dep = (gen << 10) | 1023u;
                const size_t slot = ((size_t)col * 2 + (h & 1)) * T;
                const int R = S + (RW ? 1 : 0);           // rows exchanged: delta rows (+ the reward row)
                // (+ rows 24..27: the member's head statistics mean_d, M2_d, mean_r, M2_r, lane row q = 2)
                auto xrow = [&](int row) __attribute__((always_inline)) { return row < R || (HLN && (row >> 2) == 6); };
                if constexpr (HLN)
                    if (q == 2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) mp[1][r] = hst[r];
                if (w == 0) {
                    gu64* const mine = gb + (slot + tm) * 512;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (!dead && xrow(16 * (k >> 2) + 4 * q + (k & 3)))
                            __hip_atomic_store(mine + k * 64 + lane,
                                               ((unsigned long long)ep << 32) | __float_as_uint(mp[k >> 2][k & 3]),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    tot[(tm * 2 + 0) * 64 + lane] = mp[0];
                    tot[(tm * 2 + 1) * 64 + lane] = mp[1];
                }
                rstamp(h, 1);
                // member (tm + o) % T is collected by wave o % NWV; a wave with several members polls them
                // together (round 4: one round trip for all of them, not one after the other)
                constexpr int MO = (T - 1 + NWV - 1) / NWV;   // members per collecting wave (at most)
                f4 got[MO][2];
                bool have[MO];
                const gu64* srcs[MO];
                int tsrc[MO];
#pragma unroll
                for (int i = 0; i < MO; ++i) {
                    const int o = (w == 0 ? NWV : w) + i * NWV;  // o in [1, T), o % NWV == w
                    have[i] = !(o < T);                            // (no such member: nothing to collect)
                    tsrc[i] = (tm + (o < T ? o : 0)) % T;
                    srcs[i] = gb + (slot + tsrc[i]) * 512;
                    got[i][0] = got[i][1] = (f4){0.f, 0.f, 0.f, 0.f};
                }
                bool all_have = true;
#pragma unroll
                for (int i = 0; i < MO; ++i) all_have = all_have && have[i];
                for (int spins = 0; !dead && !all_have; ++spins) {
                    // one sweep: every granule of every missing member requested before any is tested (loads
                    // under a per-lane row test were each issued in an exec-masked branch and waited for
                    // before the next: 8 round trips per member per sweep, ~3 us from the last member's
                    // publish to every member in, TEAM_STAMP 3).  Granules of rows nobody exchanges are
                    // read too (in the buffer, never written) and ignored.
                    unsigned long long xv[MO][8];
#pragma unroll
                    for (int i = 0; i < MO; ++i)
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            xv[i][k] = have[i] ? 0ull
                                               : __hip_atomic_load(srcs[i] + k * 64 + lane, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                    all_have = true;
#pragma unroll
                    for (int i = 0; i < MO; ++i) {
                        if (have[i]) continue;
                        bool ok = true;
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            const bool vr = xrow(16 * (k >> 2) + 4 * q + (k & 3));
                            got[i][k >> 2][k & 3] = __uint_as_float((unsigned)xv[i][k]);
                            ok &= !vr || (unsigned)(xv[i][k] >> 32) == ep;
                        }
                        have[i] = __all(ok);
                        all_have = all_have && have[i];
                    }
                    if (all_have) break;
                    // (off the success path: every 32nd failed poll looks for a dead tag in row 0)
                    bool gone = false;
                    if ((spins & 31) == 31)
#pragma unroll
                        for (int i = 0; i < MO; ++i)
                            if (!have[i])
                                gone = gone || (unsigned)(__hip_atomic_load(srcs[i] + lane, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT) >> 32) == dep;
                    if (__any(gone) || spins >= spin_limit) {
                        // give up: raise the mapped error word (the host reruns the call on its fallback
                        // engine), tell this member's other waves (LDS) and the team (dead tags)
                        dead = true;
                        if (lane == 0) {
                            *tdead = 1;
                            if (a.team_err)
                                __hip_atomic_store(a.team_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                        // (granule row k = 0 of both parities: every poller reads it, rows 4q < R)
                        gu64* const mine = gb + ((size_t)col * 2 * T + tm) * 512 + lane;
                        __hip_atomic_store(mine, (unsigned long long)dep << 32, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(mine + (size_t)T * 512, (unsigned long long)dep << 32,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                rstamp(h, 2);
#pragma unroll
                for (int i = 0; i < MO; ++i) {
                    const int o = (w == 0 ? NWV : w) + i * NWV;
                    if (o < T) {
                        tot[(tsrc[i] * 2 + 0) * 64 + lane] = got[i][0];
                        tot[(tsrc[i] * 2 + 1) * 64 + lane] = got[i][1];
                    }
                }
                lds_barrier();                               // every member's partial in LDS
                rstamp(h, 3);
                dead = dead || *tdead != 0;
                ordered_sum2<T>(tot, lane, ot);              // member order
                if constexpr (HLN) {
                    // the heads' LayerNorm, completed: the team's (mean, M2) per head from the members'
                    // statistics (Chan, member order, identical in every member), then per output row i
                    // (delta rows < S: the delta head; row S: the reward head)
                    //   ot_i = rsqrt(M2 / hidden + eps) (sum_t P_t,i + sum_t (mean_t - mean) rs_t,i)
                    const float* const rs = lnp + HP;
                    const float* const tw = rs + T * 32;
                    float mean[2] = {0.f, 0.f}, m2[2] = {0.f, 0.f};
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        const f4 st = tot[(t * 2 + 1) * 64 + 32 + m];
                        const float w0 = tw[2 * t], w1 = tw[2 * t + 1];
#pragma unroll
                        for (int hd = 0; hd < 2; ++hd) {
                            const float d = st[2 * hd] - mean[hd];
                            mean[hd] = mean[hd] + d * w0;
                            m2[hd] = m2[hd] + st[2 * hd + 1] + d * d * w1;
                        }
                    }
                    float inv[2];
#pragma unroll
                    for (int hd = 0; hd < 2; ++hd)
                        inv[hd] = __builtin_amdgcn_rsqf(m2[hd] * (1.0f / (float)a.hidden) + 1e-12f * 16777216.0f);
                    f4 corr[2] = {(f4){0.f, 0.f, 0.f, 0.f}, (f4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        const f4 st = tot[(t * 2 + 1) * 64 + 32 + m];
                        const float dd = st[0] - mean[0], dr = st[2] - mean[1];
#pragma unroll
                        for (int v = 0; v < 2; ++v) {
                            const f4 rv = *reinterpret_cast<const f4*>(rs + t * 32 + 16 * v + 4 * q);
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                corr[v][r] = fmaf(16 * v + 4 * q + r == S ? dr : dd, rv[r], corr[v][r]);
                        }
                    }
#pragma unroll
                    for (int v = 0; v < 2; ++v)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * v + 4 * q + r;
                            ot[v][r] = i > S ? 0.f : (ot[v][r] + corr[v][r]) * inv[i == S ? 1 : 0];
                        }
                }
            }
            stamp(8);
            rstamp(h, 4);
        }
        if (writer && a.costs && valid && q == qc) a.costs[cand] = cost;
        if (writer && valid && q == qc) mybest = Best{a.amin.maximize ? -cost : cost, cand};
        if constexpr (TEAM_STAMP) {
            if (a.stamps && lane == 0)
                for (int k = 0; k < 10; ++k) a.stamps[((size_t)blockIdx.x * NWV + w) * 10 + k] = ph_[k];
        }
    }
    if (a.fused_argmin && w == 0) {
        // ---- np.argmin / argmax (controllers.py:82,152) in the launch's tail: every workgroup's best (wave 0
        //      holds the costs: member 0's writer lanes) into the scratch records, the last workgroup to
        //      arrive (ticket) reduces them and writes the result record + the done word -- no argmin launch
        //      (the split kernel's recipe, wave-level: cdna_hip_programming.md "In-launch split-K reduction") ----
        const ArgminArgs& am = a.amin;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const Best o{__shfl_xor(mybest.c, off), __shfl_xor(mybest.i, off)};
            if (better(o, mybest)) mybest = o;
        }
        unsigned last = 0;
        if (lane == 0) {
            __hip_atomic_store(&am.scratch_c[blockIdx.x], mybest.c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&am.scratch_i[blockIdx.x], mybest.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the act_out rows and the record before the ticket)
            const unsigned t = __hip_atomic_fetch_add(a.amin_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = t == gridDim.x - 1 ? 1u : 0u;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        last = __shfl(last, 0);
        if (last) {
            Best best{__builtin_inf(), INT64_MAX};
            for (unsigned b = lane; b < gridDim.x; b += 64) {
                const Best o{__hip_atomic_load(&am.scratch_c[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                             __hip_atomic_load(&am.scratch_i[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
                if (better(o, best)) best = o;
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const Best o{__shfl_xor(best.c, off), __shfl_xor(best.i, off)};
                if (better(o, best)) best = o;
            }
            // the record: index, cost, first action (lanes j < BCMPC_MAX_ACTION in parallel, as argmin_write_block)
            bcmpc_result* out = am.out;
            const int64_t bi = best.i;
            if (lane == 0) {
                out->best_index = am.cand_offset + bi;
                out->best_cost = am.maximize ? -best.c : best.c;
            }
            if (lane < BCMPC_MAX_ACTION) {
                double v = 0.0;
                if (bi < am.K && lane < am.A) {
                    const uint64_t g = (uint64_t)(am.cand_offset + bi);
                    v = am.act_out ? am.act_out[bi * am.A + lane]
                        : am.actions ? am.actions[bi * am.A + lane]
                                     : rng_action(am.seed, g, 0, lane, am.consts[6 * 32 + lane], am.consts[7 * 32 + lane]);
                }
                out->first_action[lane] = v;
            }
            if (lane == 0) {
                __hip_atomic_store(a.amin_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
                if (am.done) {
                    __threadfence_system();
                    __hip_atomic_store(am.done, am.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    if constexpr (T > 1) {
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
}

// geometry per padded hidden width and model kind (0 plain delta net, 1 + fused policy, 2 reward net
// with or without the policy): waves per member, layer-1 (head) tiles per wave, members per team
struct TeamShape {
    int nwv, tpw, members;
};
static TeamShape team_shape_of(int hidden_padded, int kind) {
    if (kind == 0) {
        switch (hidden_padded) {
            case 64: return {2, 2, 1};
            case 128: return {4, 2, 1};
            case 256: return {TEAM_NWV256, 16 / TEAM_NWV256, 1};
            case 512: return {4, 2, 4};
            default: return {0, 0, 0};
        }
    }
    if (kind == 1) {                                   // + fused policy (2 policy tiles per wave)
        switch (hidden_padded) {
            case 128: return {4, 2, 1};
            case 256: return {4, 4, 1};
            case 512: return {4, 2, 4};
            default: return {0, 0, 0};
        }
    }
    if (hidden_padded != 512) return {0, 0, 0};
    return TeamShape{TEAM_RW_NWV, 8 / TEAM_RW_NWV, 8};   // reward: delta / reward waves
}

int team_members(int hidden_padded, int kind) { return team_shape_of(hidden_padded, kind).members; }
int team_layer0_tiles(int hidden_padded, int kind) {
    const TeamShape t = team_shape_of(hidden_padded, kind);
    return t.nwv ? hidden_padded / 16 / t.nwv : 0;
}
int team_layer1_tiles(int hidden_padded, int kind) { return team_shape_of(hidden_padded, kind).tpw; }
int64_t team_blocks(int64_t K, int hidden_padded, int kind) {
    const int64_t ncol = (K + 15) / 16;
    return ((ncol + 7) / 8) * 8 * team_members(hidden_padded, kind);
}
size_t team_buf_bytes(int64_t K, int hidden_padded, int kind) {
    const int T = team_members(hidden_padded, kind);
    return T > 1 ? (size_t)((K + 15) / 16 + 8) * 2 * T * 512 * sizeof(unsigned long long) : 0;
}
bool team_rw_ln_built() { return true; }
static int team_kind(const RolloutArgs& a) { return a.model == BCMPC_MODEL_REWARD ? 2 : a.pL > 0 ? 1 : 0; }

template <int HP, int NWV, int TPW, int T, int AK, int PHP = 0, bool RW = false>
static hipError_t launch_team_t(const RolloutArgs& a, hipStream_t st) {
    int pw_bytes = 0;
    if constexpr (PHP > 0) {
        if (a.pL < 1 || a.pL > BCMPC_MAX_LAYERS || a.phidden_padded != PHP) return hipErrorInvalidValue;
        for (int l = 1; l < a.pL; ++l) pw_bytes += a.pwbytes[l];      // (LDS: the hidden->hidden layers)
    }
    const int lds = team_lds_bytes(HP, NWV, T, AK, RW, PHP, PHP > 0 ? a.pL : 0, pw_bytes);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)rollout_team<HP, NWV, TPW, T, AK, PHP, RW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (a.L != 2 || (a.model == BCMPC_MODEL_REWARD) != RW || (a.pL > 0) != (PHP > 0) || a.S + a.A > 32 ||
        a.S > 32 || a.A > 15 || a.H > 1022 || ((RW || PHP > 0) && a.S < 16) ||
        (a.cost == BCMPC_COST_CHEETAH && a.S < 18) || AK != ((a.act == BCMPC_ACT_RELU ? 1 : 0) | (a.ln ? 2 : 0)) ||
        (T > 1 && (!a.team_buf || !a.team_ctl)))
        return hipErrorInvalidValue;
    const int64_t blocks = team_blocks(a.K, HP, team_kind(a));
    hipLaunchKernelGGL((rollout_team<HP, NWV, TPW, T, AK, PHP, RW>), dim3((unsigned)blocks), dim3(64 * NWV), lds, st, a);
    return hipGetLastError();
}

template <int HP, int NWV, int TPW, int T, int PHP = 0>
static hipError_t launch_team_ak(const RolloutArgs& a, hipStream_t st) {
    const int ak = (a.act == BCMPC_ACT_RELU ? 1 : 0) | (a.ln ? 2 : 0);
    switch (ak) {
        case 0: return launch_team_t<HP, NWV, TPW, T, 0, PHP>(a, st);
        case 1: return launch_team_t<HP, NWV, TPW, T, 1, PHP>(a, st);
        case 2:
            if constexpr (T == 1) return launch_team_t<HP, NWV, TPW, T, 2, PHP>(a, st);
            return hipErrorInvalidValue;
        case 3:
            if constexpr (T == 1) return launch_team_t<HP, NWV, TPW, T, 3, PHP>(a, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rollout_team(const RolloutArgs& a, int hidden_padded, hipStream_t st) {
    const int kind = team_kind(a);
    if (kind == 1) {
        // + fused policy: any activation / LayerNorm at hidden <= 256 (one workgroup per column, e.g.
        // train_mpc_ppo.py's 2x256 relu + LN net); hidden 512: tanh, no LayerNorm (4 members)
        switch (hidden_padded) {
            case 128: return launch_team_ak<128, 4, 2, 1, 128>(a, st);
            case 256: return launch_team_ak<256, 4, 4, 1, 128>(a, st);
            case 512:
                if (a.act != BCMPC_ACT_TANH || a.ln) return hipErrorInvalidValue;
                return launch_team_t<512, 4, 2, 4, 0, 128, false>(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    if (kind > 0) {
        // the reward net: hidden 512, tanh (+ LayerNorm: the run.sh recipe's net, train_mpc_ppo.py:52)
        if (hidden_padded != 512 || a.act != BCMPC_ACT_TANH) return hipErrorInvalidValue;
        if (a.ln) {
            if (a.S > 23 || !a.head_rs) return hipErrorInvalidValue;
            if (a.pL > 0) return launch_team_t<512, TEAM_RW_NWV, 8 / TEAM_RW_NWV, 8, 2, 128, true>(a, st);
            return launch_team_t<512, TEAM_RW_NWV, 8 / TEAM_RW_NWV, 8, 2, 0, true>(a, st);
        }
        if (a.pL > 0) return launch_team_t<512, TEAM_RW_NWV, 8 / TEAM_RW_NWV, 8, 0, 128, true>(a, st);
        return launch_team_t<512, TEAM_RW_NWV, 8 / TEAM_RW_NWV, 8, 0, 0, true>(a, st);
    }
    switch (hidden_padded) {
        case 64: return launch_team_ak<64, 2, 2, 1>(a, st);
        case 128: return launch_team_ak<128, 4, 2, 1>(a, st);
        case 256: return launch_team_ak<256, TEAM_NWV256, 16 / TEAM_NWV256, 1>(a, st);
        case 512: return launch_team_ak<512, 4, 2, 4>(a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace bcmpc
