// capi.cpp -- C ABI of libbcmpc (include/bcmpc.h): engine lifetime, weight
// packing into MFMA fragment order, host<->device staging, launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/bcmpc.h"
#include "kernels.h"
#include "mt19937.h"

using namespace bcmpc;

// a host thread of the split NumPy-stream draw gets at least this many generator words
// (BCMPC_MT_MIN_WORDS overrides): below it the jump-ahead (~0.1 ms per thread) does not pay
static int64_t mt_min_words() {
    const char* v = std::getenv("BCMPC_MT_MIN_WORDS");
    return (v && *v) ? std::max<int64_t>(1, std::atoll(v)) : int64_t(1) << 20;
}

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(BCMPC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

int kern_waves(int kern) {
    return kern == BCMPC_KERNEL_GROUP8 ? 8 : kern == BCMPC_KERNEL_GROUP4 ? 4 : 1;
}

int padded_hidden(int h) {
    for (int hp : {64, 128, 256, 512, 768, 1024})
        if (h <= hp) return hp;
    return -1;
}

// Dense kernel W [in][out] (tf.layers.dense layout) -> fragment order
// [tb][u][j][lane][r], t = tb*TB + j: element W[16u + 4(lane>>4) + r][16t + (lane&15)]
// (zero outside in x out).  See the layout note at the top of rollout.hip.
void pack_layer(const float* W, int in, int out, int Tin, int Tout, int TB, float* dst) {
    for (int t = 0; t < Tout; ++t) {
        const int tb = t / TB, j = t % TB;
        for (int u = 0; u < Tin; ++u)
            for (int lane = 0; lane < 64; ++lane)
                for (int r = 0; r < 4; ++r) {
                    const int k = 16 * u + 4 * (lane >> 4) + r;
                    const int n = 16 * t + (lane & 15);
                    const size_t o = ((((size_t)tb * Tin + u) * TB + j) * 64 + lane) * 4 + r;
                    dst[o] = (k < in && n < out) ? W[(size_t)k * out + n] : 0.f;
                }
    }
}

// Output layer of the policy: one 16-row output tile whose row n holds action
// rowmap[n] (or zero): the host places action j at row S-16+j, i.e. in exactly
// the lanes/registers where the dynamics' layer-0 input expects action j.
void pack_out_rows(const float* W, int in, int out, int Tin, const int* rowmap, float* dst) {
    for (int u = 0; u < Tin; ++u)
        for (int lane = 0; lane < 64; ++lane)
            for (int r = 0; r < 4; ++r) {
                const int k = 16 * u + 4 * (lane >> 4) + r;
                const int c = rowmap[lane & 15];
                const size_t o = (((size_t)u * 64) + lane) * 4 + r;
                dst[o] = (k < in && c >= 0 && c < out) ? W[(size_t)k * out + c] : 0.f;
            }
}

// Split-f16 kernel (rollout_x3.hip): W [in][out] scaled by sw, every element as
// hi = f16(w), lo = f16(w - hi), in fragment order [ws][p][j][hi|lo][lane][i],
// t = ws*TWp + j: lane's 8 halves of tile t, k-step p are W[k][n] with
// n = 16t + (lane&15), k = 32p + 16(i>>2) + 4(lane>>4) + (i&3) -- the k order in
// which an output tile pair's accumulators ARE the next layer's B fragment.
void pack_x3_layer(const float* W, int in, int out, int Pin, int Tout, int TWp, float sw, _Float16* dst) {
    for (int t = 0; t < Tout; ++t) {
        const int ws = t / TWp, j = t % TWp;
        for (int p = 0; p < Pin; ++p)
            for (int lane = 0; lane < 64; ++lane)
                for (int i = 0; i < 8; ++i) {
                    const int k = 32 * p + 16 * (i >> 2) + 4 * (lane >> 4) + (i & 3);
                    const int n = 16 * t + (lane & 15);
                    const float v = (k < in && n < out) ? W[(size_t)k * out + n] * sw : 0.f;
                    const _Float16 hi = (_Float16)v;
                    const _Float16 lo = (_Float16)(v - (float)hi);
                    const size_t o = ((((size_t)ws * Pin + p) * TWp + j) * 2 * 64 + lane) * 8 + i;
                    dst[o] = hi;
                    dst[o + 64 * 8] = lo;
                }
    }
}

// power of two s with max|W| * s in [2^11, 2^12) (1 for an all-zero kernel)
float x3_scale(const float* W, size_t n) {
    float mx = 0.f;
    for (size_t i = 0; i < n; ++i) mx = std::max(mx, std::fabs(W[i]));
    if (!(mx > 0.f) || !std::isfinite(mx)) return 1.f;
    int e = 0;
    (void)std::frexp(mx, &e);
    return std::ldexp(1.0f, std::max(-100, std::min(100, 12 - e)));
}

}  // namespace

namespace bcmpc {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace bcmpc

// Diagnostic hooks: the per-phase stamps of STAMP variant kernels (BCMPC_X3_STAMPS, BCMPC_STAMP_DUMP) are read
// only by a diagnostic build (-DBCMPC_DIAG_VARIANT: tools/build_variants.sh, tools/team_variants.sh); the
// production library never consults them.
static const char* diag_env(const char* name) {
#ifdef BCMPC_DIAG_VARIANT
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Fault-injection hooks the GPU tests use (BCMPC_TEAM_SPINS=-1: every team gives up; comm.hip's
// BCMPC_COMM_FORCE_FLAGS): read in every build, and announced on stderr once per process when set, so a stray
// variable on a production run is visible.
namespace bcmpc {
void announce_test_hook(const char* name, const char* value) {
    static std::atomic<unsigned> said{0};
    const unsigned bit = name[6] == 'C' ? 1u : 2u;      // BCMPC_COMM_* / BCMPC_TEAM_*
    if (!(said.fetch_or(bit) & bit))
        std::fprintf(stderr, "libbcmpc: test hook %s=%s is active (fault injection; unset it for real runs)\n",
                     name, value);
}
}  // namespace bcmpc

static thread_local bool g_no_team = false;         // bcmpc_create: never pick the team kernel (fallbacks)

struct bcmpc_engine {
    bcmpc_config cfg{};
    int HP = 0, T = 0, wpb = 4;
    int kernel = BCMPC_KERNEL_SOLO;    // resolved kernel layout
    int nw = 1;                        // waves per group (group kernels)
    int pack_tb = 4;                   // output tiles per packed block of layers 0..L-1
    bool split = false;                // BCMPC_PREC_SPLIT_F16 or F16 (rollout_x3)
    bool f16 = false;                  // BCMPC_PREC_F16: single MFMA pass
    bool pp = false;                   // BCMPC_PREC_F16 on the two-group pipelined kernel (rollout_pp)
    bool pp_fold = false;              // ... with the folded operands (rollout_pp<, FOLD>; BCMPC_PP_FOLD=0: off)
    bool pp_fold_w = false;            //     active for the current weights (|W| x 2 log2 e within f16's range)
    int nc = 0;                        // split kernel: 16-candidate columns per workgroup
    int nwl = 0;                       // packed weight layers (RolloutArgs.w entries)
    float winv[BCMPC_MAX_LAYERS + 1]{};  // split kernel: 1 / operand scales per layer
    float pwinv[BCMPC_MAX_LAYERS + 1]{}; // ... and per fused-policy layer
    float hsc[BCMPC_MAX_LAYERS]{};       // split LN nets: output scale of hidden layer l
    bool reward = false;               // BCMPC_MODEL_REWARD (NNDynamicsRewardModel)
    hipStream_t stream = nullptr;
    // device buffers
    float* d_w = nullptr;   size_t w_floats = 0;
    size_t w_off[BCMPC_MAX_LAYERS + 1]{};
    float* d_b = nullptr;   size_t b_off[BCMPC_MAX_LAYERS + 1]{};
    float* d_ln = nullptr;  // [2][L][HP]
    double* d_consts = nullptr;
    double* d_state = nullptr;
    double* d_actions = nullptr; size_t actions_cap = 0;
    double* h_stage = nullptr; size_t stage_cap = 0;   // pinned [H, K, A] staging (bcmpc_get_action_mt19937)
    // small NumPy-stream draws: two fine-grained (coherent) pinned row buffers and their device addresses
    // (the kernel reads them over the bus); a call uses one while the pre-draw worker fills the other
    double* h_zc[2] = {nullptr, nullptr}; size_t zc_cap = 0;
    double* d_zc[2] = {nullptr, nullptr};
    // late pre-draw hit (team kernel): the worker publishes each job's sequence number into this mapped
    // host word after its last row; a call that finds its rows still being drawn launches at once and the
    // kernel waits for the word (BCMPC_MT_PREDRAW_LATE=0: the call waits on the host instead)
    uint32_t* h_rows_seq = nullptr;
    uint32_t* d_rows_seq = nullptr;
    uint32_t rows_wait_seq = 0;         // (the next team launch waits for this sequence number; 0: none)
    // the pre-draw worker also copies its rows into device memory (copy stream + event per buffer) while the
    // caller's env step runs; a call whose copy has completed reads HBM instead of the bus (zero-copy rows
    // cost the K = 400 kernel 3.7 us; BCMPC_MT_PREDRAW_DEV=0 turns the copy off)
    double* d_rows[2] = {nullptr, nullptr};
    hipStream_t copy_st = nullptr;
    hipEvent_t copy_ev[2] = {nullptr, nullptr};
    bool copy_valid[2] = {false, false};
    int zc_last = 0;                    // the buffer the last successful call read
    // pre-draw (BCMPC_MT_PREDRAW, default on): after a successful small draw, a worker thread draws the
    // rows the NEXT call would draw -- from NumPy's advanced state, same bounds / shard -- into the other
    // buffer; the next call uses them only if NumPy's state is still exactly that state
    struct PreDraw {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        bool quit = false, pending = false, busy = false, ready = false;
        // lock-free mirrors for the spinning handshake: a job posted and not yet finished / shutting down
        std::atomic<bool> inflight{false}, quit_a{false};
        std::atomic<bool> claimed{false};   // a call already reads this job's pinned rows: no device copy
        uint32_t job = 0;                   // the posted job's sequence number (published to h_rows_seq)
        bool rows = true;               // false: only NumPy's state is needed (the stochastic policy)
        Mt19937 from, to;               // the state the rows were drawn from / leave behind
        std::vector<double> low, high;
        int64_t kg = 0, off = 0;
        int buf = 0;
        uint64_t hits = 0, late = 0, misses = 0;   // hits include the late ones
    } pre;
    double* d_costs = nullptr;
    bcmpc_result* d_result = nullptr;
    double* d_amin_c = nullptr;         // argmin scratch: per-block best
    int64_t* d_amin_i = nullptr;
    size_t amin_cap = 0;                // records the scratch holds
    unsigned* d_amin_ticket = nullptr;  // fused argmin (split kernel): last-workgroup ticket
    // team kernel (rollout_team.hip): exchange granules, {ticket, generation}, mapped timeout flag
    unsigned long long* d_team = nullptr;
    int team_kind = 0;                  // 0 plain delta net, 1 + policy, 2 reward net (+ policy)
    bool team_defer = false;            // the weights are packed for rollout_team's deferred last LayerNorm
    unsigned* d_team_ctl = nullptr;
    unsigned* h_team_err = nullptr;
    unsigned* d_team_err = nullptr;
    bcmpc_result* h_result = nullptr;   // pinned
    // the synchronous control steps' result: pinned, mapped, coherent host memory the argmin kernel
    // writes directly (no device-to-host copy; the stream synchronisation orders it)
    bcmpc_result* h_result_map = nullptr;
    bcmpc_result* d_result_map = nullptr;
    // ... and its completion word (argmin_write raises seq; wait_done spins on it)
    unsigned long long* h_done = nullptr;
    unsigned long long* d_done = nullptr;
    unsigned long long seq = 0;
    bool want_done = false;             // the next rollout_impl's argmin raises the done word
    double h_consts[kConstRows * kConstCols]{};
    uint64_t version = 0;
    bool has_weights = false;
    hipEvent_t ev[3]{};
    bool timed = false;                 // the last launch chain recorded ev[0..2]
    bool timing = false;                // bcmpc_engine_set_timing: bracket launches with HIP events
    // fused policy (MPCcontrollerPolicyNet)
    int PHP = 0, TP = 0, PL = 0;
    float* d_pw = nullptr;  size_t pw_floats = 0;  size_t pw_off[BCMPC_MAX_LAYERS + 1]{};
    float* d_pb = nullptr;                          // [PL][PHP] + kPolParams
    double* d_first = nullptr;                      // [K][A] step-0 actions
    // learned reward (NNDynamicsRewardModel)
    double* d_gpow = nullptr;                       // [H] gamma**h
    double mean_reward = 0.0, std_reward = 0.0;
    // CEM (bcmpc_cem_get_action)
    double* d_mu = nullptr;                         // [H][A] each
    double* d_sigma = nullptr;
    bcmpc_elite* d_elite = nullptr; int32_t elite_cap = 0;
    int32_t* d_count = nullptr;
    double explore = 0.0;
    uint64_t pol_version = 0;
    bool has_policy = false;
    // NumPy-stream draw on the device (bcmpc_get_action_mt19937, mt_device.hip): chunk plan and jump
    // polynomials per (k_global, cand_offset), built on the first call of that shape
    int64_t mt_kg = -1, mt_off = -1;
    int32_t mt_nchunks = 0, mt_cj = 0, mt_s = 0;
    uint32_t* d_mt_io = nullptr;        // [0, 625) key + pos in, [640, 1265) final key + pos out
    double* d_mt_bounds = nullptr;      // [2][A] low, high
    uint32_t* d_mt_xs = nullptr;        // [kMtStream]
    uint32_t* d_mt_polys = nullptr;     // [Cj][kMtPolyWords]
    MtChunk* d_mt_chunks = nullptr;
    uint32_t* d_mt_part = nullptr;      // [Cj][S][624]
    uint32_t* h_mt_io = nullptr;        // pinned mirror of d_mt_io (+ bounds at word 1280)
    // speculative device draw (BCMPC_MT_SPECULATE, default on): right behind a device-path call's argmin, the
    // NEXT call's draw is enqueued from this draw's final state -- still on the device, no host round trip --
    // into a slot of its own; the next call uses it when NumPy's state, bounds and shard equal its start
    // (else it is discarded: two misses in a row pause speculation for kSpecPause calls)
    struct Spec {
        uint32_t* d_io = nullptr;       // [0, 625) final key + pos, then [2][A] bounds (f64) from word 640
        uint32_t* h_io = nullptr;       // pinned mirror
        double* d_act = nullptr;        // the shard's [H][K][A] rows
    } spec[2];
    size_t spec_cap = 0;
    bool spec_armed = false;
    int spec_slot = 0, spec_miss_run = 0, spec_pause = 0;
    uint32_t spec_key[624];
    int32_t spec_pos = 0;
    int64_t spec_kg = 0, spec_off = 0;
    double spec_low[BCMPC_MAX_ACTION], spec_high[BCMPC_MAX_ACTION];
    uint64_t spec_hits = 0, spec_misses = 0;
    // slab-kernel engines draw beside the rollout: the speculative draw runs on spec_st, concurrently with
    // this call's rollout (spec_in_ev: this call's draw has left its final state), with scratch of its own;
    // spec_done_ev closes it and every later draw / rollout that touches its slots waits for it
    hipStream_t spec_st = nullptr;
    hipEvent_t spec_in_ev = nullptr, spec_done_ev = nullptr;
    bool spec_side_pending = false;
    int ncu = 0;                        // the device's CUs
    uint32_t* d_spec_xs = nullptr;
    uint32_t* d_spec_part = nullptr;
    bcmpc_comm* comm = nullptr;         // attached communicator: results exchanged after every argmin
    // team kernel: a team that could not meet (its workgroups not all resident: another process or
    // kernel holding CUs for ~1 s) makes a synchronous call rerun on this fallback engine -- the same
    // net on the split slab kernel, or the fp32 group kernel where only the team kernel takes the net
    // in split precision -- created on first need and synced from the host copies kept below
    bcmpc_engine* fb = nullptr;
    uint64_t fb_wver = 0, fb_pver = 0;
    bool fb_wset = false, fb_pset = false;
    uint64_t team_reruns = 0;
    bool sync_call = false;             // inside a synchronous entry point (its launches complete before it returns)
    struct HostNet {                    // the last bcmpc_set_weights / bcmpc_set_policy, copied
        std::vector<std::vector<float>> k, b, g, beta;
        std::vector<double> st[8];      // mean/std obs, action, deltas, reward
        std::vector<float> pvec[3];     // (policy) ob_mean, ob_std, logstd
        double explore = 0.0;
        bool ln = false;
    } hw_copy, hp_copy;
    double gamma = 1.0;
};

// (team launch ordering across streams: team_order_before / team_order_after below)
struct TeamOrder {
    std::mutex mu;
    hipEvent_t ev = nullptr;
    hipStream_t ev_stream = nullptr;
    bool pending = false;
};
static TeamOrder g_team_order[64];

extern "C" {

int bcmpc_abi_version(void) { return BCMPC_ABI_VERSION; }
const char* bcmpc_last_error(void) { return g_last_error.c_str(); }

int bcmpc_create(const bcmpc_config* cfg, bcmpc_engine** out) {
    if (!cfg || !out) return fail(BCMPC_ERR_ARG, "null argument");
    *out = nullptr;
    const bcmpc_config& c = *cfg;
    if (c.state_dim < 1 || c.state_dim > BCMPC_MAX_STATE) return fail(BCMPC_ERR_UNSUPPORTED, "state_dim must be in [1, 32]");
    if (c.action_dim < 1 || c.action_dim > BCMPC_MAX_ACTION) return fail(BCMPC_ERR_UNSUPPORTED, "action_dim must be in [1, 16]");
    if (c.state_dim + c.action_dim > BCMPC_MAX_INPUT) return fail(BCMPC_ERR_UNSUPPORTED, "state_dim + action_dim must be <= 32");
    if (c.n_layers < 1 || c.n_layers > BCMPC_MAX_LAYERS) return fail(BCMPC_ERR_UNSUPPORTED, "n_layers must be in [1, 8]");
    if (padded_hidden(c.hidden) < 0 || c.hidden < 1) return fail(BCMPC_ERR_UNSUPPORTED, "hidden must be in [1, 1024] in this build");
    if (c.activation != BCMPC_ACT_TANH && c.activation != BCMPC_ACT_RELU) return fail(BCMPC_ERR_UNSUPPORTED, "activation must be tanh or relu");
    if (c.horizon < 1) return fail(BCMPC_ERR_ARG, "horizon must be >= 1");
    if (c.num_paths < 0) return fail(BCMPC_ERR_ARG, "num_paths must be >= 0");
    if (c.cost != BCMPC_COST_CHEETAH && c.cost != BCMPC_COST_NONE && c.cost != BCMPC_COST_REWARD)
        return fail(BCMPC_ERR_UNSUPPORTED, "unknown cost");
    if (c.model != BCMPC_MODEL_DELTA && c.model != BCMPC_MODEL_REWARD) return fail(BCMPC_ERR_ARG, "unknown model");
    const bool reward = c.model == BCMPC_MODEL_REWARD;
    if ((c.cost == BCMPC_COST_REWARD) != reward)
        return fail(BCMPC_ERR_ARG, "the learned-reward objective and BCMPC_MODEL_REWARD go together "
                                   "(MPCcontrollerReward needs NNDynamicsRewardModel, controllers.py:137)");
    if (reward) {
        if (c.n_layers != 2) return fail(BCMPC_ERR_ARG, "reward model: n_layers must be 2 (trunk + head, dynamics.py:167-174)");
        if (c.activation != BCMPC_ACT_TANH) return fail(BCMPC_ERR_UNSUPPORTED, "reward model is tanh (dynamics.py:150)");
        if (c.hidden > 512) return fail(BCMPC_ERR_UNSUPPORTED, "reward model: hidden must be <= 512 in this build");
        if (c.state_dim > 31) return fail(BCMPC_ERR_UNSUPPORTED, "reward model: state_dim must be <= 31");
    }
    if (c.cost == BCMPC_COST_CHEETAH && c.state_dim < 18) return fail(BCMPC_ERR_UNSUPPORTED, "cheetah cost needs state_dim >= 18");
    if (c.precision != BCMPC_PREC_FP32 && c.precision != BCMPC_PREC_SPLIT_F16 && c.precision != BCMPC_PREC_F16)
        return fail(BCMPC_ERR_UNSUPPORTED, "precision must be FP32, SPLIT_F16 or F16");
    // single-pass f16 (BASELINE cfg3's bf16-class GEMM): the split slab kernels' plain tanh delta net only
    const bool f16 = c.precision == BCMPC_PREC_F16;
    if (f16 && (reward || c.policy_hidden > 0 || c.activation != BCMPC_ACT_TANH || c.layer_norm))
        return fail(BCMPC_ERR_UNSUPPORTED, "F16 precision: the tanh NNDynamicsModel without LayerNorm / policy only");
    if (f16 && c.kernel != BCMPC_KERNEL_AUTO && (c.kernel < BCMPC_KERNEL_SPLIT1 || c.kernel > BCMPC_KERNEL_SPLIT4))
        return fail(BCMPC_ERR_ARG, "F16 precision runs on the split1/split2/split4 kernels");
    const bool split = c.precision != BCMPC_PREC_FP32;
    // relu / LayerNorm hidden layers (per-column scales or statistics exchanged across the workgroup)
    // on the split slab kernels: the plain delta net without a policy, hidden <= 512; beyond that only
    // the small-K team kernel takes them (checked once the kernel is chosen, below)
    const bool split_needs_team = split && (c.activation != BCMPC_ACT_TANH || c.layer_norm) &&
                                  (reward || c.policy_hidden > 0 || padded_hidden(c.hidden) > 512);
    if (split) {
        if (reward && c.state_dim < 16)
            return fail(BCMPC_ERR_UNSUPPORTED, "split reward engines need state_dim >= 16 (reward row in tile 1)");
        if (c.kernel != BCMPC_KERNEL_AUTO && (c.kernel < BCMPC_KERNEL_SPLIT1 || c.kernel > BCMPC_KERNEL_TEAM))
            return fail(BCMPC_ERR_ARG, "SPLIT_F16 precision runs on the split1/split2/split4/team kernels");
        if (c.kernel == BCMPC_KERNEL_SPLITR)
            return fail(BCMPC_ERR_UNSUPPORTED, "the splitr (resident-column) kernel was retired: slower than the "
                                               "split slab kernel at every K (DESIGN.md 6.5); use auto or split4");
    } else if (c.kernel >= BCMPC_KERNEL_SPLIT1) {
        return fail(BCMPC_ERR_ARG, "split kernels need precision SPLIT_F16");
    }
    if (c.kernel == BCMPC_KERNEL_GROUP2)
        return fail(BCMPC_ERR_UNSUPPORTED, "the group2 layout (2-wave f32 groups, A/B only, never chosen by auto) "
                                           "was retired; use auto, group4 or group8");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (c.device < 0 || c.device >= ndev) return fail(BCMPC_ERR_ARG, "device ordinal out of range");
    HIP_TRY(hipSetDevice(c.device));

    bcmpc_engine* e = new bcmpc_engine();
    e->cfg = c;
    e->reward = reward;
    e->f16 = f16;
    e->HP = reward ? std::max(128, padded_hidden(c.hidden)) : padded_hidden(c.hidden);
    e->T = e->HP / 16;
    // small K: one wave per block spreads candidates over more CUs
    const int64_t waves = (c.num_paths + 15) / 16;
    e->wpb = std::min(waves >= 4 * 256 ? 4 : 1, max_waves_per_block(e->HP, c.n_layers));
    // auto: 4-wave groups; 8-wave groups when K is too small to give every SIMD two waves
    int kern = c.kernel != BCMPC_KERNEL_AUTO ? c.kernel
             : ((c.num_paths + 15) / 16 < 512 && e->T % 8 == 0 ? BCMPC_KERNEL_GROUP8 : BCMPC_KERNEL_GROUP4);
    if (reward) {
        // two-head net: 4-wave groups (16 head tiles per wave, spill-free at 2 waves/SIMD; the
        // 8-wave layout needs ~135 registers and spills at 4 waves/SIMD -- measured 2.5% slower)
        if (!split && c.kernel != BCMPC_KERNEL_AUTO && c.kernel != BCMPC_KERNEL_GROUP4 &&
            c.kernel != BCMPC_KERNEL_GROUP8)
            { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "reward engines run on the group4 / group8 kernels"); }
        if (c.kernel == BCMPC_KERNEL_AUTO) kern = BCMPC_KERNEL_GROUP4;
    }
    if (c.policy_hidden > 0) {
        // MPCcontrollerPolicyNet: the policy MLP is fused into the 4-wave group kernel
        if (c.policy_hidden > 128 || c.policy_layers < 1 || c.policy_layers > BCMPC_MAX_LAYERS)
            { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "policy: hidden must be in [1,128], layers in [1,8]"); }
        if (c.state_dim < 16) { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "policy engines need state_dim >= 16"); }
        if (e->HP < 128 || e->HP > (split ? 1024 : 512))
            { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "policy engines support dynamics hidden 65..512 (split: ..1024)"); }
        if (c.policy_mode != BCMPC_POLICY_EXPLORE && c.policy_mode != BCMPC_POLICY_STOCHASTIC)
            { delete e; return fail(BCMPC_ERR_ARG, "unknown policy_mode"); }
        if (!split && c.kernel != BCMPC_KERNEL_AUTO && c.kernel != BCMPC_KERNEL_GROUP4 &&
            c.kernel != BCMPC_KERNEL_GROUP8)
            { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "policy engines run on the group4 / group8 kernels"); }
        if (c.kernel == BCMPC_KERNEL_AUTO) kern = BCMPC_KERNEL_GROUP4;
        e->PHP = 128;
        e->TP = 8;
        e->PL = c.policy_layers;
    }
    // small-K team kernel (rollout_team.hip): the 2-layer delta net at hidden <= 512 (LayerNorm: <=
    // 256), or at hidden 512 (tanh) with a fused policy of <= 2 layers and / or the reward net (the
    // run.sh recipe), when the whole grid fits one workgroup per CU (the team members of a column wait
    // for each other).  Auto: whenever it fits, unless BCMPC_TEAM=0
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c.device);
    e->ncu = ncu;
    const int tkind = reward ? 2 : e->PL > 0 ? 1 : 0;
    const int tmem = team_members(e->HP, tkind);
    // (a LayerNorm over a layer split across members: only the reward net's heads, whose statistics
    //  ride along with the output partials in the exchange -- rows 24..27, so S + 1 <= 24)
    const bool team_shape = split && !f16 && c.n_layers == 2 && e->HP <= 512 && c.state_dim + c.action_dim <= 32 &&
                            c.action_dim <= 15 && c.horizon <= 1022 && tmem > 0 &&
                            !(c.layer_norm && tmem > 1 && tkind != 2) &&
                            (tkind == 0 || (c.state_dim >= 16 && e->PL <= 2 &&
                                            (tmem == 1 || c.activation == BCMPC_ACT_TANH))) &&
                            !(tkind == 2 && c.layer_norm && (c.state_dim > 23 || !team_rw_ln_built()));
    const bool team_fits = team_shape && c.num_paths > 0 && team_blocks(c.num_paths, e->HP, tkind) <= (int64_t)ncu;
    bool use_team = c.kernel == BCMPC_KERNEL_TEAM;
    if (use_team && !team_fits) {
        delete e;
        return fail(BCMPC_ERR_UNSUPPORTED, "team kernel: 2-layer net, hidden <= 512 (LayerNorm: <= 256; with a "
                                           "policy: hidden <= 256, or 512 tanh without LayerNorm; the reward "
                                           "net: 512, tanh, LayerNorm with S <= 23), S + A <= 32, "
                                           "ceil(K / 128) * 8 * members workgroups <= the device's CUs");
    }
    if (c.kernel == BCMPC_KERNEL_AUTO && team_fits && !g_no_team) {
        const char* ev = std::getenv("BCMPC_TEAM");
        use_team = !(ev && ev[0] == '0');
    }
    if (use_team) {
        e->split = true;
        e->nc = 1;
        e->kernel = BCMPC_KERNEL_TEAM;
        e->nw = e->HP / 16 / team_layer0_tiles(e->HP, tkind);
        e->team_kind = tkind;
        kern = e->kernel;
    } else if (split) {
        // widest workgroup (most candidates per weight read) that still gives every CU work and fits LDS
        const int64_t cols = (c.num_paths + 15) / 16;
        int nc = c.kernel == BCMPC_KERNEL_SPLIT1 ? 1 : c.kernel == BCMPC_KERNEL_SPLIT2 ? 2
               : c.kernel == BCMPC_KERNEL_SPLIT4 ? 4 : 0;
        const int nwx = x3_waves(e->HP);
        auto fits = [&](int n) {
            return n <= nwx && n <= x3_max_nc(e->HP) && (e->PL == 0 || x3_policy_ok(e->HP, n)) &&
                   x3_lds(e->HP, reward ? 3 : c.n_layers, n, c.action_dim, e->PL, e->PHP,
                          (c.activation == BCMPC_ACT_RELU ? 1 : 0) | (c.layer_norm ? 2 : 0)) <= 160 * 1024;
        };
        int nw = nwx;
        if (f16) {
            // single-pass f16: the hi-only slab admits wider groups (x3_f16_layout_ok); BCMPC_F16_NC /
            // BCMPC_F16_NW pick a layout for A/B runs
            auto f16_fits = [&](int n, int w) {
                return x3_f16_layout_ok(e->HP, n, w) &&
                       x3_f16_lds(e->HP, c.n_layers, n, w, c.action_dim) <= 160 * 1024;
            };
            const char* en = std::getenv("BCMPC_F16_NC");
            const char* ew = std::getenv("BCMPC_F16_NW");
            const char* ep = std::getenv("BCMPC_F16_PP");
            // (default at large K, where it measured ahead of the two-group 4x4 layout below on every box:
            //  0.835-0.848 vs 0.898-0.900 ms at cfg3, profiles/r04_pp_ab.jsonl; BCMPC_F16_PP=1 forces it at any
            //  K, =0 turns it off)
            const bool pp_env = ep && *ep;
            if (!(en && *en) && !(ew && *ew) && x3_pp_ok(e->HP, c.n_layers, c.state_dim, c.action_dim) &&
                !reward && e->PL == 0 && c.activation == BCMPC_ACT_TANH && !c.layer_norm &&
                (pp_env ? ep[0] == '1' && cols >= 8 : cols >= 4 * 512)) {
                // the two-group pipelined kernel (rollout_pp): 128 candidates per workgroup, 4 waves per
                // group own 8 hidden tiles each (weights packed 8 tiles per wave)
                e->pp = true;
                // FOLD's input range: layer 0's normalised input goes to f16 without a power-of-two scale,
                // clamped to +-65504 (a dim normalising beyond saturates; the first tanh has saturated long
                // before) and below 6.1e-5 subnormal (< 6e-8 absolute error); the fold check below bounds
                // only the weights.  Pinned by tests/test_gpu_f16.py::test_f16_pp_fold_input_range
                const char* ef = std::getenv("BCMPC_PP_FOLD");
                e->pp_fold = !(ef && ef[0] == '0');
                nc = 8;
                nw = 8;
            }
            if (en && *en) nc = std::atoi(en);
            if (ew && *ew) nw = std::atoi(ew);
            if (!e->pp && nc == 0 && !(ew && *ew) && e->HP == 512 && cols >= 4 * 512 && f16_fits(4, 4)) {
                // two 64-candidate 4-wave groups per CU: 0.90 ms at cfg3 against 0.94 (one 8-wave group of
                // 64) and 0.91 (one of 128), three boxes (profiles/r04_f16_layouts_ab.txt)
                nc = 4;
                nw = 4;
            }
            if (nc == 0) {
                nc = 1;
                for (int n : {8, 4, 2})
                    if (f16_fits(n, nw) && cols >= (int64_t)n * 256 && !(n >= 4 && e->HP <= 256)) { nc = n; break; }
            }
            if (!e->pp && !f16_fits(nc, nw)) {
                delete e;
                return fail(BCMPC_ERR_UNSUPPORTED, "F16 precision: no single-pass layout for this shape / NC / NW");
            }
        } else if (nc == 0) {
            nc = 1;
            // (hidden <= 256: 32-candidate groups, two or three workgroups per CU, measured 6-18% ahead of 64)
            for (int n : {4, 2})
                if (fits(n) && cols >= (int64_t)n * 256 && !(n == 4 && e->HP <= 256)) { nc = n; break; }
        }
        if (!f16 && !fits(nc)) {
            delete e;
            return fail(BCMPC_ERR_UNSUPPORTED, e->PL ? "split kernel with a fused policy needs dynamics hidden 449..1024"
                                                     : "split kernel does not fit this shape");
        }
        e->split = true;
        e->nc = nc;
        e->kernel = nc == 1 ? BCMPC_KERNEL_SPLIT1 : nc == 2 ? BCMPC_KERNEL_SPLIT2 : BCMPC_KERNEL_SPLIT4;
        e->nw = nw;
        kern = e->kernel;
    }
    if (split_needs_team && !use_team) {
        delete e;
        return fail(BCMPC_ERR_UNSUPPORTED, "SPLIT_F16 precision supports relu / LayerNorm nets with a policy, the "
                                           "reward net or hidden > 512 only on the small-K team kernel (use FP32)");
    }
    if (kern < BCMPC_KERNEL_SOLO || kern > BCMPC_KERNEL_TEAM) { delete e; return fail(BCMPC_ERR_ARG, "unknown kernel"); }
    const int nw = split ? e->nw : kern_waves(kern);
    if (!split && kern != BCMPC_KERNEL_SOLO &&
        (e->T % nw != 0 || grp_lds_bytes(e->HP, c.n_layers, nw, e->PHP, e->PL, c.model) > 160 * 1024)) {
        if (c.kernel != BCMPC_KERNEL_AUTO) { delete e; return fail(BCMPC_ERR_UNSUPPORTED, "group kernel does not fit this shape"); }
        kern = BCMPC_KERNEL_SOLO;
    }
    if (kern == BCMPC_KERNEL_SOLO && (e->wpb < 1 || e->HP > 512)) {
        delete e;
        return fail(BCMPC_ERR_UNSUPPORTED, "solo kernel supports hidden <= 512 and needs LDS for its slabs");
    }
    e->kernel = kern;
    e->nw = nw;
    e->pack_tb = kern == BCMPC_KERNEL_SOLO ? 4 : e->pp ? e->T / 4 : e->T / nw;   // split: output tiles per wave
    const int L = c.n_layers, T = e->T;
    size_t off = 0, boff = 0;
    e->nwl = reward ? 3 : L + 1;
    if (reward && split) {
        // split layout: trunk, delta head hidden (dense_1), delta out (dense_2), reward head
        // hidden (dense_3), reward out (dense_4, one 16-row tile); 512 floats = one 2-KiB fragment pair
        const int P = T / 2;
        e->w_off[0] = off; off += (size_t)T * 512;
        e->w_off[1] = off; off += (size_t)T * P * 512;
        e->w_off[2] = off; off += (size_t)2 * P * 512;
        e->w_off[3] = off; off += (size_t)T * P * 512;
        e->w_off[4] = off; off += (size_t)P * 512;
        e->nwl = 5;
        // biases: trunk | delta head | reward head | out (rows 0..S-1 dense_2, row S dense_4) | (team kernel,
        // LayerNorm heads) the centring table [8 members][32 rows]
        e->b_off[0] = 0; e->b_off[1] = e->HP; e->b_off[2] = 2 * e->HP; e->b_off[3] = 3 * e->HP;
        e->b_off[4] = 3 * e->HP + 32;
        boff = 3 * e->HP + 32 + 8 * 32;
    } else if (reward) {
        // [S+A -> h] trunk, [h -> 2h] both heads' hidden layers, [2h -> S+1] block-diagonal output
        e->w_off[0] = off; off += (size_t)T * 2 * 64 * 4;
        e->w_off[1] = off; off += (size_t)2 * T * T * 64 * 4;
        e->w_off[2] = off; off += (size_t)2 * 2 * T * 64 * 4;
        e->b_off[0] = 0; e->b_off[1] = e->HP; e->b_off[2] = 3 * e->HP; boff = 3 * e->HP + 32 + 8 * 32;   // (same size as the split layout)
    } else {
        e->w_off[0] = off; off += (size_t)T * 2 * 64 * 4;                   // [S+A -> h]
        for (int l = 1; l < L; ++l) { e->w_off[l] = off; off += (size_t)T * T * 64 * 4; }
        e->w_off[L] = off; off += (size_t)2 * T * 64 * 4;                   // [h -> S]
        for (int l = 0; l < L; ++l) { e->b_off[l] = boff; boff += e->HP; }
        e->b_off[L] = boff; boff += 32;
    }
    e->w_floats = off;
    const size_t ln_floats = 2 * (size_t)(reward ? 3 : L) * e->HP;
    auto cleanup = [&](int code) { bcmpc_destroy(e); return code; };
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_w, e->w_floats * sizeof(float)) != hipSuccess ||
        hipMalloc(&e->d_b, boff * sizeof(float)) != hipSuccess ||
        hipMalloc(&e->d_ln, ln_floats * sizeof(float)) != hipSuccess ||
        hipMalloc(&e->d_consts, sizeof(e->h_consts)) != hipSuccess ||
        hipMalloc(&e->d_state, BCMPC_MAX_STATE * sizeof(double)) != hipSuccess ||
        hipMalloc(&e->d_costs, std::max<int64_t>(1, c.num_paths) * sizeof(double)) != hipSuccess ||
        hipMalloc(&e->d_result, sizeof(bcmpc_result)) != hipSuccess ||
        // (the split kernel's fused argmin keeps one record per workgroup)
        hipMalloc(&e->d_amin_c, (e->amin_cap = std::max<size_t>(kArgminParts, (size_t)(c.num_paths + 15) / 16)) *
                                    sizeof(double)) != hipSuccess ||
        hipMalloc(&e->d_amin_i, e->amin_cap * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&e->d_amin_ticket, sizeof(unsigned)) != hipSuccess ||
        hipMemset(e->d_amin_ticket, 0, sizeof(unsigned)) != hipSuccess ||
        hipHostMalloc(&e->h_result, sizeof(bcmpc_result), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&e->h_result_map, sizeof(bcmpc_result), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&e->d_result_map, e->h_result_map, 0) != hipSuccess ||
        hipHostMalloc(&e->h_done, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&e->d_done, e->h_done, 0) != hipSuccess) {
        g_last_error = "device allocation failed";
        return cleanup(BCMPC_ERR_HIP);
    }
    for (int i = 0; i < 3; ++i)
        if (hipEventCreate(&e->ev[i]) != hipSuccess) { g_last_error = "event create failed"; return cleanup(BCMPC_ERR_HIP); }
    if (e->kernel == BCMPC_KERNEL_TEAM) {
        const size_t tb = team_buf_bytes(c.num_paths, e->HP, e->team_kind);
        if ((tb && hipMalloc(&e->d_team, tb) != hipSuccess) ||
            (tb && hipMemset(e->d_team, 0, tb) != hipSuccess) ||
            hipMalloc(&e->d_team_ctl, 4 * sizeof(unsigned)) != hipSuccess ||
            hipMemset(e->d_team_ctl, 0, 4 * sizeof(unsigned)) != hipSuccess ||
            hipHostMalloc(&e->h_team_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void**)&e->d_team_err, e->h_team_err, 0) != hipSuccess) {
            g_last_error = "device allocation failed";
            return cleanup(BCMPC_ERR_HIP);
        }
        *e->h_team_err = 0;
    }
    if (e->PL > 0) {
        size_t poff = 0;
        e->pw_off[0] = poff; poff += (size_t)e->TP * 2 * 64 * 4;                    // [S -> ph]
        for (int l = 1; l < e->PL; ++l) { e->pw_off[l] = poff; poff += (size_t)e->TP * e->TP * 64 * 4; }
        e->pw_off[e->PL] = poff; poff += (size_t)e->TP * 64 * 4;                  // [ph -> one 16-row tile]
        e->pw_floats = poff;
        if (hipMalloc(&e->d_pw, poff * sizeof(float)) != hipSuccess ||
            hipMalloc(&e->d_pb, ((size_t)e->PL * e->PHP + kPolParams) * sizeof(float)) != hipSuccess ||
            hipMalloc(&e->d_first, std::max<int64_t>(1, c.num_paths) * c.action_dim * sizeof(double)) != hipSuccess) {
            g_last_error = "device allocation failed";
            return cleanup(BCMPC_ERR_HIP);
        }
    }
    if (reward) {
        if (hipMalloc(&e->d_gpow, (size_t)c.horizon * sizeof(double)) != hipSuccess) {
            g_last_error = "device allocation failed";
            return cleanup(BCMPC_ERR_HIP);
        }
        std::vector<double> ones((size_t)c.horizon, 1.0);
        if (hipMemcpy(e->d_gpow, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
            g_last_error = "gamma upload failed";
            return cleanup(BCMPC_ERR_HIP);
        }
    }
    // default action bounds: HalfCheetah ctrlrange [-1, 1]
    for (int j = 0; j < BCMPC_MAX_ACTION && j < kConstCols; ++j) {
        e->h_consts[6 * kConstCols + j] = -1.0;
        e->h_consts[7 * kConstCols + j] = 1.0;
    }
    *out = e;
    return BCMPC_OK;
}

int bcmpc_destroy(bcmpc_engine* e) {
    if (!e) return BCMPC_OK;
    if (e->fb) (void)bcmpc_destroy(e->fb);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->stream && e->cfg.device >= 0 && e->cfg.device < 64) {   // its team launches have completed
        TeamOrder& d = g_team_order[e->cfg.device];
        std::lock_guard<std::mutex> lk(d.mu);
        if (d.ev_stream == e->stream) {
            d.pending = false;
            d.ev_stream = nullptr;
        }
    }
    if (e->spec_st) {
        (void)hipStreamSynchronize(e->spec_st);
        (void)hipStreamDestroy(e->spec_st);
    }
    for (hipEvent_t ev : {e->spec_in_ev, e->spec_done_ev})
        if (ev) (void)hipEventDestroy(ev);
    for (void* p : {(void*)e->d_spec_xs, (void*)e->d_spec_part})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)e->d_w, (void*)e->d_b, (void*)e->d_ln, (void*)e->d_consts, (void*)e->d_state,
                    (void*)e->d_actions, (void*)e->d_costs, (void*)e->d_result, (void*)e->d_pw, (void*)e->d_pb,
                    (void*)e->d_first, (void*)e->d_gpow, (void*)e->d_mu, (void*)e->d_sigma, (void*)e->d_elite,
                    (void*)e->d_count, (void*)e->d_amin_c, (void*)e->d_amin_i,
                    (void*)e->d_amin_ticket, (void*)e->d_team, (void*)e->d_team_ctl, (void*)e->d_mt_io, (void*)e->d_mt_bounds, (void*)e->d_mt_xs,
                    (void*)e->d_mt_polys, (void*)e->d_mt_chunks, (void*)e->d_mt_part})
        if (p) (void)hipFree(p);
    if (e->h_result) (void)hipHostFree(e->h_result);
    if (e->h_result_map) (void)hipHostFree(e->h_result_map);
    if (e->h_team_err) (void)hipHostFree(e->h_team_err);
    if (e->h_done) (void)hipHostFree(e->h_done);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->pre.th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(e->pre.mu);
            e->pre.quit = true;
            e->pre.quit_a.store(true, std::memory_order_release);
        }
        e->pre.cv.notify_all();
        e->pre.th.join();
    }
    for (double* p : e->h_zc)
        if (p) (void)hipHostFree(p);
    if (e->h_rows_seq) (void)hipHostFree(e->h_rows_seq);
    if (e->copy_st) (void)hipStreamSynchronize(e->copy_st);
    for (int i = 0; i < 2; ++i) {
        if (e->d_rows[i]) (void)hipFree(e->d_rows[i]);
        if (e->copy_ev[i]) (void)hipEventDestroy(e->copy_ev[i]);
    }
    if (e->copy_st) (void)hipStreamDestroy(e->copy_st);
    if (e->h_mt_io) (void)hipHostFree(e->h_mt_io);
    for (auto& sp : e->spec) {
        if (sp.d_io) (void)hipFree(sp.d_io);
        if (sp.h_io) (void)hipHostFree(sp.h_io);
        if (sp.d_act) (void)hipFree(sp.d_act);
    }
    for (auto& ev : e->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return BCMPC_OK;
}

uint64_t bcmpc_weights_version(const bcmpc_engine* e) { return e ? e->version : 0; }

int bcmpc_predraw_stats(const bcmpc_engine* e, uint64_t* out5) {
    if (!e || !out5) return fail(BCMPC_ERR_ARG, "null argument");
    out5[0] = e->pre.hits;
    out5[1] = e->pre.late;
    out5[2] = e->pre.misses;
    out5[3] = e->spec_hits;
    out5[4] = e->spec_misses;
    return BCMPC_OK;
}

int bcmpc_set_weights(bcmpc_engine* e, const bcmpc_weights* w, uint64_t version) {
    if (!e || !w || !w->kernels || !w->biases) return fail(BCMPC_ERR_ARG, "null argument");
    if (e->has_weights && version == e->version) return BCMPC_OK;    // idempotent re-sync
    const bcmpc_config& c = e->cfg;
    const int L = c.n_layers, S = c.state_dim, A = c.action_dim, h = c.hidden, HP = e->HP, T = e->T;
    if (c.layer_norm && (!w->ln_gamma || !w->ln_beta)) return fail(BCMPC_ERR_ARG, "layer_norm enabled but LN params missing");
    if (!w->mean_obs || !w->std_obs || !w->mean_action || !w->std_action || !w->mean_deltas || !w->std_deltas)
        return fail(BCMPC_ERR_ARG, "normalization stats missing");
    const bool rw = e->reward;
    if (rw && (!w->mean_reward || !w->std_reward)) return fail(BCMPC_ERR_ARG, "reward model: mean_reward / std_reward missing");
    const int NK = rw ? 5 : L + 1, NLN = rw ? 3 : L;      // kernels, LayerNorms
    for (int l = 0; l < NK; ++l)
        if (!w->kernels[l] || !w->biases[l]) return fail(BCMPC_ERR_ARG, "null kernel/bias pointer");
    if (c.layer_norm)
        for (int l = 0; l < NLN; ++l)
            if (!w->ln_gamma[l] || !w->ln_beta[l]) return fail(BCMPC_ERR_ARG, "null LayerNorm pointer");
    HIP_TRY(hipSetDevice(c.device));
    std::vector<float> hw(e->w_floats, 0.f);
    const int tb = e->pack_tb;
    std::vector<float> hb(rw ? 3 * (size_t)HP + 32 + 8 * 32 : (size_t)L * HP + 32, 0.f);
    std::vector<float> hln(2 * (size_t)NLN * HP, 0.f);
    if (e->split && rw) {
        _Float16* hh = reinterpret_cast<_Float16*>(hw.data());
        const int P = T / 2;
        const bool ln = c.layer_norm != 0;                // (team kernel only: bcmpc_create)
        const float s0 = x3_scale(w->kernels[0], (size_t)(S + A) * h);
        pack_x3_layer(w->kernels[0], S + A, h, 1, T, tb, s0, hh + 2 * e->w_off[0]);
        e->winv[0] = 1.0f / s0;
        // the heads' input: the trunk's tanh x 2^12, or its LayerNorm output x hsc[0] (|LN(x)_i| <=
        // sqrt(h) |gamma_i| + |beta_i|, the power of two that keeps it below 2^12)
        float hin = 4096.0f;
        if (ln) {
            float gm = 0.f, bm = 0.f;
            for (int i = 0; i < h; ++i) {
                gm = std::max(gm, std::fabs(w->ln_gamma[0][i]));
                bm = std::max(bm, std::fabs(w->ln_beta[0][i]));
            }
            const float bound = std::sqrt((float)h) * gm + bm;
            int ex = 0;
            if (bound > 0.f && std::isfinite(bound)) (void)std::frexp(bound, &ex);
            hin = std::ldexp(1.0f, std::max(-100, std::min(100, 12 - ex)));
            e->hsc[0] = hin;
        }
        const float sd = x3_scale(w->kernels[1], (size_t)h * h), sr = x3_scale(w->kernels[3], (size_t)h * h);
        const int tbh = e->kernel == BCMPC_KERNEL_TEAM ? team_layer1_tiles(HP, e->team_kind) : tb;   // (team: head tiles per wave)
        pack_x3_layer(w->kernels[1], h, h, P, T, tbh, sd, hh + 2 * e->w_off[1]);
        pack_x3_layer(w->kernels[3], h, h, P, T, tbh, sr, hh + 2 * e->w_off[3]);
        e->winv[1] = (1.0f / sd) / hin;
        e->winv[3] = (1.0f / sr) / hin;
        // LayerNorm heads (rollout_team.hip HLN): out = rsqrt(var + eps) (dense_2 diag(gamma))^T (h - mean)
        // + (dense_2^T beta + b): gamma folded into the output kernels, beta into their biases
        std::vector<float> w2((size_t)h * S), w4((size_t)h);
        for (int k = 0; k < h; ++k) {
            const float gd = ln ? w->ln_gamma[1][k] : 1.0f, gr = ln ? w->ln_gamma[2][k] : 1.0f;
            for (int n = 0; n < S; ++n) w2[(size_t)k * S + n] = w->kernels[2][(size_t)k * S + n] * gd;
            w4[k] = w->kernels[4][k] * gr;
        }
        // both output kernels feed one accumulator: one scale (the smaller of the two)
        const float so = std::min(x3_scale(w2.data(), (size_t)h * S), x3_scale(w4.data(), (size_t)h));
        pack_x3_layer(w2.data(), h, S, P, 2, 2, so, hh + 2 * e->w_off[2]);
        std::vector<float> wr((size_t)h * 16, 0.f);      // dense_4 at row S of the second output tile
        for (int k = 0; k < h; ++k) wr[(size_t)k * 16 + (S - 16)] = w4[k];
        pack_x3_layer(wr.data(), h, 16, P, 1, 1, so, hh + 2 * e->w_off[4]);
        // (LN: the heads' normalised output carries no 2^12 -- rsqrt of the x 2^12 variance undoes it)
        e->winv[2] = e->winv[4] = ln ? 1.0f / so : (1.0f / so) / 4096.0f;
        std::memcpy(hb.data() + e->b_off[0], w->biases[0], sizeof(float) * h);
        std::memcpy(hb.data() + e->b_off[1], w->biases[1], sizeof(float) * h);
        std::memcpy(hb.data() + e->b_off[2], w->biases[3], sizeof(float) * h);
        std::memcpy(hb.data() + e->b_off[3], w->biases[2], sizeof(float) * S);
        hb[e->b_off[3] + S] = w->biases[4][0];
        if (ln) {
            for (int n = 0; n <= S; ++n) {                // b + kernel^T beta (f64 sum, one rounding)
                double acc = n < S ? (double)w->biases[2][n] : (double)w->biases[4][0];
                for (int k = 0; k < h; ++k)
                    acc += n < S ? (double)w->kernels[2][(size_t)k * S + n] * (double)w->ln_beta[1][k]
                                 : (double)w->kernels[4][k] * (double)w->ln_beta[2][k];
                hb[e->b_off[3] + n] = (float)acc;
            }
            // centring table: member t's rows [64 t, 64 t + 64) of the folded, scaled output kernels
            for (int t = 0; t < 8; ++t)
                for (int n = 0; n <= S; ++n) {
                    double acc = 0.0;
                    for (int k = 64 * t; k < std::min(h, 64 * t + 64); ++k)
                        acc += n < S ? (double)w2[(size_t)k * S + n] * so : (double)w4[k] * so;
                    hb[e->b_off[4] + (size_t)t * 32 + n] = (float)acc;
                }
            std::memcpy(hln.data(), w->ln_gamma[0], sizeof(float) * h);               // trunk gamma
            std::memcpy(hln.data() + (size_t)3 * HP, w->ln_beta[0], sizeof(float) * h);   // trunk beta
        }
        e->mean_reward = w->mean_reward[0];
        e->std_reward = w->std_reward[0];
    } else if (e->split) {
        // same sizes as the f32 layout (4 bytes per weight: two halves)
        _Float16* hh = reinterpret_cast<_Float16*>(hw.data());
        const int P = T / 2;
        // rollout_pp's folded operands: the hidden-producing layers as f16(W x 2 log2 e), unscaled, when that
        // stays well inside f16's range (else the scaled single-pass layout of the same kernel)
        constexpr float kTanhKh = 2.8853900817779268f;     // 2 log2(e) (split_common.h kTanhK)
        bool fold = e->pp && e->pp_fold;
        for (int l = 0; l < L && fold; ++l) {
            const int in = l == 0 ? S + A : h;
            float mx = 0.f;
            for (size_t i = 0; i < (size_t)in * h; ++i) mx = std::max(mx, std::fabs(w->kernels[l][i]));
            fold = std::isfinite(mx) && mx * kTanhKh < 16384.0f;
        }
        e->pp_fold_w = fold;
        for (int l = 0; l <= L; ++l) {
            const int in = l == 0 ? S + A : h, out = l == L ? S : h;
            const float sw = fold && l < L ? kTanhKh : x3_scale(w->kernels[l], (size_t)in * out);
            // (team kernel: layer 0 in tb = team_layer0_tiles per wave, hidden layers in team_layer1_tiles)
            const int tbh = e->kernel == BCMPC_KERNEL_TEAM ? team_layer1_tiles(HP, e->team_kind) : tb;
            if (l == 0) pack_x3_layer(w->kernels[0], in, out, 1, T, tb, sw, hh + 2 * e->w_off[0]);
            else if (l < L) pack_x3_layer(w->kernels[l], in, out, P, T, tbh, sw, hh + 2 * e->w_off[l]);
            else pack_x3_layer(w->kernels[L], in, out, P, 2, 2, sw, hh + 2 * e->w_off[L]);
            // layer 0's input scale is per candidate (kernel); hidden inputs are tanh * 2^12, an LN
            // output x hsc[l-1] (static), or relu x its column's power of two (undone in the kernel)
            float in_scale = 4096.0f;
            if (l > 0 && c.layer_norm) {
                // |LN(x)_i| <= sqrt(h) |gamma_i| + |beta_i|: the power of two that keeps it below 2^12
                float gm = 0.f, bm = 0.f;
                for (int i = 0; i < h; ++i) {
                    gm = std::max(gm, std::fabs(w->ln_gamma[l - 1][i]));
                    bm = std::max(bm, std::fabs(w->ln_beta[l - 1][i]));
                }
                const float bound = std::sqrt((float)h) * gm + bm;
                int ex = 0;
                if (bound > 0.f && std::isfinite(bound)) (void)std::frexp(bound, &ex);
                in_scale = std::ldexp(1.0f, std::max(-100, std::min(100, 12 - ex)));
                e->hsc[l - 1] = in_scale;
            } else if (l > 0 && c.activation == BCMPC_ACT_RELU) {
                in_scale = 1.0f;
            }
            if (fold) in_scale = 1.0f;                     // (folded: hidden activations are tanh in [-1, 1])
            e->winv[l] = (1.0f / sw) * (l == 0 ? 1.0f : 1.0f / in_scale);
        }
        for (int l = 0; l < L; ++l) std::memcpy(hb.data() + e->b_off[l], w->biases[l], sizeof(float) * h);
        std::memcpy(hb.data() + e->b_off[L], w->biases[L], sizeof(float) * S);
        if (c.layer_norm)
            for (int l = 0; l < L; ++l) {
                std::memcpy(hln.data() + (size_t)l * HP, w->ln_gamma[l], sizeof(float) * h);
                std::memcpy(hln.data() + (size_t)(L + l) * HP, w->ln_beta[l], sizeof(float) * h);
            }
        // the team kernel's deferred last LayerNorm (rollout_team.hip DEFER; relu + LN, T = 1): the output
        // kernel as dense_2 diag(gamma_1), scaled by its own power of two, its inputs the activations centred
        // on each wave's column mean (no hsc); bias row b + dense_2^T beta_1 (f64 sum, one rounding); in
        // gamma_1's slot the per-wave row sums c_w[n] = so sum_{k in wave w} (dense_2 diag(gamma_1))[k][n]
        e->team_defer = TEAM_DEFER && e->kernel == BCMPC_KERNEL_TEAM && e->team_kind == 0 && c.layer_norm &&
                        c.activation == BCMPC_ACT_RELU && L == 2 && team_members(HP, e->team_kind) == 1;
        if (e->team_defer) {
            const int tpw = team_layer1_tiles(HP, e->team_kind), nwv = HP / 16 / tpw;
            std::vector<float> wg((size_t)h * S);
            for (int k = 0; k < h; ++k)
                for (int n = 0; n < S; ++n) wg[(size_t)k * S + n] = w->kernels[L][(size_t)k * S + n] * w->ln_gamma[L - 1][k];
            const float so = x3_scale(wg.data(), (size_t)h * S);
            pack_x3_layer(wg.data(), h, S, P, 2, 2, so, hh + 2 * e->w_off[L]);
            e->winv[L] = 1.0f / so;
            for (int n = 0; n < S; ++n) {
                double acc = w->biases[L][n];
                for (int k = 0; k < h; ++k) acc += (double)w->kernels[L][(size_t)k * S + n] * (double)w->ln_beta[L - 1][k];
                hb[e->b_off[L] + n] = (float)acc;
            }
            std::fill(hln.begin() + HP, hln.begin() + 2 * HP, 0.f);
            for (int x = 0; x < nwv; ++x)
                for (int n = 0; n < S; ++n) {
                    double acc = 0.0;
                    for (int k = 16 * tpw * x; k < std::min(h, 16 * tpw * (x + 1)); ++k) acc += (double)wg[(size_t)k * S + n];
                    hln[(size_t)HP + x * 32 + n] = (float)(acc * so);
                }
        }
    } else {
    pack_layer(w->kernels[0], S + A, h, 2, T, tb, hw.data() + e->w_off[0]);
    if (rw) {
        // heads' hidden layers side by side: W1c[k][n] = dense_1 (n < HP) | dense_3 (n >= HP)
        std::vector<float> w1((size_t)h * 2 * HP, 0.f), wo((size_t)2 * HP * 32, 0.f);
        for (int k = 0; k < h; ++k)
            for (int n = 0; n < h; ++n) {
                w1[(size_t)k * 2 * HP + n] = w->kernels[1][(size_t)k * h + n];
                w1[(size_t)k * 2 * HP + HP + n] = w->kernels[3][(size_t)k * h + n];
            }
        // block-diagonal output: rows [0,h) x cols [0,S) = dense_2; rows [HP,HP+h) x col S = dense_4
        for (int k = 0; k < h; ++k) {
            for (int n = 0; n < S; ++n) wo[(size_t)k * 32 + n] = w->kernels[2][(size_t)k * S + n];
            wo[(size_t)(HP + k) * 32 + S] = w->kernels[4][k];
        }
        pack_layer(w1.data(), h, 2 * HP, T, 2 * T, 2 * T / e->nw, hw.data() + e->w_off[1]);
        pack_layer(wo.data(), 2 * HP, 32, 2 * T, 2, 2, hw.data() + e->w_off[2]);
        std::memcpy(hb.data(), w->biases[0], sizeof(float) * h);
        std::memcpy(hb.data() + HP, w->biases[1], sizeof(float) * h);
        std::memcpy(hb.data() + 2 * HP, w->biases[3], sizeof(float) * h);
        std::memcpy(hb.data() + 3 * HP, w->biases[2], sizeof(float) * S);
        hb[3 * HP + S] = w->biases[4][0];
        // LN: [gamma trunk HP | delta HP | reward HP][beta ...], i.e. the heads' params side by side
        if (c.layer_norm)
            for (int l = 0; l < 3; ++l) {
                std::memcpy(hln.data() + (size_t)l * HP, w->ln_gamma[l], sizeof(float) * h);
                std::memcpy(hln.data() + (size_t)(3 + l) * HP, w->ln_beta[l], sizeof(float) * h);
            }
        e->mean_reward = w->mean_reward[0];
        e->std_reward = w->std_reward[0];
    } else {
        for (int l = 1; l < L; ++l) pack_layer(w->kernels[l], h, h, T, T, tb, hw.data() + e->w_off[l]);
        pack_layer(w->kernels[L], h, S, T, 2, 2, hw.data() + e->w_off[L]);
        for (int l = 0; l < L; ++l) std::memcpy(hb.data() + e->b_off[l], w->biases[l], sizeof(float) * h);
        std::memcpy(hb.data() + e->b_off[L], w->biases[L], sizeof(float) * S);
        if (c.layer_norm)
            for (int l = 0; l < L; ++l) {
                std::memcpy(hln.data() + (size_t)l * HP, w->ln_gamma[l], sizeof(float) * h);
                std::memcpy(hln.data() + (size_t)(L + l) * HP, w->ln_beta[l], sizeof(float) * h);
            }
    }
    }
    double* C = e->h_consts;
    for (int i = 0; i < kConstCols; ++i) {
        C[0 * 32 + i] = i < S ? w->mean_obs[i] : 0.0;
        C[1 * 32 + i] = i < S ? w->std_obs[i] + 1e-10 : 1.0;       // dynamics.py:109 (std + 1e-10)
        C[2 * 32 + i] = i < A ? w->mean_action[i] : 0.0;
        C[3 * 32 + i] = i < A ? w->std_action[i] + 1e-10 : 1.0;    // dynamics.py:110
        C[4 * 32 + i] = i < S ? w->mean_deltas[i] : 0.0;
        C[5 * 32 + i] = i < S ? w->std_deltas[i] : 0.0;
        C[8 * 32 + i] = 1.0 / C[1 * 32 + i];
        C[9 * 32 + i] = 1.0 / C[3 * 32 + i];
    }
    HIP_TRY(hipMemcpyAsync(e->d_w, hw.data(), hw.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_b, hb.data(), hb.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_ln, hln.data(), hln.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_consts, C, sizeof(e->h_consts), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));   // host vectors die at scope exit
    if (e->kernel == BCMPC_KERNEL_TEAM) {
        // (the fallback engine's copy: created only if a team ever fails to meet)
        auto& hc = e->hw_copy;
        hc = bcmpc_engine::HostNet{};
        const int nin[5] = {S + A, h, h, h, h}, nout[5] = {h, h, S, h, 1};   // (reward net: dense .. dense_4)
        for (int l = 0; l < NK; ++l) {
            const int in = rw ? nin[l] : (l == 0 ? S + A : h), out = rw ? nout[l] : (l == L ? S : h);
            hc.k.emplace_back(w->kernels[l], w->kernels[l] + (size_t)in * out);
            hc.b.emplace_back(w->biases[l], w->biases[l] + out);
        }
        hc.ln = c.layer_norm != 0;
        if (hc.ln)
            for (int l = 0; l < NLN; ++l) {
                hc.g.emplace_back(w->ln_gamma[l], w->ln_gamma[l] + h);
                hc.beta.emplace_back(w->ln_beta[l], w->ln_beta[l] + h);
            }
        const double* sp[8] = {w->mean_obs, w->std_obs, w->mean_action, w->std_action, w->mean_deltas,
                               w->std_deltas, rw ? w->mean_reward : nullptr, rw ? w->std_reward : nullptr};
        const int sn[8] = {S, S, A, A, S, S, 1, 1};
        for (int i = 0; i < 8; ++i)
            if (sp[i]) hc.st[i].assign(sp[i], sp[i] + sn[i]);
    }
    e->version = version;
    e->has_weights = true;
    return BCMPC_OK;
}

int bcmpc_set_policy(bcmpc_engine* e, const bcmpc_policy* p, uint64_t version) {
    if (!e || !p || !p->kernels || !p->biases || !p->ob_mean || !p->ob_std || !p->logstd)
        return fail(BCMPC_ERR_ARG, "null argument");
    if (e->PL == 0) return fail(BCMPC_ERR_STATE, "engine was created without a policy (config.policy_hidden == 0)");
    if (e->has_policy && version == e->pol_version) { e->explore = p->explore; return BCMPC_OK; }
    const bcmpc_config& c = e->cfg;
    const int S = c.state_dim, A = c.action_dim, ph = c.policy_hidden, PL = e->PL, TP = e->TP, PHP = e->PHP;
    for (int l = 0; l <= PL; ++l)
        if (!p->kernels[l] || !p->biases[l]) return fail(BCMPC_ERR_ARG, "null policy kernel/bias pointer");
    HIP_TRY(hipSetDevice(c.device));
    std::vector<float> hw(e->pw_floats, 0.f);
    int rowmap[16];
    for (int n = 0; n < 16; ++n) {
        const int j = n - (S - 16);                     // action j sits at output-tile row S-16+j
        rowmap[n] = (j >= 0 && j < A) ? j : -1;
    }
    if (e->split) {
        // one tile per wave (TWp = 1); same byte sizes as the f32 layout.  Input scales:
        // obz (|z| <= 5) x 2^11, hidden tanh x 2^12
        _Float16* hh = reinterpret_cast<_Float16*>(hw.data());
        const int PP = PHP / 32;
        for (int l = 0; l < PL; ++l) {
            const int in = l == 0 ? S : ph;
            const float sw = x3_scale(p->kernels[l], (size_t)in * ph);
            pack_x3_layer(p->kernels[l], in, ph, l == 0 ? 1 : PP, TP, 1, sw, hh + 2 * e->pw_off[l]);
            e->pwinv[l] = (1.0f / sw) * (l == 0 ? 1.0f / 2048.0f : 1.0f / 4096.0f);
        }
        std::vector<float> wo((size_t)ph * 16, 0.f);    // output kernel with its columns at rows S-16+j
        for (int k = 0; k < ph; ++k)
            for (int n = 0; n < 16; ++n)
                if (rowmap[n] >= 0) wo[(size_t)k * 16 + n] = p->kernels[PL][(size_t)k * A + rowmap[n]];
        const float sw = x3_scale(p->kernels[PL], (size_t)ph * A);
        pack_x3_layer(wo.data(), ph, 16, PP, 1, 1, sw, hh + 2 * e->pw_off[PL]);
        e->pwinv[PL] = (1.0f / sw) * (1.0f / 4096.0f);
    } else {
        const int tb = TP / e->nw;
        pack_layer(p->kernels[0], S, ph, 2, TP, tb, hw.data() + e->pw_off[0]);
        for (int l = 1; l < PL; ++l) pack_layer(p->kernels[l], ph, ph, TP, TP, tb, hw.data() + e->pw_off[l]);
        pack_out_rows(p->kernels[PL], ph, A, TP, rowmap, hw.data() + e->pw_off[PL]);
    }
    std::vector<float> hb((size_t)PL * PHP + kPolParams, 0.f);
    for (int l = 0; l < PL; ++l) std::memcpy(hb.data() + (size_t)l * PHP, p->biases[l], sizeof(float) * ph);
    float* pm = hb.data() + (size_t)PL * PHP;           // [obmean 32][obstd 32][logstd 16][outbias 16]
    for (int d = 0; d < 32; ++d) {
        pm[d] = d < S ? p->ob_mean[d] : 0.f;
        pm[32 + d] = d < S ? p->ob_std[d] : 1.f;
    }
    for (int j = 0; j < A; ++j) {
        pm[64 + j] = p->logstd[j];
        pm[80 + (S - 16 + j)] = p->biases[PL][j];
    }
    HIP_TRY(hipMemcpyAsync(e->d_pw, hw.data(), hw.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_pb, hb.data(), hb.size() * sizeof(float), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->kernel == BCMPC_KERNEL_TEAM) {               // (the fallback engine's copy)
        auto& hc = e->hp_copy;
        hc = bcmpc_engine::HostNet{};
        for (int l = 0; l <= PL; ++l) {
            const int in = l == 0 ? S : ph, out = l == PL ? A : ph;
            hc.k.emplace_back(p->kernels[l], p->kernels[l] + (size_t)in * out);
            hc.b.emplace_back(p->biases[l], p->biases[l] + out);
        }
        hc.pvec[0].assign(p->ob_mean, p->ob_mean + S);
        hc.pvec[1].assign(p->ob_std, p->ob_std + S);
        hc.pvec[2].assign(p->logstd, p->logstd + A);
    }
    e->explore = p->explore;
    e->pol_version = version;
    e->has_policy = true;
    return BCMPC_OK;
}

int bcmpc_first_actions(bcmpc_engine* e, double* out) {
    if (!e || !out) return fail(BCMPC_ERR_ARG, "null argument");
    if (!e->d_first) return fail(BCMPC_ERR_STATE, "engine has no policy");
    HIP_TRY(hipSetDevice(e->cfg.device));
    HIP_TRY(hipMemcpy(out, e->d_first, sizeof(double) * e->cfg.num_paths * e->cfg.action_dim, hipMemcpyDeviceToHost));
    return BCMPC_OK;
}

int bcmpc_set_action_bounds(bcmpc_engine* e, const double* low, const double* high) {
    if (!e || !low || !high) return fail(BCMPC_ERR_ARG, "null argument");
    for (int j = 0; j < e->cfg.action_dim; ++j) {
        e->h_consts[6 * 32 + j] = low[j];
        e->h_consts[7 * 32 + j] = high[j];
    }
    HIP_TRY(hipSetDevice(e->cfg.device));
    HIP_TRY(hipMemcpyAsync(e->d_consts, e->h_consts, sizeof(e->h_consts), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return BCMPC_OK;
}

int bcmpc_set_discount(bcmpc_engine* e, double gamma) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    if (!e->reward) return fail(BCMPC_ERR_STATE, "discount applies to reward engines (config.model == BCMPC_MODEL_REWARD)");
    std::vector<double> g((size_t)e->cfg.horizon);
    for (int i = 0; i < e->cfg.horizon; ++i) g[i] = std::pow(gamma, (double)i);   // Python float ** int
    e->gamma = gamma;
    HIP_TRY(hipSetDevice(e->cfg.device));
    HIP_TRY(hipMemcpyAsync(e->d_gpow, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return BCMPC_OK;
}

void* bcmpc_stream(bcmpc_engine* e) { return e ? (void*)e->stream : nullptr; }

struct CemLaunch {           // one CEM iteration's sampling distribution + result merge rule
    const double* mu;
    const double* sigma;
    int32_t iter;
    int32_t merge;
    int64_t pos_base;
};

// team kernel: a team whose workgroups could not all become resident gives up after its bounded
// spin and raises the mapped flag (rollout_team.hip).  Synchronous calls check it after their
// synchronisation and rerun on the fallback engine (team_rerun); stream-ordered callers read it with
// bcmpc_engine_status once their stream is done.  Reading clears it.
static bool team_failed(bcmpc_engine* e) {
    if (e->h_team_err && __atomic_load_n(e->h_team_err, __ATOMIC_ACQUIRE) != 0) {
        __atomic_store_n(e->h_team_err, 0u, __ATOMIC_RELEASE);
        return true;
    }
    return false;
}
// a synchronous control step's failure check after its stream completed.  With a communicator
// attached, the exchange carried every rank's team status (comm.hip, wire record flags): the answer
// is the OR over the ranks, identical on every rank, so every rank reruns the step together (each on
// its fallback engine, which exchanges again) or none does
static bool step_failed(bcmpc_engine* e) {
    const bool local = team_failed(e);
    if (e->comm) return comm_any_flags(e->comm);
    return local;
}

// the stream synchronisation of a synchronous call; with a communicator attached it is bounded
// (BCMPC_COMM_TIMEOUT_MS, default 60 s): a rank that never joins the exchange aborts the
// communicator and fails the call instead of holding every other rank forever
static int sync_step(bcmpc_engine* e, hipStream_t st) {
    if (!e->comm) {
        const hipError_t se = hipStreamSynchronize(st);
        if (se != hipSuccess) return fail(BCMPC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
        return BCMPC_OK;
    }
    static const int64_t timeout_ms = [] {
        const char* v = std::getenv("BCMPC_COMM_TIMEOUT_MS");
        return v && *v ? std::max<int64_t>(1, std::atoll(v)) : int64_t(60000);
    }();
    std::string err;
    const int rc = comm_wait(e->comm, st, timeout_ms, &err);
    return rc == BCMPC_OK ? BCMPC_OK : fail(rc, err);
}

// the engine a failed synchronous step reruns on: a team engine's fallback engine.  With a communicator
// attached the failure is the OR over the ranks (step_failed), so a rank whose own kernel is not the team
// kernel also sees it: that rank reruns the same call on its own engine, which joins the collective
// rerun's exchange (it has no fallback engine and no host copies of its weights to build one from)
static int rerun_engine(bcmpc_engine* e, bcmpc_engine** r);

static int team_status(bcmpc_engine* e) {
    if (team_failed(e))
        return fail(BCMPC_ERR_HIP, "team kernel: a workgroup team did not meet (its grid was not resident -- "
                                   "another kernel holding the CUs?)");
    return BCMPC_OK;
}

// the fallback engine of a team engine, created on first need and kept in sync with the team
// engine's weights / policy / discount / action bounds (host copies)
static int team_fallback(bcmpc_engine* e, bool collective = false) {
    // (collective: every rank learned of the failure from the exchange and reruns with it; otherwise a
    //  rank with a communicator attached cannot rerun one step alone)
    if (e->comm && !collective)
        return fail(BCMPC_ERR_HIP, "team kernel: a workgroup team did not meet; with a communicator attached "
                                   "the ranks cannot rerun the step alone");
    if (!e->fb) {
        bcmpc_config c = e->cfg;
        c.kernel = BCMPC_KERNEL_AUTO;
        c.precision = BCMPC_PREC_SPLIT_F16;
        g_no_team = true;
        int rc = bcmpc_create(&c, &e->fb);
        if (rc == BCMPC_ERR_UNSUPPORTED) {               // split precision only on the team kernel: fp32
            c.precision = BCMPC_PREC_FP32;
            rc = bcmpc_create(&c, &e->fb);
        }
        g_no_team = false;
        if (rc != BCMPC_OK) return rc;
    }
    bcmpc_engine* f = e->fb;
    f->comm = collective ? e->comm : nullptr;        // (the rerun's exchange: every rank reruns)
    if (!e->fb_wset || e->fb_wver != e->version) {
        const auto& hc = e->hw_copy;
        std::vector<const float*> k, b, g, be;
        for (auto& v : hc.k) k.push_back(v.data());
        for (auto& v : hc.b) b.push_back(v.data());
        for (auto& v : hc.g) g.push_back(v.data());
        for (auto& v : hc.beta) be.push_back(v.data());
        bcmpc_weights w{};
        w.kernels = k.data(); w.biases = b.data();
        w.ln_gamma = hc.ln ? g.data() : nullptr; w.ln_beta = hc.ln ? be.data() : nullptr;
        w.mean_obs = hc.st[0].data(); w.std_obs = hc.st[1].data(); w.mean_action = hc.st[2].data();
        w.std_action = hc.st[3].data(); w.mean_deltas = hc.st[4].data(); w.std_deltas = hc.st[5].data();
        w.mean_reward = hc.st[6].empty() ? nullptr : hc.st[6].data();
        w.std_reward = hc.st[7].empty() ? nullptr : hc.st[7].data();
        if (const int rc = bcmpc_set_weights(f, &w, e->version)) return rc;
        e->fb_wver = e->version;
        e->fb_wset = true;
    }
    if (e->PL > 0) {
        if (!e->fb_pset || e->fb_pver != e->pol_version) {
            const auto& hc = e->hp_copy;
            std::vector<const float*> k, b;
            for (auto& v : hc.k) k.push_back(v.data());
            for (auto& v : hc.b) b.push_back(v.data());
            const bcmpc_policy p{k.data(), b.data(), hc.pvec[0].data(), hc.pvec[1].data(), hc.pvec[2].data(),
                                 e->explore};
            if (const int rc = bcmpc_set_policy(f, &p, e->pol_version)) return rc;
            e->fb_pver = e->pol_version;
            e->fb_pset = true;
        }
        f->explore = e->explore;
    }
    if (e->reward)
        if (const int rc = bcmpc_set_discount(f, e->gamma)) return rc;
    double lo[BCMPC_MAX_ACTION], hi[BCMPC_MAX_ACTION];
    for (int j = 0; j < e->cfg.action_dim; ++j) {
        lo[j] = e->h_consts[6 * kConstCols + j];
        hi[j] = e->h_consts[7 * kConstCols + j];
    }
    if (const int rc = bcmpc_set_action_bounds(f, lo, hi)) return rc;
    f->timing = e->timing;
    ++e->team_reruns;
    return BCMPC_OK;
}

static int rerun_engine(bcmpc_engine* e, bcmpc_engine** r) {
    if (e->comm && e->kernel != BCMPC_KERNEL_TEAM) {
        *r = e;
        return BCMPC_OK;
    }
    if (const int fr = team_fallback(e, e->comm != nullptr)) return fr;
    *r = e->fb;
    return BCMPC_OK;
}

// Team launches of one process on a device are ordered across streams: two team grids running at
// once could each hold part of the CUs the other needs.  A synchronous call's launch has completed
// when the call returns (the host waits for its argmin), so only stream-ordered launches can still
// be in flight: each records an event, and a team launch on another stream waits for it while it is
// pending.  No call on the earlier stream is made later (it may be gone by then); graph capture
// skips the ordering.

struct SyncCall {                                   // marks a synchronous entry point's launches
    bcmpc_engine* e;
    explicit SyncCall(bcmpc_engine* x) : e(x) { e->sync_call = true; }
    ~SyncCall() { e->sync_call = false; }
};

// (the same-stream shortcut only for an engine's own stream, which lives as long as the engine and is
//  cleared from the record in bcmpc_destroy: a caller's stream may be destroyed and its handle handed to a
//  new stream, whose team launch must then still wait for the old grid)
static int team_order_before(int device, hipStream_t st, hipStream_t own) {
    if (device < 0 || device >= 64) return BCMPC_OK;
    TeamOrder& d = g_team_order[device];
    std::lock_guard<std::mutex> lk(d.mu);
    if (!d.pending || (d.ev_stream == st && st == own)) return BCMPC_OK;
    const hipError_t q = hipEventQuery(d.ev);
    if (q == hipSuccess) {
        d.pending = false;
        return BCMPC_OK;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs == hipStreamCaptureStatusNone) HIP_TRY(hipStreamWaitEvent(st, d.ev, 0));
    return BCMPC_OK;
}

static int team_order_after(int device, hipStream_t st) {
    if (device < 0 || device >= 64) return BCMPC_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) return BCMPC_OK;
    TeamOrder& d = g_team_order[device];
    std::lock_guard<std::mutex> lk(d.mu);
    if (!d.ev) HIP_TRY(hipEventCreateWithFlags(&d.ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(d.ev, st));
    d.ev_stream = st;
    d.pending = true;
    return BCMPC_OK;
}

// A synchronous control step's completion: spin on the mapped word the argmin raises after its
// record (system-scope release) instead of a stream synchronisation, whose completion signal
// arrives several microseconds later; a stream synchronisation after 2 s (or BCMPC_SYNC=stream)
// reports whatever went wrong.  The stream may still run the argmin's epilogue: later work on it
// is stream-ordered.
static int wait_done(bcmpc_engine* e, unsigned long long seq) {
    static const bool stream_sync = [] {
        const char* v = std::getenv("BCMPC_SYNC");
        return v && std::strcmp(v, "stream") == 0;
    }();
    if (!stream_sync) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 1;; ++i) {
            if (__atomic_load_n(e->h_done, __ATOMIC_ACQUIRE) == seq) return BCMPC_OK;
            if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
            __builtin_ia32_pause();
        }
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    return BCMPC_OK;
}

static int rollout_impl(bcmpc_engine* e, const double* d_state, int64_t stride, const double* d_actions,
                        uint64_t seed, int64_t cand_offset, double* d_costs, double* d_traj,
                        bcmpc_result* d_result, hipStream_t st, const CemLaunch* cem = nullptr,
                        bool record_events = true, double* act_out_all = nullptr,
                        const double* state_inline = nullptr) {
    const bcmpc_config& c = e->cfg;
    if (!e->has_weights) return fail(BCMPC_ERR_STATE, "bcmpc_set_weights has not been called");
    if (c.num_paths == 0) return fail(BCMPC_ERR_EMPTY, "attempt to get argmin of an empty sequence");
    if (stride != 0 && stride != c.state_dim) return fail(BCMPC_ERR_ARG, "state_stride must be 0 or state_dim");
    if (c.cost != BCMPC_COST_NONE && !d_costs) return fail(BCMPC_ERR_ARG, "the fused objective needs a costs buffer");
    if (d_result && c.cost == BCMPC_COST_NONE) return fail(BCMPC_ERR_ARG, "argmin needs the fused cost");
    RolloutArgs a{};
    for (int l = 0; l < e->nwl; ++l) {
        const size_t end = l + 1 < e->nwl ? e->w_off[l + 1] : e->w_floats;
        a.wbytes[l] = (int32_t)((end - e->w_off[l]) * sizeof(float));
        a.w[l] = reinterpret_cast<const float __attribute__((ext_vector_type(4)))*>(e->d_w + e->w_off[l]);
    }
    for (int l = 0; l < (e->split && e->reward ? 4 : e->nwl); ++l) a.b[l] = e->d_b + e->b_off[l];
    if (e->reward) {   // trunk LN, then the two heads' LN params side by side (2*HP)
        a.lng[0] = e->d_ln;               a.lng[1] = e->d_ln + e->HP;
        a.lnb[0] = e->d_ln + 3 * e->HP;   a.lnb[1] = e->d_ln + 4 * e->HP;
        if (e->split) a.head_rs = e->d_b + e->b_off[4];
        a.model = BCMPC_MODEL_REWARD;
        a.mean_reward = e->mean_reward;
        a.std_reward = e->std_reward;
        a.gpow = e->d_gpow;
    } else {
        for (int l = 0; l < c.n_layers; ++l) {
            a.lng[l] = e->d_ln + (size_t)l * e->HP;
            a.lnb[l] = e->d_ln + (size_t)(c.n_layers + l) * e->HP;
        }
    }
    a.f16_single = e->f16 ? 1 : 0;
    a.x3_nw = e->nw;
    a.x3_pp = e->pp ? (e->pp_fold_w ? 2 : 1) : 0;
    a.consts = e->d_consts;
    a.state = d_state; a.state_stride = stride;
    if (state_inline) {                       // the tiled state by value in the kernel arguments
        a.state_inline = 1;
        for (int i = 0; i < c.state_dim; ++i) a.state_v[i] = state_inline[i];
    }
    a.actions = d_actions; a.costs = d_costs; a.traj = d_traj;
    a.seed = seed; a.cand_offset = cand_offset; a.K = c.num_paths;
    a.H = c.horizon; a.S = c.state_dim; a.A = c.action_dim; a.L = c.n_layers;
    a.hidden = c.hidden; a.act = c.activation; a.ln = c.layer_norm; a.cost = c.cost;
    if (e->PL > 0) {
        if (!e->has_policy) return fail(BCMPC_ERR_STATE, "bcmpc_set_policy has not been called");
        if (c.cost == BCMPC_COST_NONE) return fail(BCMPC_ERR_UNSUPPORTED, "policy engines need the fused cost");
        for (int l = 0; l <= e->PL; ++l) {
            const size_t end = l < e->PL ? e->pw_off[l + 1] : e->pw_floats;
            a.pwbytes[l] = (int32_t)((end - e->pw_off[l]) * sizeof(float));
            a.pw[l] = reinterpret_cast<const float __attribute__((ext_vector_type(4)))*>(e->d_pw + e->pw_off[l]);
        }
        for (int l = 0; l < e->PL; ++l) a.pb[l] = e->d_pb + (size_t)l * e->PHP;
        a.pparams = e->d_pb + (size_t)e->PL * e->PHP;
        a.pL = e->PL;
        a.phidden_padded = e->PHP;
        a.pol_mode = c.policy_mode;
        a.explore = e->explore;
        a.act_out = act_out_all ? act_out_all : e->d_first;      // [H][K][A] or step 0 only
        a.act_out_steps = act_out_all ? c.horizon : 1;
    }
    for (int l = 0; l < e->nwl; ++l) a.winv[l] = e->winv[l];
    for (int l = 0; l <= e->PL; ++l) a.pwinv[l] = e->pwinv[l];
    for (int l = 0; l < c.n_layers; ++l) a.hsc[l] = e->hsc[l];
    if (cem) {
        if (e->kernel == BCMPC_KERNEL_SOLO || e->PL > 0)
            return fail(BCMPC_ERR_UNSUPPORTED, "CEM runs on group-kernel engines without a policy");
        a.cem_mu = cem->mu;
        a.cem_sigma = cem->sigma;
        a.cem_iter = cem->iter;
    }
    ArgminArgs m{};
    if (d_result) {
        m.costs = d_costs; m.actions = d_actions; m.consts = e->d_consts; m.out = d_result;
        m.act_out = e->PL > 0 ? (act_out_all ? act_out_all : e->d_first) : nullptr;
        m.seed = seed; m.cand_offset = cand_offset; m.K = c.num_paths; m.A = c.action_dim;
        m.maximize = c.cost == BCMPC_COST_REWARD;
        m.scratch_c = e->d_amin_c;
        m.scratch_i = e->d_amin_i;
        m.nparts = argmin_parts(c.num_paths);
        if (e->want_done && !e->comm) {
            m.done = e->d_done;
            m.seq = ++e->seq;
        }
        if (cem) {
            m.cem_mu = cem->mu; m.cem_sigma = cem->sigma; m.cem_iter = cem->iter;
            m.merge = cem->merge; m.pos_base = cem->pos_base;
        }
    }
    // BCMPC_FUSED_ARGMIN=1: the split kernel reduces np.argmin in its own tail (one launch per
    // get_action).  Off by default: the tail's ticket + acquire cost ~6 us in-kernel, as much as the
    // two argmin launches it replaces, and p50 did not move (cfg1/cfg2/run.sh recipe)
    // The team kernel (small K: a few dozen workgroups) reduces it in its tail by default (round 3; one
    // launch per control step instead of two; BCMPC_TEAM_FUSED_ARGMIN=0 restores the argmin launch)
    const char* fa = std::getenv("BCMPC_FUSED_ARGMIN");
    static const bool team_fused = [] {
        const char* v = std::getenv("BCMPC_TEAM_FUSED_ARGMIN");
        return !(v && v[0] == '0');
    }();
    const bool fused = d_result && !cem &&
                       (e->kernel == BCMPC_KERNEL_TEAM ? team_fused
                                                       : e->split && fa && fa[0] == '1');
    if (fused) {
        a.fused_argmin = 1;
        a.amin = m;
        a.amin_ticket = e->d_amin_ticket;
    }
    record_events = record_events && e->timing;
    e->timed = false;
    if (record_events) HIP_TRY(hipEventRecord(e->ev[0], st));
    bool team_skipped = false;
    if (e->kernel == BCMPC_KERNEL_TEAM) {
        a.team_buf = e->d_team;
        a.team_ctl = e->d_team_ctl;
        a.team_err = e->d_team_err;
        a.rows_flag = e->rows_wait_seq ? e->d_rows_seq : nullptr;
        a.rows_seq = e->rows_wait_seq;
        e->rows_wait_seq = 0;
        // BCMPC_TEAM_SPINS (tests): exchange polls before a member gives up; -1: the launch is skipped and
        // reported as a team that gave up (forces the fallback path deterministically)
        const char* sv = std::getenv("BCMPC_TEAM_SPINS");
        if (sv && *sv) announce_test_hook("BCMPC_TEAM_SPINS", sv);
        a.team_spins = sv && *sv ? std::max(-1, std::atoi(sv)) : 0;
        if (const int rc = team_order_before(c.device, st, e->stream)) return rc;
        // diagnostics: TEAM_STAMP variant builds record per-phase cycles per wave (BCMPC_X3_STAMPS=1 prints them)
        static uint64_t* d_tst = nullptr;
        static size_t tst_n = 0;
        const bool stamps = diag_env("BCMPC_X3_STAMPS") != nullptr;
        const size_t nwv = (size_t)(e->HP / 16 / team_layer0_tiles(e->HP, e->team_kind));
        const size_t blocks = (size_t)team_blocks(c.num_paths, e->HP, e->team_kind);
        if (stamps) {
            if (tst_n < blocks * nwv * 10) {
                if (d_tst) (void)hipFree(d_tst);
                tst_n = blocks * nwv * 10;
                HIP_TRY(hipMalloc(&d_tst, tst_n * sizeof(uint64_t)));
            }
            HIP_TRY(hipMemsetAsync(d_tst, 0, tst_n * sizeof(uint64_t), st));
            a.stamps = d_tst;
        }
        if (a.team_spins < 0) {
            __atomic_store_n(e->h_team_err, 1u, __ATOMIC_RELEASE);
            team_skipped = true;                      // (no tail ran: the argmin launch raises the done word)
        } else {
            HIP_TRY(launch_rollout_team(a, e->HP, st));
        }
        if (!e->sync_call)
            if (const int rc = team_order_after(c.device, st)) return rc;
        if (stamps) {
            std::vector<uint64_t> h(blocks * nwv * 10);
            HIP_TRY(hipMemcpyAsync(h.data(), d_tst, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            const char* names[10] = {"tail", "fill", "l0in", "layer0", "slabbar", "l1mm", "l1epi", "out+bar",
                                     "xchg", "prologue"};
            if (const char* dump = diag_env("BCMPC_STAMP_DUMP")) {   // raw [blocks][waves][10] records
                if (FILE* f = std::fopen(dump, "ab")) {
                    const int32_t hdr[4] = {(int32_t)blocks, (int32_t)nwv, c.horizon, (int32_t)c.num_paths};
                    std::fwrite(hdr, sizeof(hdr), 1, f);
                    std::fwrite(h.data(), sizeof(uint64_t), h.size(), f);
                    std::fclose(f);
                }
            }
            std::fprintf(stderr, "team stamps (per step, s_memtime ticks; wave 0 | others):");
            for (int k = 0; k < 10; ++k) {
                double s0 = 0, s1 = 0;
                size_t n0 = 0, n1 = 0;
                for (size_t b = 0; b < blocks; ++b)
                    for (size_t w = 0; w < nwv; ++w) {
                        const double v = (double)h[(b * nwv + w) * 10 + k];
                        if (v == 0) continue;
                        if (w == 0) { s0 += v; ++n0; } else { s1 += v; ++n1; }
                    }
                const double div = k == 9 ? 1.0 : (double)c.horizon;
                std::fprintf(stderr, " %s=%.0f|%.0f", names[k], n0 ? s0 / n0 / div : 0.0, n1 ? s1 / n1 / div : 0.0);
            }
            std::fprintf(stderr, "\n");
        }
    } else if (e->split) {
        // diagnostics: X3_STAMP builds record per-phase cycles per wave (BCMPC_X3_STAMPS=1 prints them)
        static uint64_t* d_st = nullptr;
        static size_t st_n = 0;
        const bool stamps = diag_env("BCMPC_X3_STAMPS") != nullptr;
        const int nw = e->nw;
        const size_t blocks = (size_t)((c.num_paths + 16 * e->nc - 1) / (16 * e->nc));
        if (stamps) {
            if (st_n < blocks * nw * 10) {
                if (d_st) (void)hipFree(d_st);
                st_n = blocks * nw * 10;
                HIP_TRY(hipMalloc(&d_st, st_n * sizeof(uint64_t)));
            }
            HIP_TRY(hipMemsetAsync(d_st, 0, st_n * sizeof(uint64_t), st));
            a.stamps = d_st;
        }
        HIP_TRY(e->f16 ? launch_rollout_x3_f16(a, e->HP, e->nc, st) : launch_rollout_x3(a, e->HP, e->nc, st));
        if (stamps) {
            std::vector<uint64_t> h(blocks * nw * 10);
            HIP_TRY(hipMemcpyAsync(h.data(), d_st, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            const char* names[10] = {"owner", "input", "B1", "layer0", "slab", "mm", "epi", "out", "B3B4", "-"};
            // (waves 0..nw/2-1, the older half that wins the MFMA / VALU arbitration, vs the younger half)
            for (int grp = 0; grp < 2; ++grp) {
                std::fprintf(stderr, "x3 stamps %s:", grp == 0 ? "waves<nw/2 " : "waves>=nw/2");
                for (int k = 0; k < 9; ++k) {
                    double sum = 0; size_t n = 0;
                    for (size_t b = 0; b < blocks; ++b)
                        for (int w = 0; w < nw; ++w)
                            if ((2 * w < nw) == (grp == 0)) { sum += (double)h[(b * nw + w) * 10 + k]; ++n; }
                    std::fprintf(stderr, " %s=%.0f", names[k], n ? sum / n / c.horizon : 0.0);
                }
                std::fprintf(stderr, "  (per step, s_memtime ticks)\n");
            }
        }
    } else if (e->kernel == BCMPC_KERNEL_SOLO) {
        HIP_TRY(launch_rollout(a, e->HP, e->wpb, st));
    } else {
        HIP_TRY(launch_rollout_grp(a, e->HP, kern_waves(e->kernel), st));
    }
    if (record_events) HIP_TRY(hipEventRecord(e->ev[1], st));
    if (d_result && (!fused || team_skipped)) HIP_TRY(launch_argmin(m, st));
    if (d_result && e->comm && !cem) {
        // the one collective of a sharded control step: every rank's record, then np.argmin's rule
        std::string err;
        if (const int xr = comm_exchange(e->comm, d_result, c.cost == BCMPC_COST_REWARD, st, &err,
                                         e->kernel == BCMPC_KERNEL_TEAM ? e->d_team_err : nullptr))
            return fail(xr, err);
    }
    if (record_events) HIP_TRY(hipEventRecord(e->ev[2], st));
    e->timed = record_events && d_result != nullptr;
    return BCMPC_OK;
}

static int cem_buffers(bcmpc_engine* e, int32_t n_elite) {
    const size_t ha = (size_t)e->cfg.horizon * e->cfg.action_dim;
    if (!e->d_mu) {
        HIP_TRY(hipMalloc(&e->d_mu, ha * sizeof(double)));
        HIP_TRY(hipMalloc(&e->d_sigma, ha * sizeof(double)));
        HIP_TRY(hipMalloc(&e->d_count, sizeof(int32_t)));
    }
    if (n_elite > e->elite_cap) {
        if (e->d_elite) (void)hipFree(e->d_elite);
        e->d_elite = nullptr;
        e->elite_cap = 0;
        HIP_TRY(hipMalloc(&e->d_elite, (size_t)n_elite * sizeof(bcmpc_elite)));
        e->elite_cap = n_elite;
    }
    return BCMPC_OK;
}

static int select_impl(bcmpc_engine* e, const bcmpc_elite* d_pairs, const double* d_costs, int64_t m,
                       int64_t index_base, int32_t n_elite, bcmpc_elite* d_out, int32_t* d_count, hipStream_t st) {
    if (n_elite < 1) return fail(BCMPC_ERR_ARG, "n_elite must be >= 1");
    if (m < 0 || (!d_pairs && !d_costs) || !d_out || !d_count) return fail(BCMPC_ERR_ARG, "null argument");
    SelectArgs s{};
    s.pairs = d_pairs; s.costs = d_costs; s.m = m; s.index_base = index_base; s.n_elite = n_elite;
    s.maximize = e->cfg.cost == BCMPC_COST_REWARD;
    s.out = d_out; s.count = d_count;
    HIP_TRY(launch_select(s, st));
    return BCMPC_OK;
}

static int refit_impl(bcmpc_engine* e, const bcmpc_elite* d_elite, const int32_t* d_count, uint64_t seed,
                      int32_t iter, double alpha, double* d_mu, double* d_sigma, hipStream_t st) {
    if (!d_elite || !d_count || !d_mu || !d_sigma) return fail(BCMPC_ERR_ARG, "null argument");
    RefitArgs r{};
    r.elite = d_elite; r.count = d_count; r.mu = d_mu; r.sigma = d_sigma; r.consts = e->d_consts;
    r.seed = seed; r.iter = iter; r.H = e->cfg.horizon; r.A = e->cfg.action_dim; r.alpha = alpha;
    HIP_TRY(launch_refit(r, st));
    return BCMPC_OK;
}

int bcmpc_rollout_async(bcmpc_engine* e, const double* d_state, int64_t state_stride, const double* d_actions,
                        uint64_t seed, int64_t cand_offset, double* d_costs, double* d_traj,
                        bcmpc_result* d_result, void* stream) {
    if (!e || !d_state) return fail(BCMPC_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(e->cfg.device));
    // `stream` is used verbatim: NULL is HIP's null stream (bcmpc_stream() gives the engine's own)
    return rollout_impl(e, d_state, state_stride, d_actions, seed, cand_offset, d_costs, d_traj, d_result,
                        (hipStream_t)stream);
}

int bcmpc_rollout_policy_async(bcmpc_engine* e, const double* d_state, const double* d_actions, uint64_t seed,
                               int64_t cand_offset, double* d_costs, double* d_traj, double* d_actions_out,
                               bcmpc_result* d_result, void* stream) {
    if (!e || !d_state || !d_actions_out) return fail(BCMPC_ERR_ARG, "null argument");
    if (e->PL == 0) return fail(BCMPC_ERR_STATE, "engine was created without a policy (config.policy_hidden == 0)");
    HIP_TRY(hipSetDevice(e->cfg.device));
    return rollout_impl(e, d_state, 0, d_actions, seed, cand_offset, d_costs, d_traj, d_result, (hipStream_t)stream,
                        nullptr, true, d_actions_out);
}

int bcmpc_get_action(bcmpc_engine* e, const double* state, const double* actions, uint64_t seed,
                     int64_t cand_offset, bcmpc_result* out, double* costs_out) {
    if (!e || !state || !out) return fail(BCMPC_ERR_ARG, "null argument");
    const bcmpc_config& c = e->cfg;
    if (c.cost == BCMPC_COST_NONE) return fail(BCMPC_ERR_ARG, "get_action needs a fused objective (cheetah cost or learned reward)");
    HIP_TRY(hipSetDevice(c.device));
    const SyncCall sync_guard(e);
    // one launch chain per control step: the state travels in the kernel arguments and the argmin
    // writes the result record straight into mapped host memory (a communicator all-gathers the
    // device record instead)
    const bool lean = e->comm == nullptr;
    if (!lean) HIP_TRY(hipMemcpyAsync(e->d_state, state, sizeof(double) * c.state_dim, hipMemcpyHostToDevice, e->stream));
    const double* d_act = nullptr;
    if (actions) {
        const size_t n = (size_t)c.horizon * (size_t)c.num_paths * (size_t)c.action_dim;
        if (n > e->actions_cap) {
            if (e->d_actions) (void)hipFree(e->d_actions);
            e->d_actions = nullptr;
            e->actions_cap = 0;
            HIP_TRY(hipMalloc(&e->d_actions, n * sizeof(double)));
            e->actions_cap = n;
        }
        HIP_TRY(hipMemcpyAsync(e->d_actions, actions, n * sizeof(double), hipMemcpyHostToDevice, e->stream));
        d_act = e->d_actions;
    }
    e->want_done = lean && !costs_out;
    int rc = rollout_impl(e, lean ? nullptr : e->d_state, 0, d_act, seed, cand_offset, e->d_costs, nullptr,
                          lean ? e->d_result_map : e->d_result, e->stream, nullptr, true, nullptr,
                          lean ? state : nullptr);
    const bool spin = e->want_done;
    e->want_done = false;
    if (rc != BCMPC_OK) return rc;
    if (!lean) HIP_TRY(hipMemcpyAsync(e->h_result, e->d_result, sizeof(bcmpc_result), hipMemcpyDeviceToHost, e->stream));
    if (costs_out)
        HIP_TRY(hipMemcpyAsync(costs_out, e->d_costs, sizeof(double) * c.num_paths, hipMemcpyDeviceToHost, e->stream));
    if (spin) {
        if (const int wr = wait_done(e, e->seq)) return wr;
    } else {
        if (const int sr = sync_step(e, e->stream)) return sr;
    }
    if (step_failed(e)) {
        bcmpc_engine* re = nullptr;
        if (const int fr = rerun_engine(e, &re)) return fr;
        return bcmpc_get_action(re, state, actions, seed, cand_offset, out, costs_out);
    }
    *out = lean ? *e->h_result_map : *e->h_result;
    return BCMPC_OK;
}

// ---- NumPy-stream draw on the device -------------------------------------------------------
// Generator words per chunk (one workgroup each; BCMPC_MT_CHUNK_WORDS overrides) and coefficient
// slices per jump polynomial (BCMPC_MT_SPLITS): chunks trade jump work (one 624 x 19937 GF(2)
// correlation each, ~0.35 us of the whole chip, VALU-bound) against serial generation (~0.9 words
// per ns per workgroup).  cfg3 (15.7M words): 2^16 words -> 240 chunks x 17 slices, draw ~0.18 ms
// (tools/mt_device_sweep.py, profiles/r02_mt_device_sweep.txt).  Smaller draws want smaller chunks (the
// serial generation of one chunk is the draw's critical path once the chip has spare workgroups): ~60
// chunks per draw, as a power of two in [2^12, 2^16] words -- cfg2 (983k words) 0.366 -> 0.322 ms and a
// K = 1000 x 15 draw 0.262 -> 0.223 ms per drop-in get_action at 2^14 (profiles/r02c_mt_chunk_sweep.txt);
// round 4 (the team kernel 30% faster): the K = 1000 x 15 draw at 2^12-word chunks, back to back 0.162 ->
// 0.153 ms, with host work between calls 0.111 -> 0.105 (profiles/r04_cfg1_chunk_ab.jsonl; 2^13 0.155, 2^15 0.173).
static int64_t mt_chunk_words(int64_t shard_words) {
    const char* v = std::getenv("BCMPC_MT_CHUNK_WORDS");
    if (v && *v) return std::max<int64_t>(2, std::atoll(v)) & ~int64_t(1);
    int64_t w = int64_t(1) << 12;
    while (w < (int64_t(1) << 16) && 2 * w <= shard_words / 60) w *= 2;
    return w;
}
static int mt_splits(int cj) {
    const char* v = std::getenv("BCMPC_MT_SPLITS");
    if (v && *v) return std::max(1, std::min(64, std::atoi(v)));
    return std::max(2, std::min(32, (4096 + cj - 1) / std::max(1, cj)));
}
// NumPy-stream draws of at most this many generator words (2 A H k_global; BCMPC_MT_ZC_WORDS overrides)
// are drawn on the host straight into pinned memory that the rollout kernel reads over the bus
// (zero copy): there the device draw is a few chunks whose serial generation chains (one workgroup,
// 227 words per LDS-synchronised step) and copies cost more than the host's ~0.5 ns per word.  2^16:
// the reference's K = 400 steps (33.6k words at H = 7); a K = 1000 x 15 draw (180k) is faster on the
// device with 2^14-word chunks (0.223 vs 0.250 ms per drop-in get_action)
// ---- pre-draw worker (small NumPy-stream draws) ----
static bool mt_predraw_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("BCMPC_MT_PREDRAW");
        return !(v && v[0] == '0');
    }();
    return on;
}

static bool mt_predraw_late() {
    static const bool on = [] {
        const char* v = std::getenv("BCMPC_MT_PREDRAW_LATE");
        return !(v && v[0] == '0');
    }();
    return on;
}

static bool mt_predraw_dev() {
    static const bool on = [] {
        const char* v = std::getenv("BCMPC_MT_PREDRAW_DEV");
        return !(v && v[0] == '0');
    }();
    return on;
}

// The worker and the control thread hand jobs over by spinning first (BCMPC_MT_PREDRAW_SPIN_US, default
// 200 us) and only then blocking on the condition variable: a futex wake of either side costs several
// microseconds on a loaded host, the same order as the K = 400 draw itself
static int64_t predraw_spin_ns() {
    static const int64_t ns = [] {
        const char* v = std::getenv("BCMPC_MT_PREDRAW_SPIN_US");
        return (v && *v) ? std::max<int64_t>(0, std::atoll(v)) * 1000 : int64_t(200000);
    }();
    return ns;
}

// spin until *a == want or (b and *b), at most predraw_spin_ns()
static void spin_until(const std::atomic<bool>* a, bool want, const std::atomic<bool>* b = nullptr) {
    const int64_t lim = predraw_spin_ns();
    if (lim <= 0) return;
    const auto t0 = std::chrono::steady_clock::now();
    auto done = [&] {
        return a->load(std::memory_order_acquire) == want || (b && b->load(std::memory_order_acquire));
    };
    for (uint32_t i = 1; !done(); ++i) {
        if ((i & 255) == 0 && std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now() - t0).count() > lim)
            return;
        __builtin_ia32_pause();
    }
}

// wait until the worker is idle (its buffer complete); returns the buffer index it last filled
static int predraw_wait(bcmpc_engine* e) {
    spin_until(&e->pre.inflight, false);
    std::unique_lock<std::mutex> lk(e->pre.mu);
    e->pre.cv.wait(lk, [&] { return !e->pre.pending && !e->pre.busy; });
    return e->pre.buf;
}

// rows [H][shard] of the draw that starts at NumPy state `from`, into the buffer the last call did not read
static void predraw_post(bcmpc_engine* e, const Mt19937& from, const double* low, const double* high, int A,
                         int64_t k_global, int64_t cand_offset, bool rows) {
    auto& p = e->pre;
    {
        std::lock_guard<std::mutex> lk(p.mu);
        p.rows = rows;
        p.from = from;
        p.low.assign(low, low + A);
        p.high.assign(high, high + A);
        p.kg = k_global;
        p.off = cand_offset;
        p.buf = e->zc_last ^ 1;
        p.ready = false;
        p.pending = true;
        p.job = p.job + 1 == 0 ? 1 : p.job + 1;       // (0 is "no wait")
        p.claimed.store(false, std::memory_order_relaxed);
        p.inflight.store(true, std::memory_order_release);
    }
    if (!p.th.joinable()) {
        p.th = std::thread([e] {
            auto& q = e->pre;
            const bcmpc_config& c = e->cfg;
            std::unique_lock<std::mutex> lk(q.mu);
            for (;;) {
                if (!q.quit && !q.pending) {              // spin for the next job before sleeping
                    lk.unlock();
                    spin_until(&q.inflight, true, &q.quit_a);
                    lk.lock();
                }
                q.cv.wait(lk, [&] { return q.quit || q.pending; });
                if (q.quit) return;
                q.pending = false;
                q.busy = true;
                Mt19937 g = q.from;
                const std::vector<double> lo = q.low, hi = q.high;
                const int64_t kg = q.kg, off = q.off;
                const bool rows = q.rows;
                const uint32_t job = q.job;
                double* dst = e->h_zc[q.buf];
                lk.unlock();
                // (tests: BCMPC_MT_PREDRAW_DELAY_US holds every job back, so calls find it in flight)
                if (const char* dv = std::getenv("BCMPC_MT_PREDRAW_DELAY_US"))
                    std::this_thread::sleep_for(std::chrono::microseconds(std::atoll(dv)));
                const int64_t K = c.num_paths;
                const size_t row = (size_t)K * c.action_dim;
                if (rows && off == 0 && K == kg)          // the whole draw: one pass over [H * K] rows
                    mt_uniform_rows(g, lo.data(), hi.data(), c.action_dim, (int64_t)c.horizon * kg, 0,
                                    (int64_t)c.horizon * kg, dst);
                else if (rows)
                    for (int h = 0; h < c.horizon; ++h)
                        mt_uniform_rows(g, lo.data(), hi.data(), c.action_dim, kg, off, off + K, dst + h * row);
                else
                    g.advance(2 * (int64_t)c.action_dim * c.horizon * kg);
                if (rows && e->h_rows_seq)                // (x86 stores are ordered: the rows before the word)
                    __atomic_store_n(e->h_rows_seq, job, __ATOMIC_RELEASE);
                bool copied = false;
                const int qb = (int)(dst == e->h_zc[0] ? 0 : 1);
                // the rows into HBM while the caller's env step runs (not when a call already reads them
                // from the pinned buffer: the copy would only share the bus with that kernel)
                if (rows && e->copy_st && e->d_rows[qb] && !q.claimed.load(std::memory_order_acquire)) {
                    (void)hipSetDevice(c.device);
                    copied = hipMemcpyAsync(e->d_rows[qb], dst, (size_t)c.horizon * row * sizeof(double),
                                            hipMemcpyHostToDevice, e->copy_st) == hipSuccess &&
                             hipEventRecord(e->copy_ev[qb], e->copy_st) == hipSuccess;
                }
                lk.lock();
                e->copy_valid[qb] = copied;
                q.to = g;
                q.ready = true;
                q.busy = false;
                q.inflight.store(false, std::memory_order_release);
                q.cv.notify_all();
            }
        });
    }
    p.cv.notify_all();
}

// (2^18 with the pre-draw worker measured worse at cfg1's 180k words back to back: the kernel's own reads of
// 720 KB of rows over the bus, +30 us -- profiles/r03_dropin_zc_bound_ab.txt; draws whose rows are not read,
// the stochastic policy's, take the host path at any size: only NumPy's state advances)
// (round 4: the next call's rows are drawn from the moment this call's rollout is launched.  Taking cfg1's
//  180k-word draw on the host that way measured worse back to back than the device draw -- 0.234 vs 0.197 ms,
//  the host draw outlasts the 0.14-ms rollout it overlaps -- and equal with host work between calls:
//  profiles/r04_dropin_zc_ab.jsonl; the bound stays 2^16)
static int64_t mt_zero_copy_words(const bcmpc_engine*) {
    const char* v = std::getenv("BCMPC_MT_ZC_WORDS");
    if (v && *v) return std::max<int64_t>(0, std::atoll(v));
    return int64_t(1) << 16;
}

static bool mt_device_path() {
    const char* v = std::getenv("BCMPC_MT_PATH");
    return !(v && std::strcmp(v, "host") == 0);
}

// The draw's chunks for this engine's shard of [H, k_global, A]: the shard's rows of step h are the
// draw words [2A (h kg + off), 2A (h kg + off + K)) (one run; all steps merge into one when the shard
// is the whole draw), each run cut into pieces of <= mt_chunk_words(..) words; the chunk that draws
// the draw's last word also leaves NumPy's final state, else one extra chunk draws that word alone.
static int mt_plan(bcmpc_engine* e, int64_t kg, int64_t off) {
    if (e->mt_kg == kg && e->mt_off == off) return BCMPC_OK;
    HIP_TRY(hipStreamSynchronize(e->stream));         // (a queued speculative draw may still read the old plan)
    if (e->spec_st) HIP_TRY(hipStreamSynchronize(e->spec_st));
    if (e->d_spec_part) (void)hipFree(e->d_spec_part);
    e->d_spec_part = nullptr;
    const int64_t K = e->cfg.num_paths, A = e->cfg.action_dim, H = e->cfg.horizon;
    const int64_t N = 2 * A * H * kg;
    struct Run { int64_t s, len, out0; };
    std::vector<Run> runs;
    if (off == 0 && K == kg) runs.push_back({0, N, 0});
    else
        for (int64_t h = 0; h < H; ++h) runs.push_back({2 * A * (h * kg + off), 2 * A * K, h * K * A});
    const int64_t target = mt_chunk_words(2 * A * H * K);
    std::vector<MtChunk> ch;
    bool has_final = false;
    for (const Run& r : runs) {
        const int64_t R = r.len / 2, P = std::max<int64_t>(1, (r.len + target - 1) / target);
        for (int64_t p = 0; p < P; ++p) {
            const int64_t d0 = R * p / P, d1 = R * (p + 1) / P;
            if (d1 <= d0) continue;
            MtChunk c{};
            c.s = r.s + 2 * d0;
            c.n = 2 * (d1 - d0);
            c.out0 = r.out0 + d0;
            c.f = (int32_t)(c.s / kMtN);
            c.j0 = (int32_t)((c.s / 2) % A);
            c.final_ = c.s + c.n == N;
            has_final |= c.final_ != 0;
            ch.push_back(c);
        }
    }
    if (!has_final) {
        MtChunk c{};
        c.s = N - 2; c.n = 2; c.out0 = -1; c.f = (int32_t)((N - 2) / kMtN); c.final_ = 1;
        ch.push_back(c);
    }
    std::vector<int64_t> fs;
    for (MtChunk& c : ch) {
        c.jidx = -1;
        if (c.f >= 2) { c.jidx = (int32_t)fs.size(); fs.push_back(c.f); }
    }
    const int cj = (int)fs.size(), S = mt_splits(cj);
    std::vector<uint32_t> polys((size_t)std::max(1, cj) * kMtPolyWords, 0);
    if (cj) mt_block_polys(fs, polys.data());
    for (void* p : {(void*)e->d_mt_polys, (void*)e->d_mt_chunks, (void*)e->d_mt_part})
        if (p) (void)hipFree(p);
    e->d_mt_polys = nullptr; e->d_mt_chunks = nullptr; e->d_mt_part = nullptr;
    e->mt_kg = e->mt_off = -1;
    if (!e->d_mt_io) {
        HIP_TRY(hipMalloc(&e->d_mt_io, 1280 * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&e->d_mt_bounds, 2 * BCMPC_MAX_ACTION * sizeof(double)));
        HIP_TRY(hipMalloc(&e->d_mt_xs, (size_t)kMtStream * sizeof(uint32_t)));
        HIP_TRY(hipHostMalloc(&e->h_mt_io, 1280 * sizeof(uint32_t) + 2 * BCMPC_MAX_ACTION * sizeof(double),
                              hipHostMallocDefault));
    }
    HIP_TRY(hipMalloc(&e->d_mt_polys, polys.size() * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&e->d_mt_chunks, ch.size() * sizeof(MtChunk)));
    HIP_TRY(hipMalloc(&e->d_mt_part, (size_t)std::max(1, cj) * S * kMtN * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&e->d_spec_part, (size_t)std::max(1, cj) * S * kMtN * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(e->d_mt_polys, polys.data(), polys.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_mt_chunks, ch.data(), ch.size() * sizeof(MtChunk), hipMemcpyHostToDevice));
    e->mt_nchunks = (int32_t)ch.size();
    e->mt_cj = cj;
    e->mt_s = S;
    e->mt_kg = kg;
    e->mt_off = off;
    return BCMPC_OK;
}

static int ensure_actions(bcmpc_engine* e) {
    const size_t n = (size_t)e->cfg.horizon * (size_t)e->cfg.num_paths * (size_t)e->cfg.action_dim;
    if (n > e->actions_cap) {
        if (e->d_actions) (void)hipFree(e->d_actions);
        e->d_actions = nullptr;
        e->actions_cap = 0;
        HIP_TRY(hipMalloc(&e->d_actions, n * sizeof(double)));
        e->actions_cap = n;
    }
    return BCMPC_OK;
}

// enqueue the draw of this shard's [H, K, A] from NumPy's state (key, pos) into e->d_actions and the
// final state into d_mt_io[640..1265) (copied back by the caller after its sync)
static int mt_draw_enqueue(bcmpc_engine* e, const uint32_t* mt_key, int32_t pos, const double* low,
                           const double* high, int64_t kg, int64_t off) {
    int rc = mt_plan(e, kg, off);
    if (rc != BCMPC_OK) return rc;
    rc = ensure_actions(e);
    if (rc != BCMPC_OK) return rc;
    const int A = e->cfg.action_dim;
    std::memcpy(e->h_mt_io, mt_key, kMtN * sizeof(uint32_t));
    e->h_mt_io[kMtN] = (uint32_t)pos;
    double* hb = reinterpret_cast<double*>(e->h_mt_io + 1280);
    for (int j = 0; j < A; ++j) { hb[j] = low[j]; hb[A + j] = high[j]; }
    HIP_TRY(hipMemcpyAsync(e->d_mt_io, e->h_mt_io, (kMtN + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_mt_bounds, hb, 2 * A * sizeof(double), hipMemcpyHostToDevice, e->stream));
    MtDrawArgs a{};
    a.in = e->d_mt_io;
    a.bounds = e->d_mt_bounds;
    a.xs = e->d_mt_xs;
    a.polys = e->d_mt_polys;
    a.chunks = e->d_mt_chunks;
    a.part = e->d_mt_part;
    a.final_state = e->d_mt_io + 640;
    a.out = e->d_actions;
    a.nchunks = e->mt_nchunks; a.Cj = e->mt_cj; a.S = e->mt_s; a.A = A;
    HIP_TRY(launch_mt_draw(a, e->stream));
    HIP_TRY(hipMemcpyAsync(e->h_mt_io + 640, e->d_mt_io + 640, (kMtN + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           e->stream));
    return BCMPC_OK;
}

static bool mt_speculate() {
    static const bool on = [] {
        const char* v = std::getenv("BCMPC_MT_SPECULATE");
        return !(v && v[0] == '0');
    }();
    return on;
}
constexpr int kSpecPause = 32;

// the main stream waits for a speculative draw still running beside it (its slots, its input -- the final
// state of the draw before it -- and the MT scratch are read or rewritten by what follows)
static int spec_join(bcmpc_engine* e) {
    if (!e->spec_side_pending) return BCMPC_OK;
    HIP_TRY(hipStreamWaitEvent(e->stream, e->spec_done_ev, 0));
    e->spec_side_pending = false;
    return BCMPC_OK;
}

// enqueue the speculative draw of the next call's rows into spec slot `slot`: from the device-resident
// final state `in` of the draw just enqueued, same bounds and shard (mt_plan is the current one)
static int mt_spec_enqueue(bcmpc_engine* e, const uint32_t* in, int slot, const double* low, const double* high,
                           bool side) {
    const bcmpc_config& c = e->cfg;
    const int A = c.action_dim;
    const size_t n = (size_t)c.horizon * (size_t)c.num_paths * (size_t)A;
    if (n > e->spec_cap) {
        for (auto& sp : e->spec) {
            if (sp.d_act) (void)hipFree(sp.d_act);
            sp.d_act = nullptr;
        }
        e->spec_cap = 0;
        for (auto& sp : e->spec) HIP_TRY(hipMalloc(&sp.d_act, n * sizeof(double)));
        e->spec_cap = n;
    }
    auto& sp = e->spec[slot];
    const size_t io_bytes = 640 * sizeof(uint32_t) + 2 * BCMPC_MAX_ACTION * sizeof(double);
    if (!sp.d_io) {
        HIP_TRY(hipMalloc(&sp.d_io, io_bytes));
        HIP_TRY(hipHostMalloc(&sp.h_io, io_bytes, hipHostMallocDefault));
    }
    hipStream_t st = e->stream;
    if (side) {                                   // beside this call's rollout, after its draw
        if (!e->spec_st) {
            HIP_TRY(hipStreamCreateWithFlags(&e->spec_st, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&e->spec_in_ev, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&e->spec_done_ev, hipEventDisableTiming));
        }
        if (!e->d_spec_xs) HIP_TRY(hipMalloc(&e->d_spec_xs, (size_t)kMtStream * sizeof(uint32_t)));
        HIP_TRY(hipEventRecord(e->spec_in_ev, e->stream));
        HIP_TRY(hipStreamWaitEvent(e->spec_st, e->spec_in_ev, 0));
        st = e->spec_st;
    }
    // (the slot's staging is rewritten two calls later at the earliest: its copy has run by then)
    double* hb = reinterpret_cast<double*>(sp.h_io + 640);
    for (int j = 0; j < A; ++j) { hb[j] = low[j]; hb[A + j] = high[j]; }
    HIP_TRY(hipMemcpyAsync(sp.d_io + 640, hb, 2 * A * sizeof(double), hipMemcpyHostToDevice, st));
    MtDrawArgs a{};
    a.in = in;
    a.bounds = reinterpret_cast<const double*>(sp.d_io + 640);
    a.xs = side ? e->d_spec_xs : e->d_mt_xs;
    a.polys = e->d_mt_polys;
    a.chunks = e->d_mt_chunks;
    a.part = side ? e->d_spec_part : e->d_mt_part;
    a.final_state = sp.d_io;
    a.out = sp.d_act;
    a.nchunks = e->mt_nchunks; a.Cj = e->mt_cj; a.S = e->mt_s; a.A = A;
    HIP_TRY(launch_mt_draw(a, st));
    HIP_TRY(hipMemcpyAsync(sp.h_io, sp.d_io, (kMtN + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (side) {
        HIP_TRY(hipEventRecord(e->spec_done_ev, st));
        e->spec_side_pending = true;
    }
    return BCMPC_OK;
}

int bcmpc_get_action_mt19937(bcmpc_engine* e, const double* state, uint32_t* mt_key, int32_t* mt_pos,
                             const double* low, const double* high, int64_t k_global, int64_t cand_offset,
                             uint64_t seed, bcmpc_result* out, double* costs_out) {
    if (!e || !state || !mt_key || !mt_pos || !low || !high || !out) return fail(BCMPC_ERR_ARG, "null argument");
    const bcmpc_config& c = e->cfg;
    if (c.cost == BCMPC_COST_NONE) return fail(BCMPC_ERR_ARG, "get_action needs a fused objective (cheetah cost or learned reward)");
    if (k_global < c.num_paths || cand_offset < 0 || cand_offset + c.num_paths > k_global)
        return fail(BCMPC_ERR_ARG, "this engine's candidates must lie inside [0, k_global)");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(BCMPC_ERR_ARG, "MT19937 position out of range");
    HIP_TRY(hipSetDevice(c.device));
    const SyncCall sync_guard(e);
    const int64_t draw_words = 2 * (int64_t)c.action_dim * c.horizon * k_global;
    // MPCcontrollerPolicyNet with self_exp=True draws its exploration array (controllers.py:191) but rolls out
    // the policy's own samples (:202-203): only NumPy's state has to advance, no row is read
    const bool rows_needed = !(e->PL > 0 && c.policy_mode == BCMPC_POLICY_STOCHASTIC);
    if ((draw_words <= mt_zero_copy_words(e) || !rows_needed) && mt_device_path()) {
        // small draw: the host generates the shard's rows of every step into pinned memory (the
        // reference's own draw order), the kernel reads them in place; state in the kernel
        // arguments, result into mapped memory, one spin -- no copy either way
        const int64_t K = c.num_paths;
        const int A = c.action_dim, H = c.horizon;
        const size_t row = (size_t)K * A, n = (size_t)H * row;
        const bool predraw = mt_predraw_enabled();
        Mt19937 g;
        std::memcpy(g.key, mt_key, sizeof(g.key));
        g.pos = *mt_pos;
        auto same_job = [&] {                         // the posted job draws exactly this call's rows
            const auto& p = e->pre;
            return p.rows == rows_needed && p.kg == k_global && p.off == cand_offset && g.pos == p.from.pos &&
                   std::memcmp(g.key, p.from.key, sizeof(g.key)) == 0 &&
                   std::memcmp(low, p.low.data(), sizeof(double) * A) == 0 &&
                   std::memcmp(high, p.high.data(), sizeof(double) * A) == 0;
        };
        // late hit (team kernel): the worker is still drawing this call's rows (a caller with no host work
        // between calls) -- launch now, the kernel waits for the rows' sequence word instead of the host
        // waiting for the worker (the job's parameters are written only by this thread, in predraw_post)
        // (not with a communicator attached: a kernel that gave up waiting would have run the exchange on
        //  unpublished rows, and the ranks cannot rerun one step alone -- the host waits for the worker)
        const bool late = predraw && mt_predraw_late() && e->kernel == BCMPC_KERNEL_TEAM && e->h_rows_seq && !e->comm &&
                          n <= e->zc_cap && e->pre.inflight.load(std::memory_order_acquire) && same_job();
        if (late) e->pre.claimed.store(true, std::memory_order_release);
        // (otherwise no pre-draw is running past this point: the worker finishes its job before the buffers
        //  change)
        int b = late ? e->pre.buf : predraw_wait(e);
        if (!late && n > e->zc_cap) {
            // fine-grained host memory: no GPU cache keeps an earlier call's rows (the rows change every call)
            for (int i = 0; i < 2; ++i) {
                if (e->h_zc[i]) (void)hipHostFree(e->h_zc[i]);
                e->h_zc[i] = nullptr;
                e->d_zc[i] = nullptr;
            }
            e->zc_cap = 0;
            e->pre.ready = false;
            for (int i = 0; i < 2; ++i) {
                HIP_TRY(hipHostMalloc(&e->h_zc[i], n * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
                HIP_TRY(hipHostGetDevicePointer((void**)&e->d_zc[i], e->h_zc[i], 0));
            }
            if (mt_predraw_dev()) {
                if (!e->copy_st) {
                    HIP_TRY(hipStreamCreateWithFlags(&e->copy_st, hipStreamNonBlocking));
                    for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&e->copy_ev[i], hipEventDisableTiming));
                }
                for (int i = 0; i < 2; ++i) {
                    if (e->d_rows[i]) (void)hipFree(e->d_rows[i]);
                    e->d_rows[i] = nullptr;
                    e->copy_valid[i] = false;
                    HIP_TRY(hipMalloc(&e->d_rows[i], n * sizeof(double)));
                }
            }
            if (!e->h_rows_seq) {
                HIP_TRY(hipHostMalloc(&e->h_rows_seq, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
                HIP_TRY(hipHostGetDevicePointer((void**)&e->d_rows_seq, e->h_rows_seq, 0));
                __atomic_store_n(e->h_rows_seq, 0u, __ATOMIC_RELEASE);
            }
            e->zc_cap = n;
        }
        const bool hit = !late && predraw && e->pre.ready && same_job();
        if (!late) e->pre.ready = false;
        const double* rows_ptr = nullptr;
        if (late) {                                   // the kernel reads the pinned rows once published
            if (rows_needed) {
                rows_ptr = e->d_zc[b];
                e->rows_wait_seq = e->pre.job;
            }
            ++e->pre.hits;
            ++e->pre.late;
        } else if (hit) {                                    // NumPy's stream is exactly where the worker drew from
            b = e->pre.buf;
            g = e->pre.to;
            ++e->pre.hits;
            // (its device copy, when it has landed: the kernel then reads HBM instead of the bus)
            // (the stream wait orders and publishes the copy for the kernel; it has already completed)
            if (rows_needed && e->copy_valid[b] && hipEventQuery(e->copy_ev[b]) == hipSuccess &&
                hipStreamWaitEvent(e->stream, e->copy_ev[b], 0) == hipSuccess)
                rows_ptr = e->d_rows[b];
        } else {
            b = e->zc_last ^ 1;
            if (predraw) ++e->pre.misses;
            if (rows_needed && cand_offset == 0 && K == k_global)   // the whole draw: one pass
                mt_uniform_rows(g, low, high, A, (int64_t)H * k_global, 0, (int64_t)H * k_global, e->h_zc[b]);
            else if (rows_needed)
                for (int h = 0; h < H; ++h)
                    mt_uniform_rows(g, low, high, A, k_global, cand_offset, cand_offset + K, e->h_zc[b] + h * row);
            else
                g.advance(draw_words);
        }
        const bool lean = e->comm == nullptr;
        if (!lean)
            HIP_TRY(hipMemcpyAsync(e->d_state, state, sizeof(double) * c.state_dim, hipMemcpyHostToDevice, e->stream));
        e->want_done = lean && !costs_out;
        if (!rows_ptr && rows_needed) rows_ptr = e->d_zc[b];
        if (!late) e->copy_valid[b] = false;          // (the next fill of this buffer replaces it)
        int rc = rollout_impl(e, lean ? nullptr : e->d_state, 0, rows_ptr, seed, cand_offset,
                              e->d_costs, nullptr,
                              lean ? e->d_result_map : e->d_result, e->stream, nullptr, true, nullptr,
                              lean ? state : nullptr);
        e->rows_wait_seq = 0;
        // the next call's rows start at once, while this call's rollout runs (round 4; the worker is idle
        // here unless this call claimed its in-flight job late).  They start from NumPy's state after this
        // call's draw: a rerun on the fallback engine consumes the same draw, and a call that fails leaves
        // NumPy's state unadvanced, so the next call misses them (same_job) and draws afresh
        const bool posted_early = predraw && !late && rc == BCMPC_OK;
        if (posted_early) {
            e->zc_last = b;
            predraw_post(e, g, low, high, A, k_global, cand_offset, rows_needed);
        }
        const bool spin = e->want_done && rc == BCMPC_OK;
        e->want_done = false;
        if (rc == BCMPC_OK && !lean &&
            hipMemcpyAsync(e->h_result, e->d_result, sizeof(bcmpc_result), hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            rc = fail(BCMPC_ERR_HIP, "result copy failed");
        if (rc == BCMPC_OK && costs_out &&
            hipMemcpyAsync(costs_out, e->d_costs, sizeof(double) * c.num_paths, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            rc = fail(BCMPC_ERR_HIP, "costs copy failed");
        if (spin) {
            if (const int wr = wait_done(e, e->seq)) return wr;
        } else {
            if (e->comm && rc == BCMPC_OK) {                // (bounded: the exchange's peers)
                if (const int sr = sync_step(e, e->stream)) return sr;
            } else {
                const hipError_t se = hipStreamSynchronize(e->stream);   // (also on error: the kernel reads h_zc)
                if (rc != BCMPC_OK) return rc;
                if (se != hipSuccess) return fail(BCMPC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
            }
        }
        if (late) {                                   // (the job is finished: the kernel has read its rows)
            predraw_wait(e);
            g = e->pre.to;
            e->pre.ready = false;
        }
        if (step_failed(e)) {                         // (NumPy's state not yet advanced)
            bcmpc_engine* re = nullptr;
            if (const int fr = rerun_engine(e, &re)) return fr;
            return bcmpc_get_action_mt19937(re, state, mt_key, mt_pos, low, high, k_global, cand_offset, seed,
                                            out, costs_out);
        }
        std::memcpy(mt_key, g.key, sizeof(g.key));
        *mt_pos = g.pos;
        *out = lean ? *e->h_result_map : *e->h_result;
        e->zc_last = b;
        if (predraw && !posted_early) predraw_post(e, g, low, high, A, k_global, cand_offset, rows_needed);
        return BCMPC_OK;
    }
    if (mt_device_path()) {
        // the draw on the device: state + (key, pos) up, draw, rollout, argmin, result + final state down,
        // one synchronisation.  NumPy's state is handed back only when the whole call succeeded.
        const bool lean = e->comm == nullptr;         // (as bcmpc_get_action)
        if (!lean)
            HIP_TRY(hipMemcpyAsync(e->d_state, state, sizeof(double) * c.state_dim, hipMemcpyHostToDevice, e->stream));
        const int A = c.action_dim;
        // the previous call's speculative draw, when it starts exactly where NumPy's stream is
        const bool shit = e->spec_armed && e->spec_kg == k_global && e->spec_off == cand_offset &&
                          e->spec_pos == *mt_pos && std::memcmp(e->spec_key, mt_key, sizeof(e->spec_key)) == 0 &&
                          std::memcmp(e->spec_low, low, sizeof(double) * A) == 0 &&
                          std::memcmp(e->spec_high, high, sizeof(double) * A) == 0;
        if (e->spec_armed) {
            if (shit) {
                ++e->spec_hits;
                e->spec_miss_run = 0;
            } else {
                ++e->spec_misses;
                if (++e->spec_miss_run >= 2) {
                    e->spec_pause = kSpecPause;
                    e->spec_miss_run = 0;
                }
            }
        }
        e->spec_armed = false;
        const int cur = e->spec_slot;
        if (const int jr = spec_join(e)) return jr;
        int rc = shit ? BCMPC_OK : mt_draw_enqueue(e, mt_key, *mt_pos, low, high, k_global, cand_offset);
        // (the final-state copy was enqueued before the rollout: the argmin's done word implies it)
        const uint32_t* fin_d = shit ? e->spec[cur].d_io : e->d_mt_io + 640;
        const uint32_t* fin_h = shit ? e->spec[cur].h_io : e->h_mt_io + 640;
        e->want_done = lean && !costs_out;
        // the next call's draw: slab-kernel engines whose grid leaves CUs free (K <= 32 per CU: cfg2's 4096)
        // draw it beside this rollout (on spec_st, from this draw's final state); the others behind the argmin
        // -- a team's grid needs every CU it was given, and at cfg3 (1024 workgroups) a draw beside the
        // rollout delays it by more than it hides (profiles/r03_spec2_ab.txt)
        int nslot = -1;
        const bool speculate = rc == BCMPC_OK && e->want_done && mt_speculate();
        const bool side = e->kernel != BCMPC_KERNEL_TEAM && e->ncu > 0 && c.num_paths <= 32 * (int64_t)e->ncu;
        bool paused = false;
        if (speculate && e->spec_pause > 0) {
            --e->spec_pause;
            paused = true;
        } else if (speculate && side) {
            nslot = shit ? cur ^ 1 : 0;
            if (mt_plan(e, k_global, cand_offset) != BCMPC_OK || mt_spec_enqueue(e, fin_d, nslot, low, high, true) != BCMPC_OK)
                nslot = -1;
        }
        if (rc == BCMPC_OK)
            rc = rollout_impl(e, lean ? nullptr : e->d_state, 0, shit ? e->spec[cur].d_act : e->d_actions, seed,
                              cand_offset, e->d_costs, nullptr,
                              lean ? e->d_result_map : e->d_result, e->stream, nullptr, true, nullptr,
                              lean ? state : nullptr);
        const bool spin = e->want_done && rc == BCMPC_OK;
        e->want_done = false;
        // team engines: the next call's draw behind this call's argmin (a spinning call returns at the done
        // word, so the draw runs while the caller steps its env); not when the call synchronises the stream
        // (a hit skipped mt_plan: another shard / size drawn in between may have replaced the plan)
        if (spin && speculate && !side && !paused) {
            nslot = shit ? cur ^ 1 : 0;
            if (mt_plan(e, k_global, cand_offset) != BCMPC_OK ||
                mt_spec_enqueue(e, fin_d, nslot, low, high, false) != BCMPC_OK)
                nslot = -1;
        }
        if (!spin) nslot = -1;
        if (rc == BCMPC_OK && !lean &&
            hipMemcpyAsync(e->h_result, e->d_result, sizeof(bcmpc_result), hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            rc = fail(BCMPC_ERR_HIP, "result copy failed");
        if (rc == BCMPC_OK && costs_out &&
            hipMemcpyAsync(costs_out, e->d_costs, sizeof(double) * c.num_paths, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            rc = fail(BCMPC_ERR_HIP, "costs copy failed");
        if (spin) {
            if (const int wr = wait_done(e, e->seq)) return wr;
        } else {
            if (e->comm && rc == BCMPC_OK) {                // (bounded: the exchange's peers)
                if (const int sr = sync_step(e, e->stream)) return sr;
            } else {
                const hipError_t se = hipStreamSynchronize(e->stream);   // (also on error: nothing left in flight)
                if (rc != BCMPC_OK) return rc;
                if (se != hipSuccess) return fail(BCMPC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
            }
        }
        if (step_failed(e)) {                         // (NumPy's state not yet advanced)
            bcmpc_engine* re = nullptr;
            if (const int fr = rerun_engine(e, &re)) return fr;
            return bcmpc_get_action_mt19937(re, state, mt_key, mt_pos, low, high, k_global, cand_offset, seed,
                                            out, costs_out);
        }
        std::memcpy(mt_key, fin_h, kMtN * sizeof(uint32_t));
        *mt_pos = (int32_t)fin_h[kMtN];
        *out = lean ? *e->h_result_map : *e->h_result;
        if (nslot >= 0) {                             // armed: it starts where this call leaves NumPy
            e->spec_armed = true;
            e->spec_slot = nslot;
            std::memcpy(e->spec_key, mt_key, sizeof(e->spec_key));
            e->spec_pos = *mt_pos;
            e->spec_kg = k_global;
            e->spec_off = cand_offset;
            std::memcpy(e->spec_low, low, sizeof(double) * A);
            std::memcpy(e->spec_high, high, sizeof(double) * A);
        }
        return BCMPC_OK;
    }
    const int64_t K = c.num_paths;
    const int A = c.action_dim, H = c.horizon;
    const size_t row = (size_t)K * A, n = (size_t)H * row;
    if (n > e->actions_cap) {
        if (e->d_actions) (void)hipFree(e->d_actions);
        e->d_actions = nullptr;
        e->actions_cap = 0;
        HIP_TRY(hipMalloc(&e->d_actions, n * sizeof(double)));
        e->actions_cap = n;
    }
    if (n > e->stage_cap) {                       // pinned staging: the generator writes, the DMA reads
        if (e->h_stage) (void)hipHostFree(e->h_stage);
        e->h_stage = nullptr;
        e->stage_cap = 0;
        HIP_TRY(hipHostMalloc(&e->h_stage, n * sizeof(double), hipHostMallocDefault));
        e->stage_cap = n;
    }
    HIP_TRY(hipMemcpyAsync(e->d_state, state, sizeof(double) * c.state_dim, hipMemcpyHostToDevice, e->stream));
    Mt19937 g;
    std::memcpy(g.key, mt_key, sizeof(g.key));
    g.pos = *mt_pos;
    // Large draws: the stream split over host threads by jump-ahead (mt_jump.cpp); each thread
    // copies its own slice as soon as it is drawn.  Otherwise [H, k_global, A] in C order, one
    // step at a time, the drawn steps copied while the next ones are drawn.
    int chunk_rc = 0;
    auto copy_chunk = [&](int64_t o_lo, int64_t o_hi) -> int {
        return hipMemcpyAsync(e->d_actions + o_lo, e->h_stage + o_lo, (size_t)(o_hi - o_lo) * sizeof(double),
                              hipMemcpyHostToDevice, e->stream) == hipSuccess ? 0 : 1;
    };
    if (mt_uniform_rows_par(g, low, high, A, (int64_t)H * k_global, k_global, cand_offset, cand_offset + K,
                            e->h_stage, mt_default_threads(), mt_min_words(), copy_chunk, &chunk_rc) > 0) {
        if (chunk_rc) {
            (void)hipStreamSynchronize(e->stream);     // slices already enqueued still read the staging buffer
            return fail(BCMPC_ERR_HIP, "hipMemcpyAsync of a drawn action slice failed");
        }
    } else {
        // copies go out in pieces of >= 2 MiB (one per call for small draws: each copy costs ~5-10 us
        // of runtime overhead)
        constexpr size_t kPiece = size_t(1) << 18;   // doubles
        int h_sent = 0;
        for (int h = 0; h < H; ++h) {
            mt_uniform_rows(g, low, high, A, k_global, cand_offset, cand_offset + K, e->h_stage + h * row);
            if ((size_t)(h + 1 - h_sent) * row >= kPiece || h + 1 == H) {
                const hipError_t ce = hipMemcpyAsync(e->d_actions + h_sent * row, e->h_stage + h_sent * row,
                                                     (size_t)(h + 1 - h_sent) * row * sizeof(double),
                                                     hipMemcpyHostToDevice, e->stream);
                if (ce != hipSuccess) {
                    (void)hipStreamSynchronize(e->stream);   // (earlier pieces still read the staging buffer)
                    return fail(BCMPC_ERR_HIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(ce));
                }
                h_sent = h + 1;
            }
        }
    }
    int rc = rollout_impl(e, e->d_state, 0, e->d_actions, seed, cand_offset, e->d_costs, nullptr, e->d_result, e->stream);
    if (rc == BCMPC_OK &&
        hipMemcpyAsync(e->h_result, e->d_result, sizeof(bcmpc_result), hipMemcpyDeviceToHost, e->stream) != hipSuccess)
        rc = fail(BCMPC_ERR_HIP, "result copy failed");
    if (rc == BCMPC_OK && costs_out &&
        hipMemcpyAsync(costs_out, e->d_costs, sizeof(double) * K, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
        rc = fail(BCMPC_ERR_HIP, "costs copy failed");
    // (also on error: the staging buffer's copies are done before it can be reused)
    if (e->comm && rc == BCMPC_OK) {                // (bounded: the exchange's peers)
        if (const int sr = sync_step(e, e->stream)) return sr;
    } else {
        const hipError_t se = hipStreamSynchronize(e->stream);
        if (rc != BCMPC_OK) return rc;
        if (se != hipSuccess) return fail(BCMPC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
    }
    if (step_failed(e)) {
        bcmpc_engine* re = nullptr;
        if (const int fr = rerun_engine(e, &re)) return fr;
        return bcmpc_get_action_mt19937(re, state, mt_key, mt_pos, low, high, k_global, cand_offset, seed, out,
                                        costs_out);
    }
    std::memcpy(mt_key, g.key, sizeof(g.key));      // NumPy's state advances only when the call succeeded
    *mt_pos = g.pos;
    *out = *e->h_result;
    return BCMPC_OK;
}

int bcmpc_mt19937_uniform_device(bcmpc_engine* e, uint32_t* mt_key, int32_t* mt_pos, const double* low,
                                 const double* high, int64_t k_global, int64_t cand_offset, double* out) {
    if (!e || !mt_key || !mt_pos || !low || !high || !out) return fail(BCMPC_ERR_ARG, "null argument");
    const bcmpc_config& c = e->cfg;
    if (c.num_paths < 1 || k_global < c.num_paths || cand_offset < 0 || cand_offset + c.num_paths > k_global)
        return fail(BCMPC_ERR_ARG, "this engine's candidates must lie inside [0, k_global)");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(BCMPC_ERR_ARG, "MT19937 position out of range");
    HIP_TRY(hipSetDevice(c.device));
    if (const int jr = spec_join(e)) return jr;
    int rc = mt_draw_enqueue(e, mt_key, *mt_pos, low, high, k_global, cand_offset);
    const size_t n = (size_t)c.horizon * c.num_paths * c.action_dim;
    if (rc == BCMPC_OK &&
        hipMemcpyAsync(out, e->d_actions, n * sizeof(double), hipMemcpyDeviceToHost, e->stream) != hipSuccess)
        rc = fail(BCMPC_ERR_HIP, "action copy failed");
    if (e->comm && rc == BCMPC_OK) {                // (bounded: the exchange's peers)
        if (const int sr = sync_step(e, e->stream)) return sr;
    } else {
        const hipError_t se = hipStreamSynchronize(e->stream);
        if (rc != BCMPC_OK) return rc;
        if (se != hipSuccess) return fail(BCMPC_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
    }
    std::memcpy(mt_key, e->h_mt_io + 640, kMtN * sizeof(uint32_t));
    *mt_pos = (int32_t)e->h_mt_io[640 + kMtN];
    return BCMPC_OK;
}

int bcmpc_mt19937_uniform(uint32_t* mt_key, int32_t* mt_pos, const double* low, const double* high,
                          int32_t action_dim, int64_t n_rows, double* out) {
    if (!mt_key || !mt_pos || !low || !high || !out || action_dim < 1 || n_rows < 0)
        return fail(BCMPC_ERR_ARG, "bad argument");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(BCMPC_ERR_ARG, "MT19937 position out of range");
    Mt19937 g;
    std::memcpy(g.key, mt_key, sizeof(g.key));
    g.pos = *mt_pos;
    mt_uniform_rows(g, low, high, action_dim, n_rows, 0, n_rows, out);
    std::memcpy(mt_key, g.key, sizeof(g.key));
    *mt_pos = g.pos;
    return BCMPC_OK;
}

int bcmpc_mt19937_uniform_par(uint32_t* mt_key, int32_t* mt_pos, const double* low, const double* high,
                              int32_t action_dim, int64_t n_rows, int64_t period, int64_t keep_lo, int64_t keep_hi,
                              double* out, int32_t threads, int64_t min_words_per_thread, int32_t* used_threads) {
    if (!mt_key || !mt_pos || !low || !high || !out || action_dim < 1 || n_rows < 0 ||
        period < 1 || keep_lo < 0 || keep_hi > period || keep_lo >= keep_hi || n_rows % period)
        return fail(BCMPC_ERR_ARG, "bad argument");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(BCMPC_ERR_ARG, "MT19937 position out of range");
    Mt19937 g;
    std::memcpy(g.key, mt_key, sizeof(g.key));
    g.pos = *mt_pos;
    if (threads <= 0) threads = mt_default_threads();
    if (min_words_per_thread < 0) min_words_per_thread = mt_min_words();
    const int used = mt_uniform_rows_par(g, low, high, action_dim, n_rows, period, keep_lo, keep_hi, out, threads,
                                         min_words_per_thread, nullptr, nullptr);
    const bool par = used > 0;
    if (!par) {
        const int64_t kw = keep_hi - keep_lo;
        for (int64_t p = 0; p < n_rows / period; ++p)
            mt_uniform_rows(g, low, high, action_dim, period, keep_lo, keep_hi, out + p * kw * action_dim);
    }
    if (used_threads) *used_threads = par ? used : 1;
    std::memcpy(mt_key, g.key, sizeof(g.key));
    *mt_pos = g.pos;
    return BCMPC_OK;
}

int bcmpc_cem_get_action(bcmpc_engine* e, const double* state, const bcmpc_cem* p, uint64_t seed, double* mu,
                         double* sigma, bcmpc_result* out) {
    if (!e || !state || !p || !mu || !sigma || !out) return fail(BCMPC_ERR_ARG, "null argument");
    const bcmpc_config& c = e->cfg;
    if (c.cost == BCMPC_COST_NONE) return fail(BCMPC_ERR_ARG, "CEM needs a fused objective");
    if (p->iterations < 1 || p->iterations > (1 << 22)) return fail(BCMPC_ERR_ARG, "iterations must be in [1, 2^22]");
    if (p->n_elite < 1) return fail(BCMPC_ERR_ARG, "n_elite must be >= 1");
    if (p->k_global != 0 && p->k_global != c.num_paths)
        return fail(BCMPC_ERR_ARG, "single-device CEM: k_global must be 0 or num_paths");
    if (c.num_paths == 0) return fail(BCMPC_ERR_EMPTY, "attempt to get argmin of an empty sequence");
    HIP_TRY(hipSetDevice(c.device));
    const SyncCall sync_guard(e);
    int rc = cem_buffers(e, p->n_elite);
    if (rc != BCMPC_OK) return rc;
    const size_t ha = (size_t)c.horizon * c.action_dim;
    hipStream_t st = e->stream;
    std::vector<double> mu0, sigma0;                   // (team engines: the inputs, for a rerun)
    if (e->kernel == BCMPC_KERNEL_TEAM) {
        mu0.assign(mu, mu + ha);
        sigma0.assign(sigma, sigma + ha);
    }
    HIP_TRY(hipMemcpyAsync(e->d_state, state, sizeof(double) * c.state_dim, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d_mu, mu, ha * sizeof(double), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d_sigma, sigma, ha * sizeof(double), hipMemcpyHostToDevice, st));
    if (e->timing) HIP_TRY(hipEventRecord(e->ev[0], st));
    for (int it = 0; it < p->iterations; ++it) {
        const CemLaunch cl{e->d_mu, e->d_sigma, it, it > 0, (int64_t)it * c.num_paths};
        rc = rollout_impl(e, e->d_state, 0, nullptr, seed, 0, e->d_costs, nullptr, e->d_result, st, &cl, false);
        if (rc != BCMPC_OK) return rc;
        rc = select_impl(e, nullptr, e->d_costs, c.num_paths, 0, p->n_elite, e->d_elite, e->d_count, st);
        if (rc != BCMPC_OK) return rc;
        rc = refit_impl(e, e->d_elite, e->d_count, seed, it, p->alpha, e->d_mu, e->d_sigma, st);
        if (rc != BCMPC_OK) return rc;
    }
    if (e->timing) {
        HIP_TRY(hipEventRecord(e->ev[1], st));
        HIP_TRY(hipEventRecord(e->ev[2], st));
    }
    e->timed = e->timing;
    HIP_TRY(hipMemcpyAsync(e->h_result, e->d_result, sizeof(bcmpc_result), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(mu, e->d_mu, ha * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(sigma, e->d_sigma, ha * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (team_failed(e)) {
        if (const int fr = team_fallback(e)) return fr;
        std::memcpy(mu, mu0.data(), ha * sizeof(double));
        std::memcpy(sigma, sigma0.data(), ha * sizeof(double));
        return bcmpc_cem_get_action(e->fb, state, p, seed, mu, sigma, out);
    }
    *out = *e->h_result;
    return BCMPC_OK;
}

int bcmpc_cem_rollout_async(bcmpc_engine* e, const double* d_state, const double* d_mu, const double* d_sigma,
                            uint64_t seed, int32_t iteration, int64_t cand_offset, int64_t k_global,
                            double* d_costs, bcmpc_result* d_result, int32_t merge, void* stream) {
    if (!e || !d_state || !d_mu || !d_sigma || !d_costs) return fail(BCMPC_ERR_ARG, "null argument");
    if (iteration < 0 || iteration >= (1 << 22)) return fail(BCMPC_ERR_ARG, "iteration must be in [0, 2^22)");
    if (k_global < e->cfg.num_paths + cand_offset) return fail(BCMPC_ERR_ARG, "k_global smaller than this shard's range");
    HIP_TRY(hipSetDevice(e->cfg.device));
    const CemLaunch cl{d_mu, d_sigma, iteration, merge != 0, (int64_t)iteration * k_global + cand_offset};
    return rollout_impl(e, d_state, 0, nullptr, seed, cand_offset, d_costs, nullptr, d_result, (hipStream_t)stream,
                        &cl);
}

int bcmpc_select_async(bcmpc_engine* e, const bcmpc_elite* d_pairs, const double* d_costs, int64_t m,
                       int64_t index_base, int32_t n_elite, bcmpc_elite* d_out, int32_t* d_count, void* stream) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(e->cfg.device));
    return select_impl(e, d_pairs, d_costs, m, index_base, n_elite, d_out, d_count, (hipStream_t)stream);
}

int bcmpc_cem_refit_async(bcmpc_engine* e, const bcmpc_elite* d_elite, const int32_t* d_count, uint64_t seed,
                          int32_t iteration, double alpha, double* d_mu, double* d_sigma, void* stream) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(e->cfg.device));
    return refit_impl(e, d_elite, d_count, seed, iteration, alpha, d_mu, d_sigma, (hipStream_t)stream);
}

int bcmpc_engine_set_comm(bcmpc_engine* e, bcmpc_comm* comm) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    if (comm && comm_device(comm) != e->cfg.device)
        return fail(BCMPC_ERR_ARG, "the communicator was created for another device");
    if (comm && e->cfg.cost == BCMPC_COST_NONE)
        return fail(BCMPC_ERR_ARG, "the exchange needs the fused objective (argmin records)");
    e->comm = comm;
    return BCMPC_OK;
}

int bcmpc_engine_status(bcmpc_engine* e) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    return team_status(e);
}

int bcmpc_engine_team_reruns(const bcmpc_engine* e, uint64_t* reruns) {
    if (!e || !reruns) return fail(BCMPC_ERR_ARG, "null argument");
    *reruns = e->team_reruns;
    return BCMPC_OK;
}

int bcmpc_engine_set_timing(bcmpc_engine* e, int32_t on) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    e->timing = on != 0;
    return BCMPC_OK;
}

int bcmpc_last_kernel_ms(bcmpc_engine* e, float* rollout_ms, float* argmin_ms) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    if (!e->timed) return fail(BCMPC_ERR_ARG, "the last launch was not timed (bcmpc_engine_set_timing(eng, 1) first)");
    float r = 0.f, m = 0.f;
    HIP_TRY(hipEventSynchronize(e->ev[2]));
    HIP_TRY(hipEventElapsedTime(&r, e->ev[0], e->ev[1]));
    HIP_TRY(hipEventElapsedTime(&m, e->ev[1], e->ev[2]));
    if (rollout_ms) *rollout_ms = r;
    if (argmin_ms) *argmin_ms = m;
    return BCMPC_OK;
}

int bcmpc_engine_layout(const bcmpc_engine* e, char* buf, int32_t cap) {
    if (!e || !buf || cap <= 0) return fail(BCMPC_ERR_ARG, "null argument");
    const char* prec = e->f16 ? "f16" : e->split ? "split" : "fp32";
    char s[160];
    switch (e->kernel) {
        case BCMPC_KERNEL_SOLO: std::snprintf(s, sizeof(s), "rollout_fp32<%d> fp32", e->HP); break;
        case BCMPC_KERNEL_GROUP4:
        case BCMPC_KERNEL_GROUP8: std::snprintf(s, sizeof(s), "rollout_grp<%d,NW=%d> fp32", e->HP, e->nw); break;
        case BCMPC_KERNEL_TEAM:
            std::snprintf(s, sizeof(s), "rollout_team<%d,kind=%d%s> split", e->HP, e->team_kind,
                          e->team_defer ? ",deferLN" : "");
            break;
            break;
        default:
            if (e->pp)
                std::snprintf(s, sizeof(s), "rollout_pp<%d%s> %s", e->HP, e->pp_fold_w ? ",fold" : "", prec);
            else
                std::snprintf(s, sizeof(s), "rollout_x3<%d,NC=%d,NW=%d> %s", e->HP, e->nc, e->nw, prec);
    }
    std::snprintf(buf, (size_t)cap, "%s", s);
    return BCMPC_OK;
}

int bcmpc_engine_info(const bcmpc_engine* e, int32_t* hidden_padded, int64_t* packed_weight_bytes,
                      int32_t* waves_per_block, int32_t* kernel) {
    if (!e) return fail(BCMPC_ERR_ARG, "null argument");
    if (hidden_padded) *hidden_padded = e->HP;
    if (packed_weight_bytes) *packed_weight_bytes = (int64_t)(e->w_floats * sizeof(float));
    if (waves_per_block) *waves_per_block = e->kernel == BCMPC_KERNEL_SOLO ? e->wpb : e->nw;
    if (kernel) *kernel = e->kernel;
    return BCMPC_OK;
}

}  // extern "C"
