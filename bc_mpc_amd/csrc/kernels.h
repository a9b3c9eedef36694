// kernels.h -- device-side argument blocks and launchers (internal to libbcmpc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/bcmpc.h"

namespace bcmpc {

// consts block: [10][32] doubles
//   0 mean_obs   1 std_obs + 1e-10   2 mean_action   3 std_action + 1e-10
//   4 mean_deltas  5 std_deltas      6 action low    7 action high
//   8 1 / (std_obs + 1e-10)   9 1 / (std_action + 1e-10)   (correctly rounded, for div_rn)
constexpr int kConstRows = 10;
constexpr int kConstCols = 32;

struct ArgminArgs {
    const double* costs;
    const double* act_out;   // [.][K][A] actions written by the rollout (policy mode) or nullptr
    const double* actions;   // [H][K][A] or nullptr
    const double* consts;
    bcmpc_result* out;
    uint64_t seed;
    int64_t cand_offset;
    int64_t K;
    int32_t A;
    int32_t maximize;        // np.argmax (learned reward, controllers.py:152) instead of np.argmin
    // CEM: first action regenerated from the sampler; merge with the running best by stream position
    const double* cem_mu;
    const double* cem_sigma;
    int32_t cem_iter;
    int32_t merge;           // keep out's previous best unless strictly better (np.argmin over iterations)
    int64_t pos_base;        // position of candidate 0 in the concatenated stream (iter * K_global + offset)
    double* scratch_c;       // [kArgminParts] per-block best (argmin_partial -> argmin_final)
    int64_t* scratch_i;
    int32_t nparts;          // argmin_parts(K)
    // synchronous control steps: after the record, a system-scope release of seq into this mapped
    // host word (the host spins on it instead of a stream synchronisation), or nullptr
    unsigned long long* done;
    unsigned long long seq;
};
struct RolloutArgs {
    const float __attribute__((ext_vector_type(4)))* w[BCMPC_MAX_LAYERS + 1];  // packed kernels
    int32_t wbytes[BCMPC_MAX_LAYERS + 1];    // packed bytes per layer (buffer num_records)
    const float* b[BCMPC_MAX_LAYERS + 1];    // padded biases
    const float* lng[BCMPC_MAX_LAYERS];      // padded LN gamma (0 on pad lanes)
    const float* lnb[BCMPC_MAX_LAYERS];      // padded LN beta
    const double* consts;
    const double* state;
    int64_t state_stride;                    // 0 (tiled, controllers.py:63) or S (per-candidate)
    int32_t state_inline;                    // 1: the (tiled) state is state_v, carried in the kernel
    double state_v[BCMPC_MAX_STATE];         //    arguments (no host-to-device copy per control step)
    const double* actions;                   // [H][K][A] or nullptr => Philox
    double* costs;                           // [K] or nullptr
    double* traj;                            // [H+1][K][S] or nullptr
    uint64_t seed;
    int64_t cand_offset;
    int64_t K;
    int32_t H, S, A, L, hidden, act, ln, cost;
    // fused policy (MPCcontrollerPolicyNet, controllers.py:189-237); pL == 0: none
    const float __attribute__((ext_vector_type(4)))* pw[BCMPC_MAX_LAYERS + 1];
    int32_t pwbytes[BCMPC_MAX_LAYERS + 1];
    const float* pb[BCMPC_MAX_LAYERS];       // padded hidden biases
    const float* pparams;                    // kPolParams floats: obmean[32] obstd[32] logstd[16] outbias[16]
    int32_t pL, phidden_padded, pol_mode;
    double explore;
    double* act_out;                         // [act_out_steps][K][A] f64 actions actually rolled out, or nullptr
    int32_t act_out_steps;
    // learned-reward net (NNDynamicsRewardModel, dynamics.py:121-238); model == BCMPC_MODEL_REWARD
    int32_t model;
    double mean_reward, std_reward;          // dynamics.py:236 denomalize
    const double* gpow;                      // [H] gamma**h (controllers.py:139)
    // CEM sampling (DESIGN.md "CEM"): actions = clip(mu + sigma * IrwinHall12(seed, g, h, j, iter))
    const double* cem_mu;                    // [H][A] or nullptr
    const double* cem_sigma;                 // [H][A]
    int32_t cem_iter;
    // split kernel (BCMPC_PREC_SPLIT_F16): 1 / (operand scales) of layer l's MFMA result,
    // exact powers of two (layer 0: weight scale only; its input scale is per candidate)
    float winv[BCMPC_MAX_LAYERS + 1];
    float pwinv[BCMPC_MAX_LAYERS + 1];       // the same for the fused policy's layers
    float hsc[BCMPC_MAX_LAYERS];             // split LN nets: power-of-two scale of hidden layer l's output
    int32_t f16_single;                      // BCMPC_PREC_F16: one f16 MFMA pass (hi x hi), no lo operands
    int32_t x3_nw;                           // split kernel: waves per workgroup (0: x3_waves' default)
    int32_t x3_pp;                           // single-pass f16: the two-group pipelined kernel (rollout_pp)
    uint64_t* stamps;                        // diagnostics (X3_STAMP builds): [blocks][NW][10] phase cycles
    // split kernel: np.argmin fused into the launch's tail (fused_argmin != 0): every workgroup
    // leaves its best (cost, index) in amin.scratch_c/i[blockIdx.x], the last to finish (ticket)
    // reduces them and writes amin.out like argmin_final
    int32_t fused_argmin;
    unsigned* amin_ticket;
    ArgminArgs amin;
    // team kernel (rollout_team.hip, T > 1 members per column): exchange granules
    // [columns + 8][2][T][8][64], launch control {ticket, generation}, timeout flag (mapped host word)
    unsigned long long* team_buf;
    unsigned* team_ctl;
    unsigned* team_err;
    int32_t team_spins;                      // exchange polls before a member gives up (0: the default, ~1 s)
    // (team kernel, the drop-in's late pre-draw hit) the actions are host rows that the pre-draw worker is
    // still writing: every workgroup waits until this mapped host word equals rows_seq before its first
    // read of them (nullptr: the rows are complete at launch)
    const uint32_t* rows_flag;
    uint32_t rows_seq;
    // (team kernel, the reward net with LayerNorm heads) [8 members][32 rows]: sum over member t's head
    // rows of the gamma-folded, scaled output weights (the centring correction, rollout_team.hip)
    const float* head_rs;
};

struct SelectArgs {                          // top-E of (cost, index) pairs, NaN last, ties -> lower index
    const bcmpc_elite* pairs;                // [m] pairs (index < 0: empty), or nullptr =>
    const double* costs;                     // [m] costs with index = index_base + i
    int64_t m, index_base;
    int32_t n_elite;
    int32_t maximize;                        // learned reward: the n_elite LARGEST
    bcmpc_elite* out;                        // [n_elite], ascending index, padded with index -1
    int32_t* count;                          // number selected
};

struct RefitArgs {                           // per-(h, j) elite mean / std, smoothed in place
    const bcmpc_elite* elite;
    const int32_t* count;
    double* mu;                              // [H][A]
    double* sigma;
    const double* consts;                    // action bounds (rows 6, 7)
    uint64_t seed;
    int32_t iter, H, A;
    double alpha;
};
// ---- NumPy's legacy MT19937 stream drawn on the device (mt_device.hip) ----
// One chunk = a contiguous range of the draw's generator words [s, s + n) (both even: whole
// random_sample doubles), drawn by one workgroup starting from the 624-word window of stream block
// f = floor(s / 624) (block 0 = the caller's key; block 1 = twist(key); block f >= 2 = jump
// polynomial jidx applied to block 1), then written as uniforms to out[out0 ..).  final != 0: the
// chunk ends the draw and leaves NumPy's (key, pos) in MtDrawArgs::final_state.
struct MtChunk {
    int64_t s;        // first draw word (relative to the caller's pos)
    int64_t n;        // words (even)
    int64_t out0;     // output double index of the first double, < 0: not stored
    int32_t f;        // start block
    int32_t jidx;     // jump polynomial (f >= 2), else -1
    int32_t final_;   // 1: write final_state after the last word
    int32_t j0;       // (s / 2) % A: action column of the first double
};
constexpr int kMtN = 624;
constexpr int kMtPolyWords = 624;                // 19937 coefficient bits, padded to 624 u32
constexpr int kMtStream = 32 * kMtPolyWords + 768; // words of the block-1 stream the jumps correlate with
struct MtDrawArgs {
    const uint32_t* in;        // [624] key, [624] = pos (NumPy's get_state()[1], [2])
    const double* bounds;      // [2][A]: low, high (np.random.uniform's low / high as f64)
    uint32_t* xs;              // [kMtStream] scratch: x[0..) = block 1 onwards
    const uint32_t* polys;     // [Cj][kMtPolyWords] x^(624 (f - 1)) mod phi, bit i = coefficient of x^i
    const MtChunk* chunks;     // [nchunks]
    uint32_t* part;            // [Cj][S][624] scratch: partial jumped windows (XOR-combined)
    uint32_t* final_state;     // [625] NumPy's key + pos after the whole draw
    double* out;               // the shard's [H][K][A] action array
    int32_t nchunks, Cj, S, A;
};
hipError_t launch_mt_draw(const MtDrawArgs& a, hipStream_t st);

// ---- library-owned min-loc exchange (comm.hip) ----
int set_error(int code, const std::string& msg);          // bcmpc_last_error() text (capi.cpp)
void announce_test_hook(const char* name, const char* value);   // stderr, once per hook per process (capi.cpp)
int comm_exchange(bcmpc_comm* c, bcmpc_result* d_result, int maximize, hipStream_t st, std::string* err,
                  const unsigned* d_team_err);
bool comm_any_flags(bcmpc_comm* c);
int comm_wait(bcmpc_comm* c, hipStream_t st, int64_t timeout_ms, std::string* err);
int comm_rank(const bcmpc_comm* c);
int comm_size(const bcmpc_comm* c);
int comm_device(const bcmpc_comm* c);

constexpr int kPolParams = 96;

constexpr int kArgminParts = 256;
int argmin_parts(int64_t K);

int max_waves_per_block(int hidden_padded, int n_layers);
hipError_t launch_rollout(const RolloutArgs& a, int hidden_padded, int waves_per_block, hipStream_t st);
size_t grp_lds_bytes(int hidden_padded, int n_layers, int nw, int policy_hidden_padded, int policy_layers, int model);
hipError_t launch_rollout_grp(const RolloutArgs& a, int hidden_padded, int nw, hipStream_t st);
int x3_waves(int hidden_padded);
int x3_max_nc(int hidden_padded);
size_t x3_lds(int hidden_padded, int n_layers, int nc, int action_dim, int policy_layers, int policy_hidden_padded,
              int ak = 0);
bool x3_policy_ok(int hidden_padded, int nc);
// single-pass f16 layouts (BCMPC_PREC_F16): the (nc, nw) pairs this build instantiates, and their LDS
bool x3_f16_layout_ok(int hidden_padded, int nc, int nw);
size_t x3_f16_lds(int hidden_padded, int n_layers, int nc, int nw, int action_dim);
bool x3_pp_ok(int hidden_padded, int n_layers, int state_dim, int action_dim);   // rollout_pp's shapes
hipError_t launch_rollout_x3(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st);
hipError_t launch_rollout_x3_f16(const RolloutArgs& a, int hidden_padded, int nc, hipStream_t st);
// rollout_team.hip; kind: 0 the plain delta net, 1 + fused policy, 2 the reward net (+ policy)
int team_members(int hidden_padded, int kind);          // workgroups per candidate column (0: unsupported)
// the team kernel's deferred last LayerNorm (relu + LN delta net at T = 1; rollout_team.hip DEFER): the host
// packs the output layer for it whenever the kernel takes it -- one switch for both sides
#ifndef TEAM_DEFER
#define TEAM_DEFER 1
#endif
int team_layer0_tiles(int hidden_padded, int kind);     // layer-0 tiles per wave (weight packing)
int team_layer1_tiles(int hidden_padded, int kind);     // hidden-layer (head) tiles per wave
int64_t team_blocks(int64_t K, int hidden_padded, int kind);
size_t team_buf_bytes(int64_t K, int hidden_padded, int kind);
bool team_rw_ln_built();                                // the reward net's LayerNorm heads are in this build
hipError_t launch_rollout_team(const RolloutArgs& a, int hidden_padded, hipStream_t st);
hipError_t launch_argmin(const ArgminArgs& a, hipStream_t st);
hipError_t launch_select(const SelectArgs& a, hipStream_t st);
hipError_t launch_refit(const RefitArgs& a, hipStream_t st);

}  // namespace bcmpc
