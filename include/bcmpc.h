/*
 * bcmpc.h -- C ABI of the MI355X random-shooting MPC rollout engine.
 *
 * This is the drop-in boundary for the reference's hot path
 *   controllers.MPCcontroller.get_action            (controllers.py:57-88)
 *     -> H x dynamics.NNDynamicsModel.predict       (dynamics.py:106-119, MLP dynamics.py:54-71)
 *     -> cost_functions.trajectory_cost_fn(cheetah) (cost_functions.py:9-30, :59-63)
 *     -> np.argmin + first action                   (controllers.py:82-85)
 * and its siblings on the same engine:
 *   MPCcontrollerPolicyNet.get_action      (controllers.py:160-237; policy fused, bcmpc_set_policy)
 *   MPCcontrollerReward.get_action         (controllers.py:90-158; NNDynamicsRewardModel,
 *                                           dynamics.py:121-238; argmax of the discounted reward)
 *   MPCcontrollerPolicyNetReward.get_action (controllers.py:289-363)
 * The reference binds that path in-process from Python; the host mirror
 * (bc_mpc_amd/controllers.py) binds these symbols through ctypes.
 *
 * Plain C: pointers + sizes, no torch/HIP types in the signatures (streams
 * are passed as void*).  Every entry point returns a bcmpc_status; on error
 * bcmpc_last_error() returns a thread-local message.  One engine per device
 * per host thread; an engine is not re-entrant.
 */
#ifndef BCMPC_H_
#define BCMPC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCMPC_ABI_VERSION 4
#define BCMPC_MAX_LAYERS 8      /* hidden layers supported (dynamics.py:66 n_layers) */
#define BCMPC_MAX_STATE 32      /* S: observation dim (HalfCheetah: 20, cheetah_env.py:21-27) */
#define BCMPC_MAX_INPUT 32      /* S + A (dynamics.py:26 concat) */
#define BCMPC_MAX_ACTION 16

typedef enum bcmpc_status {
    BCMPC_OK = 0,
    BCMPC_ERR_ARG = 1,          /* bad argument (Python: ValueError)          */
    BCMPC_ERR_UNSUPPORTED = 2,  /* shape/mode this build does not implement    */
    BCMPC_ERR_HIP = 3,          /* HIP runtime failure (Python: RuntimeError)  */
    BCMPC_ERR_STATE = 4,        /* e.g. rollout before set_weights             */
    BCMPC_ERR_EMPTY = 5         /* K == 0: np.argmin of an empty sequence      */
} bcmpc_status;

typedef enum bcmpc_activation {  /* dynamics.py:60 activation / train_mpc_ppo.py:539 */
    BCMPC_ACT_TANH = 0,
    BCMPC_ACT_RELU = 1
} bcmpc_activation;

typedef enum bcmpc_cost {
    BCMPC_COST_CHEETAH = 0,     /* fused cheetah_cost_fn (cost_functions.py:10-30), argmin  */
    BCMPC_COST_NONE = 1,        /* no fused cost: caller scores the trajectory              */
    BCMPC_COST_REWARD = 2       /* learned reward: sum_h reward_h * gamma**h, ARGMAX
                                   (controllers.py:139,150-152); needs BCMPC_MODEL_REWARD  */
} bcmpc_cost;

typedef enum bcmpc_model {      /* which dynamics net (dynamics.py)                          */
    BCMPC_MODEL_DELTA = 0,      /* NNDynamicsModel: L x dense(h) -> dense(S) (:54-71)        */
    BCMPC_MODEL_REWARD = 1      /* NNDynamicsRewardModel: tanh trunk dense(h) -> {delta head
                                   dense(h) -> dense(S), reward head dense(h) -> dense(1)},
                                   LayerNorm per head (:150-177); n_layers must be 2         */
} bcmpc_model;

typedef enum bcmpc_precision {
    BCMPC_PREC_FP32 = 0,        /* f32 MLP on v_mfma_f32_16x16x4_f32 (exact f32 fma chain) */
    BCMPC_PREC_SPLIT_F16 = 1,   /* f32-accurate MLP on the f16 matrix cores: every operand as
                                   hi + lo f16 halves (22 bits), three v_mfma_f32_16x16x32_f16
                                   passes hi*hi + hi*lo + lo*hi, f32 accumulate (DESIGN.md
                                   "split kernel"); tanh, no LayerNorm, NNDynamicsModel only */
    BCMPC_PREC_F16 = 2          /* BASELINE cfg3's "bf16 MFMA GEMM + fp32 cost": one f16 pass
                                   (11-bit operands, f32 accumulate, f64 state / cost) on the
                                   split slab kernels; the tanh NNDynamicsModel only.  NOT the
                                   fp32 tolerance: DESIGN.md "single-pass f16"               */
} bcmpc_precision;

typedef enum bcmpc_kernel {     /* rollout kernel layout (DESIGN.md "kernels")              */
    BCMPC_KERNEL_AUTO = 0,
    BCMPC_KERNEL_SOLO = 1,      /* one wave owns 16 candidates, activations in VGPRs     */
    BCMPC_KERNEL_GROUP2 = 2,    /* retired in round 6 (A/B only, never chosen by auto):
                                   bcmpc_create returns BCMPC_ERR_UNSUPPORTED             */
    BCMPC_KERNEL_GROUP4 = 3,    /* 4 waves share 16 candidates                           */
    BCMPC_KERNEL_GROUP8 = 4,    /* 8 waves share 16 candidates (small K)                 */
    BCMPC_KERNEL_SPLIT1 = 5,    /* BCMPC_PREC_SPLIT_F16: one workgroup = 1 x 16 candidates  */
    BCMPC_KERNEL_SPLIT2 = 6,    /*                                      2 x 16 candidates  */
    BCMPC_KERNEL_SPLIT4 = 7,    /*                                      4 x 16 candidates  */
    BCMPC_KERNEL_SPLITR = 8,    /* retired in round 6 (the resident-column rollout_rr, slower
                                   than SPLIT4 at every K): bcmpc_create returns
                                   BCMPC_ERR_UNSUPPORTED; the value stays reserved            */
    BCMPC_KERNEL_TEAM = 9       /* BCMPC_PREC_SPLIT_F16, small K: 2-layer NNDynamicsModel (tanh
                                   / relu, LayerNorm up to hidden 256), and at hidden 449..512
                                   (tanh) with a fused policy (<= 2 x 128) and / or the
                                   NNDynamicsRewardModel: one 16-candidate column per team of 1
                                   (hidden <= 256), 4 (512) or 8 (reward net) workgroups, every
                                   weight resident in registers, the output layer's partial sums
                                   exchanged between the team's workgroups once per step
                                   (rollout_team.hip).  Needs the whole grid resident:
                                   ceil(K/128)*8*members <= the device's CUs                 */
} bcmpc_kernel;

typedef enum bcmpc_policy_mode {   /* MPCcontrollerPolicyNet.self_exp (controllers.py:201-208) */
    BCMPC_POLICY_EXPLORE = 0,      /* self_exp=False: (1-explore)*mean + explore*U(low,high)   */
    BCMPC_POLICY_STOCHASTIC = 1    /* self_exp=True: mean + exp(logstd)*N(0,1) (device Philox)  */
} bcmpc_policy_mode;

/* Replaces the constructor arguments of MPCcontroller (controllers.py:28-35)
 * plus the NNDynamicsModel shape (dynamics.py:8-19, build_network :54-62). */
typedef struct bcmpc_config {
    int32_t state_dim;    /* S  (env.observation_space.shape[0], dynamics.py:23)  */
    int32_t action_dim;   /* A  (env.action_space.shape[0], dynamics.py:24)       */
    int32_t hidden;       /* h  (dynamics.py:59 size)                              */
    int32_t n_layers;     /* L  (dynamics.py:58 n_layers)                          */
    int32_t activation;   /* bcmpc_activation                                      */
    int32_t layer_norm;   /* FLAGS.LAYER_NORM (dynamics.py:68)                     */
    int32_t horizon;      /* H  (controllers.py:31 horizon)                        */
    int32_t cost;         /* bcmpc_cost                                            */
    int64_t num_paths;    /* K on this device (controllers.py:33 num_simulated_paths) */
    int32_t precision;    /* bcmpc_precision                                       */
    int32_t device;       /* HIP device ordinal                                    */
    int32_t kernel;       /* bcmpc_kernel: 0 = auto                                */
    int32_t policy_hidden;  /* 0: MPCcontroller; >0: MPCcontrollerPolicyNet policy width (hid_size) */
    int32_t policy_layers;  /* policy hidden layers (num_hid_layers, train_mpc_ppo.py:178)         */
    int32_t policy_mode;    /* bcmpc_policy_mode                                                   */
    int32_t model;        /* bcmpc_model                                           */
    int32_t reserved[3];  /* must be zero                                          */
} bcmpc_config;

/* Replaces the state NNDynamicsModel holds: TF variables
 * NNDynamicsModel/dense{,_1,..}/{kernel,bias} (+ LayerNorm/{gamma,beta}) and
 * the normalization stats of dynamics.py:41.  Host pointers, copied.
 * BCMPC_MODEL_REWARD (dynamics.py:150-177) passes the variables in TF creation
 * order: kernels/biases = dense (trunk [S+A,h]), dense_1 (delta hidden [h,h]),
 * dense_2 (delta out [h,S]), dense_3 (reward hidden [h,h]), dense_4 (reward out
 * [h,1]); ln_gamma/ln_beta = LayerNorm (trunk), LayerNorm_1 (delta), LayerNorm_2
 * (reward); plus mean_reward / std_reward (dynamics.py:143, 236). */
typedef struct bcmpc_weights {
    const float* const* kernels;   /* L+1 arrays, kernel[l] is [in, out] row-major  */
    const float* const* biases;    /* L+1 arrays of length out                      */
    const float* const* ln_gamma;  /* L arrays of length h, or NULL when LN is off  */
    const float* const* ln_beta;   /* L arrays of length h, or NULL                 */
    const double* mean_obs;        /* S */
    const double* std_obs;         /* S */
    const double* mean_action;     /* A */
    const double* std_action;      /* A */
    const double* mean_deltas;     /* S */
    const double* std_deltas;      /* S */
    const double* mean_reward;     /* 1 (BCMPC_MODEL_REWARD only, else NULL) */
    const double* std_reward;      /* 1 (BCMPC_MODEL_REWARD only, else NULL) */
} bcmpc_weights;

/* Output of one control step (controllers.py:82-85). */
typedef struct bcmpc_result {
    int64_t best_index;                       /* global candidate index, np.argmin semantics
                                                 (np.argmax for BCMPC_COST_REWARD)           */
    double best_cost;                         /* costs[best_index] (controllers.py:83); the best
                                                 discounted reward sum for BCMPC_COST_REWARD */
    double first_action[BCMPC_MAX_ACTION];    /* action_paths[0, best_index, :]              */
} bcmpc_result;

/* Replaces the policy net MPCcontrollerPolicyNet consults each step
 * (ppo_bc_policy.py:54-88): obz = clip((ob - ob_mean)/ob_std, -5, 5);
 * tanh dense x policy_layers; mean = dense(., A); logstd.  Host pointers, copied. */
typedef struct bcmpc_policy {
    const float* const* kernels;   /* policy_layers+1 arrays [in,out] (pi/pol/fc1.., final) */
    const float* const* biases;
    const float* ob_mean;          /* S (RunningMeanStd.mean, f32)   */
    const float* ob_std;           /* S (RunningMeanStd.std, f32)    */
    const float* logstd;           /* A                              */
    double explore;                /* MPCcontrollerPolicyNet.explore */
} bcmpc_policy;

/* CEM outer loop (BASELINE cfg5 "CEM outer loop (4 elite iters)"; not in the reference,
 * semantics in DESIGN.md "CEM").  Iteration i samples every candidate's actions as
 * clip(mu + sigma * z, low, high), z = Irwin-Hall(12) - 6 from Philox keyed by
 * (seed, global candidate, h, j, i); scores them like get_action; keeps the n_elite
 * lowest (cost, index) (NaN last, ties -> lower index); refits mu / sigma [H][A] to
 * the elites' mean / std (fixed reduction order) smoothed by alpha.  The answer is
 * the first action of the best candidate over ALL iterations (np.argmin over the
 * iteration-major concatenation of the cost vectors). */
typedef struct bcmpc_cem {
    int32_t iterations;   /* CEM iterations (cfg5: 4)                                   */
    int32_t n_elite;      /* elites per iteration, over all ranks (>= 1)               */
    double alpha;         /* new = alpha * old + (1 - alpha) * elite statistic         */
    int64_t k_global;     /* candidates over all ranks; result positions are
                             iteration * k_global + global index                      */
} bcmpc_cem;

typedef struct bcmpc_elite {   /* one (cost, global candidate index) record; index < 0 = empty */
    double cost;
    int64_t index;
} bcmpc_elite;

typedef struct bcmpc_engine bcmpc_engine;

int bcmpc_abi_version(void);
const char* bcmpc_last_error(void);

/* MPCcontroller.__init__ (controllers.py:28-41) + device allocation. */
int bcmpc_create(const bcmpc_config* cfg, bcmpc_engine** out);
int bcmpc_destroy(bcmpc_engine* eng);

/* Weight re-sync hook: idempotent on `version`; a new version
 * re-packs the dense kernels into MFMA fragment order on the device. */
int bcmpc_set_weights(bcmpc_engine* eng, const bcmpc_weights* w, uint64_t version);
uint64_t bcmpc_weights_version(const bcmpc_engine* eng);

/* Policy weights for MPCcontrollerPolicyNet engines (config.policy_hidden > 0). */
int bcmpc_set_policy(bcmpc_engine* eng, const bcmpc_policy* p, uint64_t version);

/* MPCcontrollerReward.gamma (controllers.py:99,139): step h's reward is scaled by
 * gamma**h (host pow, as Python's float ** int).  Default 1.0.  Reward engines only. */
int bcmpc_set_discount(bcmpc_engine* eng, double gamma);

/* env.action_space.low / .high (controllers.py:53). Defaults: [-1, 1]^A. */
int bcmpc_set_action_bounds(bcmpc_engine* eng, const double* low, const double* high);

/* MPCcontroller.get_action (controllers.py:57-88), synchronous, host memory.
 *   state    : S doubles (tiled K times, controllers.py:63)
 *   actions  : [H, K, A] doubles in C order (the array np.random.uniform returns
 *              at controllers.py:53), or NULL => draw them on the device with
 *              Philox4x32-10 keyed by (seed, cand_offset + k, h, j)
 *   cand_offset : global index of this device's first candidate (multi-GPU shard)
 *   out      : best index (global) / cost / first action
 *   costs_out: optional K doubles, per-candidate trajectory cost (cost_functions.py:59-63),
 *              or discounted reward sum (BCMPC_COST_REWARD, controllers.py:150)
 * Without a communicator the state travels in the kernel arguments and the argmin writes the
 * result into mapped host memory: one rollout + one argmin launch, one stream synchronisation. */
int bcmpc_get_action(bcmpc_engine* eng, const double* state, const double* actions,
                     uint64_t seed, int64_t cand_offset, bcmpc_result* out, double* costs_out);

/* MPCcontroller.get_action with the reference's RNG contract (controllers.py:53): the
 * [H, k_global, A] array np.random.uniform(low, high, size) would return is drawn from NumPy's
 * legacy MT19937 state (mt_key[624] / mt_pos as np.random.get_state() holds them; advanced in
 * place, as the one NumPy call would advance them, and only when the call succeeds) -- only this
 * shard's [cand_offset, cand_offset + K) slice of each step is produced:
 *   default: ON THE GPU (mt_device.hip): the draw is cut into chunks, each chunk's start window
 *     reached by an MT19937 jump-ahead polynomial (GF(2) correlation on the device) and its words
 *     generated, tempered and scaled by one workgroup straight into HBM; no host draw, no PCIe
 *     upload of the array (the key, 2.5 KB, goes up; the final state comes back with the result);
 *   BCMPC_MT_PATH=host: on the host into pinned memory, step by step or split over host threads
 *     by jump-ahead (bcmpc_mt19937_uniform_par), each slice copied as soon as it is drawn.
 * Then as bcmpc_get_action (seed: the stochastic policy's Philox normals); out->first_action is
 * action_paths[0, best] of that same array (policy engines: the mixed action, the array being the
 * exploration draw of controllers.py:191). */
int bcmpc_get_action_mt19937(bcmpc_engine* eng, const double* state, uint32_t* mt_key, int32_t* mt_pos,
                             const double* low, const double* high, int64_t k_global, int64_t cand_offset,
                             uint64_t seed, bcmpc_result* out, double* costs_out);

/* Small draws (<= BCMPC_MT_ZC_WORDS generator words, the reference's K = 400 steps) of
 * bcmpc_get_action_mt19937: after a call, a worker thread draws the NEXT call's rows from the advanced
 * state; a call whose (key, pos, bounds, shard) equal that job's start uses them -- a hit (rows
 * complete, copied into HBM when the copy has landed) or, on team-kernel engines, a late hit (the job
 * still running: the kernel waits for the rows' sequence word in mapped memory) -- else it draws itself
 * (a miss).  Larger draws (the device path): the NEXT call's draw is enqueued on the device from this
 * draw's final state -- behind a synchronous call's argmin, or beside its rollout on a stream of its own
 * when the slab grid leaves CUs free (K <= 32 per CU) -- (BCMPC_MT_SPECULATE=0: off), used by the
 * next call when NumPy's state, bounds and shard equal its start (two misses in a row pause it for 32
 * calls).  out5 = {hits incl. late, late hits, misses, speculative hits, speculative misses} since
 * bcmpc_create. */
int bcmpc_predraw_stats(const bcmpc_engine* eng, uint64_t* out5);

/* The same draw as bcmpc_get_action_mt19937 on the device, alone: this engine's shard
 * [H, K, A] of np.random.uniform(low, high, [H, k_global, A]) (controllers.py:53) drawn on the GPU
 * from (mt_key, mt_pos), copied to `out` (host, H*K*A doubles); mt_key / mt_pos advance as the one
 * NumPy call would advance them.  For tests and for callers that want the array itself. */
int bcmpc_mt19937_uniform_device(bcmpc_engine* eng, uint32_t* mt_key, int32_t* mt_pos, const double* low,
                                 const double* high, int64_t k_global, int64_t cand_offset, double* out);

/* Host only (no GPU): n_rows x action_dim doubles of np.random.uniform(low, high) from the
 * legacy MT19937 state (mt_key / mt_pos in/out) -- the generator bcmpc_get_action_mt19937 uses. */
int bcmpc_mt19937_uniform(uint32_t* mt_key, int32_t* mt_pos, const double* low, const double* high,
                          int32_t action_dim, int64_t n_rows, double* out);

/* Host only (no GPU): the same stream as bcmpc_mt19937_uniform, drawn by up to `threads` host
 * threads (<= 0: BCMPC_MT_THREADS, else min(8, hardware threads)) that each jump ahead to their own
 * block of the stream (MT19937 jump-ahead, csrc/mt_jump.cpp) and draw at least
 * min_words_per_thread generator words (< 0: the library's default, 2^20).  n_rows rows in
 * repeating groups of `period` rows; only rows r with r % period in [keep_lo, keep_hi) are stored
 * (a shard's candidates of each step: period = k_global), densely in row order.  mt_key / mt_pos
 * end exactly where the serial draw leaves them; *used_threads (optional) = threads used (1: serial).
 * The path bcmpc_get_action_mt19937 takes for large draws. */
int bcmpc_mt19937_uniform_par(uint32_t* mt_key, int32_t* mt_pos, const double* low, const double* high,
                              int32_t action_dim, int64_t n_rows, int64_t period, int64_t keep_lo, int64_t keep_hi,
                              double* out, int32_t threads, int64_t min_words_per_thread, int32_t* used_threads);

/* Actions the last rollout actually used for step 0 (policy engines:
 * action_paths[0] of controllers.py:233), copied to host K x A doubles. */
int bcmpc_first_actions(bcmpc_engine* eng, double* out);

/* Device-memory, asynchronous form (no host sync; graph-capturable).
 *   d_state      : device, S doubles, or [K, S] when state_stride == S (predict mode,
 *                  dynamics.py:106 on per-candidate states)
 *   d_actions    : device [H, K, A] doubles, or NULL => device RNG
 *   d_costs      : device K doubles (required when cost == CHEETAH or REWARD)
 *   d_traj       : device [H+1, K, S] doubles or NULL (states_paths_all, controllers.py:65-74)
 *   d_result     : device bcmpc_result or NULL (argmin + first action)
 *   stream       : hipStream_t the launches are enqueued on, used verbatim (NULL is HIP's
 *                  null stream; pass bcmpc_stream(eng) for the engine's own stream) */
int bcmpc_rollout_async(bcmpc_engine* eng, const double* d_state, int64_t state_stride,
                        const double* d_actions, uint64_t seed, int64_t cand_offset,
                        double* d_costs, double* d_traj, bcmpc_result* d_result, void* stream);

/* MPCcontrollerPolicyNet engines: bcmpc_rollout_async plus the actions actually rolled out at
 * EVERY step -- d_actions_out [H, K, A] f64, the reference's action_paths (controllers.py:208-213:
 * the policy mean mixed with the exploration draw, or mean + exp(logstd) * N(0,1) when self_exp)
 * -- and optionally the states (d_traj [H+1, K, S]), so a caller (or a test) can replay each step.
 * d_actions: the [H, K, A] exploration draw or NULL (device Philox). */
int bcmpc_rollout_policy_async(bcmpc_engine* eng, const double* d_state, const double* d_actions, uint64_t seed,
                               int64_t cand_offset, double* d_costs, double* d_traj, double* d_actions_out,
                               bcmpc_result* d_result, void* stream);

/* CEM, single device, synchronous: all iterations on the engine's stream.
 *   mu, sigma : host [H][A] doubles, in: the initial distribution, out: the refit one
 *   out       : best_index = iteration * K + candidate, best_cost, first action
 * Needs a group-kernel engine with the fused objective (cheetah cost or learned reward;
 * for the reward objective "best" is the argmax). */
int bcmpc_cem_get_action(bcmpc_engine* eng, const double* state, const bcmpc_cem* params, uint64_t seed,
                         double* mu, double* sigma, bcmpc_result* out);

/* CEM building blocks for multi-device runs (device pointers, stream-ordered):
 *   cem_rollout : one iteration's sampling + rollout of this device's shard into d_costs;
 *                 with d_result, also the shard's best, merged (merge != 0) with the
 *                 running best already in d_result
 *   select      : the n_elite lowest of m records -- d_pairs, or d_costs (index =
 *                 index_base + i) when d_pairs is NULL -- written in ascending index
 *                 order to d_out (padded with index -1), the count to d_count
 *   cem_refit   : mu / sigma update from the selected elites (regenerated from Philox) */
int bcmpc_cem_rollout_async(bcmpc_engine* eng, const double* d_state, const double* d_mu, const double* d_sigma,
                            uint64_t seed, int32_t iteration, int64_t cand_offset, int64_t k_global,
                            double* d_costs, bcmpc_result* d_result, int32_t merge, void* stream);
int bcmpc_select_async(bcmpc_engine* eng, const bcmpc_elite* d_pairs, const double* d_costs, int64_t m,
                       int64_t index_base, int32_t n_elite, bcmpc_elite* d_out, int32_t* d_count, void* stream);
int bcmpc_cem_refit_async(bcmpc_engine* eng, const bcmpc_elite* d_elite, const int32_t* d_count, uint64_t seed,
                          int32_t iteration, double alpha, double* d_mu, double* d_sigma, void* stream);

/* ------------------------------------------------------------------------
 * NNDynamicsModel.fit (dynamics.py:81-104) on the GPU:
 * `iterations` Adam steps (TF1 AdamOptimizer, dynamics.py:50-52) on the mean
 * squared error of the normalised state deltas, batches gathered on the device
 * from a resident copy of the model data buffer by host-chosen row indices (the
 * caller draws them exactly as DataBufferGeneral.sample does, data_buffer.py:45-57).
 * A fitter owns the f32 parameters and the Adam slots (m, v, beta powers), which
 * persist across runs like the reference's optimizer variables. */
typedef struct bcmpc_fit_config {
    int32_t state_dim;     /* S */
    int32_t action_dim;    /* A */
    int32_t hidden;        /* h (true width, no padding) */
    int32_t n_layers;      /* L */
    int32_t activation;    /* bcmpc_activation */
    int32_t layer_norm;    /* FLAGS.LAYER_NORM (dynamics.py:68) */
    int32_t batch_size;    /* dynamics.py:48 batch_size (max rows per step) */
    int32_t device;
    float learning_rate;   /* dynamics.py:47 */
    float beta1, beta2, epsilon;   /* tf.train.AdamOptimizer defaults 0.9, 0.999, 1e-8 */
    int32_t model;         /* bcmpc_model: BCMPC_MODEL_REWARD fits NNDynamicsRewardModel (dynamics.py:153-160,
                              195-219: loss_dynamic + loss_reward over the two-head net; n_layers 2, tanh;
                              kernels / biases dense .. dense_4, LayerNorm trunk / delta / reward) */
} bcmpc_fit_config;

typedef struct bcmpc_fitter bcmpc_fitter;

int bcmpc_fit_create(const bcmpc_fit_config* cfg, bcmpc_fitter** out);
int bcmpc_fit_destroy(bcmpc_fitter* f);
/* parameters (TF layout [in, out] kernels, biases, LN gamma/beta) + the normalization stats */
int bcmpc_fit_set_params(bcmpc_fitter* f, const bcmpc_weights* w);
int bcmpc_fit_get_params(bcmpc_fitter* f, float* const* kernels, float* const* biases, float* const* ln_gamma,
                         float* const* ln_beta);
/* the model data buffer: n rows of state (S), action (A), state delta (S), f64, uploaded to HBM */
int bcmpc_fit_set_data(bcmpc_fitter* f, const double* states, const double* actions, const double* deltas,
                       int64_t n);
/* `iterations` steps; step i uses batch_sizes[i] rows, indices concatenated in `indices`;
 * losses (optional, host, [iterations]) = each step's loss before its update */
int bcmpc_fit_run(bcmpc_fitter* f, const int64_t* indices, const int32_t* batch_sizes, int32_t iterations,
                  float* losses);
/* reward model: the buffer's rewards (one f64 per row of bcmpc_fit_set_data; normalised with
 * mean_reward / std_reward of bcmpc_fit_set_params, dynamics.py:203); after a run, its per-step
 * reward losses ([iterations], before each update; bcmpc_fit_run's losses are the dynamics losses) */
int bcmpc_fit_set_rewards(bcmpc_fitter* f, const double* rewards, int64_t n);
int bcmpc_fit_reward_losses(bcmpc_fitter* f, float* losses);
const char* bcmpc_fit_last_error(void);

/* ------------------------------------------------------------------------
 * Candidate sharding over GPUs: one process per GPU, rank r owns the
 * global candidates [cand_offset, cand_offset + K).  The library owns the one
 * collective of a control step: a communicator attached to an engine makes every
 * bcmpc_get_action / bcmpc_get_action_mt19937 / bcmpc_rollout_async (with d_result)
 * of that engine all-gather the ranks' 144-byte result records over RCCL (xGMI)
 * right after the argmin launch, stream-ordered, and reduce them on the device with
 * np.argmin's rule (controllers.py:82: first NaN, else smallest cost, ties -> lowest
 * global index; np.argmax for BCMPC_COST_REWARD, controllers.py:152): every rank
 * returns the GLOBAL best.  All ranks must call with the same state and hold >= 1
 * candidate.  No Python or torch is needed: rank 0 makes the id, any out-of-band
 * channel (MPI, a file, a socket) carries its 128 bytes to the other ranks.
 * RCCL (librccl.so.1) is loaded on first use.  Replaces nothing in the reference's
 * hot path (single process); its only collective, train_mpc_ppo.py:388, gathers
 * episode statistics. */
#define BCMPC_COMM_ID_BYTES 128
typedef struct bcmpc_comm bcmpc_comm;
int bcmpc_comm_unique_id(uint8_t* id /* [BCMPC_COMM_ID_BYTES] */);             /* ncclGetUniqueId   */
int bcmpc_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                    bcmpc_comm** out);                                          /* ncclCommInitRank  */
int bcmpc_comm_destroy(bcmpc_comm* comm);
/* attach (comm != NULL) or detach (NULL); the comm's device must be the engine's.
 * CEM calls (bcmpc_cem_*) do not exchange. */
int bcmpc_engine_set_comm(bcmpc_engine* eng, bcmpc_comm* comm);
/* Host only: the np.argmin (maximize: np.argmax) winner of n result records, for hosts
 * that exchange the records themselves (e.g. MPI / gloo). */
int bcmpc_select_results(const bcmpc_result* recs, int32_t n, int32_t maximize, bcmpc_result* out);
/* The same select on the device, stream-ordered (the kernel the library's exchange runs after its
 * all-gather): d_recs [n] records -> d_out (must not overlap d_recs), 1 <= n <= 4096. */
int bcmpc_select_results_async(const bcmpc_result* d_recs, int32_t n, int32_t maximize, bcmpc_result* d_out,
                               void* stream);

/* Device stream the engine launches on (hipStream_t as void*). */
void* bcmpc_stream(bcmpc_engine* eng);

/* Small-K team kernel (bcmpc_engine_info kernel == BCMPC_KERNEL_TEAM): its workgroups wait for each
 * other once per step, so they must all be resident.  A team that cannot meet within ~1 s (another
 * process or kernel holding CUs) gives up and flags it; the synchronous entry points then rerun the
 * call on a fallback engine of the same net (the split slab kernel, else the fp32 group kernel;
 * not with a communicator attached: BCMPC_ERR_HIP).  Stream-ordered callers (bcmpc_rollout_async,
 * bcmpc_rollout_policy_async, bcmpc_cem_rollout_async) call bcmpc_engine_status once their stream has
 * completed: BCMPC_ERR_HIP when a launch of this engine since the last check gave up (its outputs
 * are not valid), BCMPC_OK otherwise; reading clears the flag.  Team launches of one process on
 * different streams of a device are serialised (stream-ordered) by the library. */
int bcmpc_engine_status(bcmpc_engine* eng);
/* number of synchronous calls of this engine rerun on the fallback engine */
int bcmpc_engine_team_reruns(const bcmpc_engine* eng, uint64_t* reruns);

/* Kernel timing (off by default): with on != 0 every launch chain of this engine is bracketed
 * by HIP event markers (~6 us per synchronous get_action at small K, measured), which
 * bcmpc_last_kernel_ms reads.  Not part of the reference interface: a measurement switch. */
int bcmpc_engine_set_timing(bcmpc_engine* eng, int32_t on);
/* Timing of the last rollout kernel launched through bcmpc_get_action /
 * bcmpc_rollout_async / bcmpc_cem_get_action, in milliseconds (HIP events on the launch
 * stream); requires timing on for that launch (else BCMPC_ERR_ARG) and waits for it. */
int bcmpc_last_kernel_ms(bcmpc_engine* eng, float* rollout_ms, float* argmin_ms);

/* Static shape facts for tests: padded hidden size and packed weight bytes. */
int bcmpc_engine_info(const bcmpc_engine* eng, int32_t* hidden_padded, int64_t* packed_weight_bytes,
                      int32_t* waves_per_block, int32_t* kernel);
/* The device kernel instance the engine launches per rollout, as text (e.g. "rollout_pp<512> f16",
 * "rollout_x3<512,NC=4,NW=8> split"), NUL-terminated and truncated to cap bytes: tests and the bench
 * assert / report which layout the engine selected.  Round 5 (ABI 4). */
int bcmpc_engine_layout(const bcmpc_engine* eng, char* buf, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* BCMPC_H_ */
