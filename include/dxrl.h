/*
 * dxrl.h -- C ABI of the MI355X-native vectorised manipulation-env hot path.
 *
 * Plain C: no torch / HIP types in the signatures.  Device buffers are
 * passed as plain pointers (HBM addresses valid on the env's device); streams
 * as `void*` (a hipStream_t, NULL = the device's null stream).  Every entry
 * point returns DXRL_OK (0) or a negative status; dxrl_last_error() returns a
 * thread-local message for the last failing call.  Calls on one handle are
 * not thread-safe; kernels are stream-ordered and asynchronous.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the I2S9/dexterous-rl-manipulation checkout).
 */
#ifndef DXRL_H_
#define DXRL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DXRL_ABI_VERSION 1

/* status codes */
#define DXRL_OK 0
#define DXRL_E_INVALID (-1)     /* bad argument (shape, null pointer, range)  -> ValueError   */
#define DXRL_E_HIP (-2)         /* HIP runtime / launch failure               -> RuntimeError */
#define DXRL_E_UNSUPPORTED (-3) /* configuration this build does not compile   -> ValueError   */
#define DXRL_E_TAPE (-4)        /* a parity tape ran out (see dxrl_rollout_*)  -> RuntimeError */

/* reward plugin selection: envs/manipulation_env.py:64-73 */
#define DXRL_REWARD_SPARSE 0 /* rewards/reward_shaping.py:190-242 SparseReward  */
#define DXRL_REWARD_DENSE 1  /* rewards/reward_shaping.py:12-187  RewardShaping */

/* number of f64 slots of one reset draw record: joints + (size, mass, friction) + spawn xyz */
#define DXRL_RESET_EXTRA 6
#define DXRL_MAX_CURRICULA 256

/* episode success rule of a rollout:
 *   TRAINING   -- training/episode_utils.py:52   info.get("success", False) -> always 0
 *   TERMINATED -- evaluation/evaluator.py:157, robustness_tests.py:303   success = terminated */
#define DXRL_SUCCESS_TRAINING 0
#define DXRL_SUCCESS_TERMINATED 1

/* One curriculum configuration -- experiments/config.py:17-42 (CurriculumConfig).
 * A range is used iff its has_* flag is set (config.py:44-84: one draw each,
 * in the order size, mass, friction).  friction_is_f64_scalar reproduces the
 * NumPy-2 promotion when the friction is a numpy.float64 (scheduler
 * interpolation, experiments/curriculum_scheduler.py:90-139): the velocity
 * damping multiply then runs in f64 (manipulation_env.py:215-216). */
typedef struct dxrl_curriculum {
    double object_size, object_mass, friction_coefficient;
    double size_range[2], mass_range[2], friction_range[2];
    double spawn_x_range[2], spawn_y_range[2], spawn_z_range[2];
    int32_t has_size_range, has_mass_range, has_friction_range, friction_is_f64_scalar;
} dxrl_curriculum;

/* Constructor arguments -- envs/manipulation_env.py:24-34 (+ reward_shaping.py:14-25 weights). */
typedef struct dxrl_env_config {
    int32_t num_envs;          /* N envs on this device (shard)                 */
    int32_t num_fingers;       /* manipulation_env.py:26 (this build: 5)         */
    int32_t joints_per_finger; /* manipulation_env.py:27 (this build: 3)         */
    int32_t max_episode_steps; /* manipulation_env.py:29                         */
    int32_t reward_type;       /* DXRL_REWARD_*  (manipulation_env.py:31)        */
    int32_t has_object_position; /* manipulation_env.py:28 object_position given */
    double object_position[3];
    double distance_weight, contact_weight, closure_weight, stability_weight;
    uint64_t seed;             /* device RNG: env i keyed by (seed, global_env_offset + i) */
    int64_t global_env_offset; /* first global env id of this shard (multi-GPU)  */
} dxrl_env_config;

/* Byte offsets (from the state base) of the struct-of-arrays env state in HBM. */
typedef struct dxrl_env_layout {
    int64_t total_bytes;
    int64_t jp, jv;      /* f32 [D][N]  joint positions / velocities            */
    int64_t op;          /* f64 [3][N]  object position                         */
    int64_t ov;          /* f32 [3][N]  object velocity                         */
    int64_t flags;       /* u32 [N]     contacts | prev<<8 | has_prev<<16 | op_is_f32<<17 | has_object<<18 */
    int64_t step_count;  /* i32 [N]                                              */
    int64_t size, mass, friction; /* f64 [N] current episode curriculum values  */
    int64_t cfg_index;   /* i32 [N]     curriculum table row per env             */
    int64_t reset_ctr;   /* u64 [N]     resets so far (device-RNG counter)       */
    int64_t curricula;   /* dxrl_curriculum [DXRL_MAX_CURRICULA]                 */
} dxrl_env_layout;

typedef struct dxrl_env dxrl_env;

int dxrl_abi_version(void);
const char* dxrl_last_error(void);

/* Layout of the state slab the caller allocates (device memory, 256-B aligned). */
int dxrl_env_layout_for(const dxrl_env_config* cfg, dxrl_env_layout* out);

/* Replaces DexterousManipulationEnv.__init__ (envs/manipulation_env.py:24-122).
 * `state` = caller-owned device slab of layout.total_bytes on `device`.
 * Initialises the SoA (zeros, has_object from cfg) on `stream`. */
int dxrl_env_create(const dxrl_env_config* cfg, int32_t device, void* state, void* stream, dxrl_env** out);
int dxrl_env_destroy(dxrl_env* env);

/* Curriculum table + per-env row (host arrays, copied on `stream`; returns after the copies
 * completed, so the arrays may be temporaries).
 * env_index == NULL -> every env uses row 0.  Takes effect at the next reset,
 * as assigning env.curriculum_config does (evaluation/component_ablation.py:166). */
int dxrl_env_set_curricula(dxrl_env* env, const dxrl_curriculum* table, int32_t n,
                           const int32_t* env_index, void* stream);
/* The same without waiting: the copies are only enqueued on `stream`, so `table` and
 * `env_index` (pinned host memory) must stay unchanged until the stream has passed them
 * (the trainer's scheduler pushes a progression mid-iteration without a host sync). */
int dxrl_env_set_curricula_async(dxrl_env* env, const dxrl_curriculum* table, int32_t n,
                                 const int32_t* env_index, void* stream);

/* Replaces reset(seed, options) (envs/manipulation_env.py:124-182).
 * mask   : device u8 [N] or NULL (all envs)
 * draws  : device f64 [N][D+6] resolved reset draws (parity mode: the host
 *          replays each env's gymnasium PCG64 stream), or NULL -> device Philox.
 *          Slots: D joint uniforms, size, mass, friction, spawn x, y, z (a slot
 *          is read only when the reference would draw it).
 * obs    : device f32 [N][obs_dim] or NULL. */
int dxrl_env_reset(dxrl_env* env, const uint8_t* mask, const double* draws, float* obs, void* stream);

/* Replaces step(action) (envs/manipulation_env.py:184-252) incl. _update_contacts
 * (:285-310), the reward plugin (rewards/reward_shaping.py:50-242),
 * _check_termination (:332-336) and _get_observation (:254-264).
 * actions f32 [N][D]; obs f32 [N][obs_dim] (nullable); reward f64 [N];
 * terminated/truncated u8 [N]; components f64 [N][4] (nullable). */
int dxrl_env_step(dxrl_env* env, const float* actions, float* obs, double* reward,
                  uint8_t* terminated, uint8_t* truncated, double* components, void* stream);

/* The reward plugins' own entry point, for callers outside env.step():
 *   rewards/reward_shaping.py:50-99   RewardShaping.compute(joint_positions, finger_tips,
 *                                     object_position, contacts, num_fingers, joints_per_finger)
 *   rewards/reward_shaping.py:205-242 SparseReward.compute(...)
 * as called at envs/manipulation_env.py:318-325, for `count` independent items.  The dense
 * terms are the step kernels' own dense_reward (csrc/dxrl_device.h) on the given inputs.
 *   weights          HOST f64 [4] distance, contact, closure, stability (dense only);
 *                    every other array is device memory
 *   joint_positions  f32 [count][15]      (the env's f32 joint array, ME:143-145)
 *   finger_tips      f64 [count][5][3]    (ME:296-303)
 *   object_position  f64 [count][3]
 *   contacts         f32 [count][5]       (ME:310; > 0.5 counts as a contact)
 *   prev_contacts    f32 [count][5], has_prev u8 [count]: RewardShaping.prev_contacts (None ==
 *                    has_prev 0), read and updated in place as RS:172-185 does (dense only)
 *   out              f64 [count][5]: total, distance, contact, closure, stability
 * num_fingers / joints_per_finger must be this build's 5 / 3 (DXRL_E_UNSUPPORTED otherwise). */
int dxrl_reward_compute(int32_t device, int32_t reward_type, const double* weights, int64_t count,
                        int32_t num_fingers, int32_t joints_per_finger, const float* joint_positions,
                        const double* finger_tips, const double* object_position, const float* contacts,
                        float* prev_contacts, uint8_t* has_prev, double* out, void* stream);

/* Recompute the observation of the current state (envs/manipulation_env.py:254-264). */
int dxrl_env_observe(dxrl_env* env, float* obs, void* stream);

/* Assigning env.max_episode_steps (read by training/episode_utils.py:38 and
 * the truncation test manipulation_env.py:245). */
int dxrl_env_set_max_episode_steps(dxrl_env* env, int32_t max_episode_steps);

/* SimpleLearner.select_action / update for a batch of independent learners
 * (policies/simple_learner.py:49-95), for callers that drive env.step()
 * themselves (the Gymnasium facade).  gauss = f64 [N][D] standard normals
 * (np.random.normal(0, s) == 0 + s * gauss); update applies to envs whose
 * mask byte is set -- the host decides `reward > best_reward` because it owns
 * the RNG stream whose consumption depends on it. */
int dxrl_learner_select(int32_t device, int32_t num_envs, const void* learner_state, double exploration_noise,
                        const double* gauss, float* actions, void* stream);
int dxrl_learner_update(int32_t device, int32_t num_envs, void* learner_state, double learning_rate,
                        double action_clip_range, const double* gauss, const double* reward, const uint8_t* mask,
                        void* stream);

/* ------------------------------------------------------------------------
 * Fused rollout with per-env SimpleLearner hill-climbers
 * (training/episode_utils.py:13-55 run_episode loop + policies/simple_learner.py:49-99).
 * One launch runs `num_steps` env steps of every env, auto-resetting at
 * episode end (terminated || truncated || step_count == max_steps) exactly as
 * consecutive run_episode() calls do.  State stays in registers across steps.
 * ------------------------------------------------------------------------ */
typedef struct dxrl_learner_layout {
    int64_t total_bytes;
    int64_t mean;        /* f32 [D][N] mean_action                             */
    int64_t best;        /* f64 [N]    best_reward                             */
    int64_t ep_return;   /* f64 [N]    running total_reward of the open episode */
    int64_t noise_ctr;   /* u64 [N]    device-RNG counter                      */
} dxrl_learner_layout;

typedef struct dxrl_learner_config {
    double learning_rate;     /* simple_learner.py:27 */
    double exploration_noise; /* :28 */
    double action_clip_range; /* :29 */
    uint64_t seed;            /* device RNG (Philox) key; the reference uses the global np.random */
} dxrl_learner_config;

typedef struct dxrl_rollout_io {
    /* parity tapes (all NULL -> device Philox streams) */
    const double* gauss;      /* f64 [N][gauss_stride] legacy-MT19937 gauss values per env  */
    int64_t gauss_stride;
    const double* reset_draws;/* f64 [N][reset_stride] consecutive reset records (D+6 each) */
    int64_t reset_stride;
    /* episode records (nullable), [N][record_cap] */
    int32_t record_cap;
    double* ep_return;
    int32_t* ep_length;
    uint8_t* ep_success;
    int32_t* ep_end_step;     /* rollout step index at which the episode ended */
    /* per-env outputs (nullable) */
    int32_t* ep_count;        /* i32 [N] episodes finished in this call   */
    int32_t* gauss_used;      /* i32 [N] tape values consumed             */
    int32_t* status;          /* i32 [1] device error word (tape overrun) */
    /* i32 [N] episode budget of this call (nullable = unbounded): an env stops once it has
       finished that many episodes, before the next episode's env.reset() -- a driver's
       `for episode in range(num_episodes)` loop (evaluation/component_ablation.py:154-166). */
    const int32_t* episode_budget;
} dxrl_rollout_io;

int dxrl_learner_layout_for(int32_t num_envs, int32_t action_dim, dxrl_learner_layout* out);
/* zero mean_action, best_reward = -inf, ep_return = 0 (SimpleLearner.__init__, simple_learner.py:45-47) */
int dxrl_learner_init(int32_t device, int32_t num_envs, void* learner_state, void* stream);
/* policy.reset() for every env: best_reward = -inf (simple_learner.py:97-99) and the
 * open-episode return = 0 (run_episode starts a new episode, episode_utils.py:33-39). */
int dxrl_learner_reset(int32_t device, int32_t num_envs, void* learner_state, const uint8_t* mask, void* stream);
/* learner_state must have been laid out for env's num_envs. */
int dxrl_rollout_simple(dxrl_env* env, void* learner_state, const dxrl_learner_config* lcfg,
                        int32_t num_steps, int32_t max_steps, int32_t success_rule,
                        const dxrl_rollout_io* io, void* stream);

/* ------------------------------------------------------------------------
 * bf16 MFMA GEMM used by the actor-critic learner (no reference counterpart;
 * exported for tests and diagnostics).  C[M][N] = epi(A[M][K] . Bt[N][K]^T):
 * bias (bias[n*bias_stride]), act (0 identity / 1 tanh), gate (multiply by
 * 1 - gate[m][n]^2), outputs f32 row-major Cf, bf16 row-major Crm, bf16
 * feature-major Cfm[n][m] (each nullable).  splits > 1: split-K over K into
 * `partial` (f32 [splits + 16][M][N]: the last 16 slabs are the two-level reduction's
 * scratch) reduced into Cf (ld = N).  K % 32 == 0.
 * ------------------------------------------------------------------------ */
int dxrl_gemm_bf16(int32_t device, const void* A, int64_t lda, const void* Bt, int64_t ldb, int64_t M, int32_t N,
                   int32_t K, const float* bias, int64_t bias_stride, int32_t act, const void* gate, int64_t ldg,
                   float* Cf, int64_t ldcf, void* Crm, int64_t ldc, void* Cfm, int64_t ldfm, float* Cffm,
                   int64_t ldffm, int32_t splits, float* partial, void* stream);
/* Weight gradient out[O][I] = sum_m Y[m][o] X[m][i] from row-major bf16 operands
 * (k-major MFMA operands via ds_read_b64_tr_b16); split-K over m into `partial`
 * (f32 [splits + 16][O][I]; the last 16 slabs are reduction scratch) reduced in fixed order
 * (deterministic).  O, I, ldy, ldx % 8 == 0. */
int dxrl_wgrad_bf16(int32_t device, const void* Y, int64_t ldy, int32_t O, const void* X, int64_t ldx, int32_t I,
                    int64_t M, int32_t splits, float* partial, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Policy-gradient learner (NEW capability: the reference has no network,
 * no GAE and no gradient -- SURVEY.md §8(a) A11-A13; parity unpinned vs the
 * reference, pinned by tests against a torch fp32 restatement).
 * Actor 45->256->256->15 (tanh) + state-independent log_std; critic
 * 45->256->256->1.  Master parameters f32 (dxrl_pg_sizes().params elements,
 * padded blocks, see csrc/dxrl_pg.h), bf16 packed copies for the MFMA GEMMs.
 * ------------------------------------------------------------------------ */
int dxrl_pg_sizes(int64_t* params, int64_t* packed_bf16);
int dxrl_pg_pack_weights(int32_t device, const float* params, void* packed, void* stream);

typedef struct dxrl_pg_rollout_args {
    int32_t horizon;           /* env steps per env in this call (T)                       */
    int32_t max_steps;         /* run_episode loop bound (episode_utils.py:38-42)          */
    uint64_t policy_seed;      /* Philox key of the action / noise streams                 */
    uint64_t iteration;        /* Philox counter base (iteration * T + t)                  */
    double obs_noise_std;      /* robustness_tests.py:199-207 (0 = off)                    */
    double dyn_noise_std;      /* robustness_tests.py:180-187 (0 = off)                    */
    void* obs_rm;              /* bf16 [(T+1) N][64] policy inputs (+ bootstrap row block) */
    void* obs_fm;              /* bf16 [64][T N] feature-major copy (nullable)             */
    float* act;                /* f32 [T N][16] sampled (pre-clip) actions                 */
    float* logp;               /* f32 [T N] log pi(a|s) at sampling time                   */
    float* rew;                /* f32 [T N]                                                */
    uint8_t* done;             /* u8  [T N] episode ended after this step                  */
    double* ep_return;         /* f64 [N] open-episode return, persists across calls       */
    int32_t* ep_count;         /* i32 [N] episodes finished in this call                   */
    double* ep_sum_return;     /* f64 [N]                                                  */
    int32_t* ep_sum_length;    /* i32 [N]                                                  */
    int32_t* ep_successes;     /* i32 [N] finished episodes that terminated (>= 3 contacts) */
    int32_t diag_flags;        /* diagnostics only (timing ablations): bit0 skip the actor MLP
                                  (mu = 0), bit1 skip the env step; kernel selection (bit-
                                  identical tapes): 16 the one-lane-per-env kernel, 1024 the
                                  32-env kernel (default at >= 32 envs per CU), 2048 the 16-env
                                  kernel at any size; 128 per-step cycle stamps of the 16- / 32-env
                                  kernel (printed to stderr); 256 skip the 16-env kernel's draws,
                                  512 its reward settle (timing only: results are wrong); 32 / 64
                                  (the retired 4-wave kernel) are rejected; 0 in every real run */
    int32_t success_rule;      /* DXRL_SUCCESS_* for the episode records                   */
    int32_t record_cap;        /* per-env episode records [N][record_cap] (0 = none)       */
    double* rec_return;
    int32_t* rec_length;
    uint8_t* rec_success;
    int32_t* rec_end_step;     /* step index t within this call                            */
    uint16_t* ep_code;         /* u16 [T N] episode-end codes for the curriculum scheduler feed
                                  (dxrl_sched_scan): 0 = no episode ended at this step, else
                                  (episode length << 1) | success (nullable)                  */
    float* applied_act;        /* f32 [T N][16] the action the env integrated, after dynamics
                                  noise (nullable; parity checks replay it on the CPU)        */
    /* Fused-noise tapes (config C5; nullable, parity checks only; default kernel only): the
       f32 noise values exactly as the kernel added them, n = f32(sigma) * z with z the
       device's Box-Muller normal -- robustness_tests.py:180-182 draws n = N(0, sigma) and
       adds f32(n) to the action; :199-207 adds f32(n) to every observation element. */
    float* dyn_noise_tape;     /* f32 [T N][16] dynamics noise per action dim (0 if off)    */
    float* obs_noise_tape;     /* f32 [(T+1) N][48] observation noise per obs element       */
    void* h2_tape;             /* bf16 [T N][264] the actor's layer-2 activations of every step
                                  (nullable; written by the 16- and 32-env kernels, not the 64-env
                                  reference one, see dxrl_pg_rollout_kernel;
                                  dxrl_pg_fused_args.h2_in of the actor's first train pass under
                                  these weights)                                               */
} dxrl_pg_rollout_args;

/* Fused policy + env rollout: T steps of actor MLP (bf16 MFMA) -> Gaussian
 * sample -> [dynamics noise] -> env step -> tape, auto-reset (device RNG). */
int dxrl_pg_rollout(dxrl_env* env, const void* packed, const float* params, const dxrl_pg_rollout_args* args,
                    void* stream);
/* Which kernel dxrl_pg_rollout runs for this env and diag_flags (without a feature-major tape):
 * 1 the 16-env kernel (< 32 envs per CU), 2 the 32-env kernel (both write h2_tape),
 * 0 the 64-env reference kernel (diag_flags & 16).  Host-only query. */
int dxrl_pg_rollout_kernel(const dxrl_env* env, int32_t diag_flags, int32_t* kernel);

/* GAE reverse scan; values f32 [(T+1) N]; writes adv/ret [T N] and this rank's advantage
 * moments stats[5] = T N, stats[6] = mean(adv), stats[7] = sum of squared deviations, and
 * stats[0..4] as dxrl_pg_adv_combine(stats + 5, world = 1) would (single rank: no second call)
 * (per-env sums about the env's own first value, merged with Chan et al.'s pairwise update
 * in a fixed order: no sum(a^2) - mean sum(a) cancellation).
 * The recurrence is A_t = delta_t + (gamma lambda)(1 - d_t) A_{t+1} per env:
 *   T <= 600 (~256 B per step in LDS, <= 152 KiB): k_gae_lds -- a 256-thread workgroup per 16
 *     envs stages the horizon in LDS with all its threads (delta_t and the chain coefficient
 *     computed in parallel), runs the recurrence as a wavefront-prefix scan (16 lanes per env:
 *     each lane's segment of 8-step chunks composed into an affine map, a suffix scan of the maps
 *     across the 16 lanes, each segment rerun from its incoming value), all threads store
 *     adv / ret; ceil(N / 16) workgroups.  Bit-exact against tests/pg_reference.py's restatement
 *     of that order; within ~1e-6 of the values' scale of the one-chain loop;
 *   longer horizons: k_gae -- one thread per env running the sequential loop, 64-env workgroups;
 *     ceil(N / 64) workgroups.
 * Each workgroup writes one (count, mean, M2) triple into `partial`.
 * partial: f64 [dxrl_pg_gae_partial_doubles(N, T)] (= 3 ceil(N / 16), enough for either kernel);
 * stats: f64 [8]. */
int dxrl_pg_gae(int32_t device, const float* rew, const uint8_t* done, const float* values, int64_t num_envs,
                int64_t horizon, double gamma, double lam, float* adv, float* ret, double* partial, double* stats,
                void* stream);
/* f64 elements of dxrl_pg_gae's `partial` scratch for (num_envs, horizon) (host-only query). */
int dxrl_pg_gae_partial_doubles(int64_t num_envs, int64_t horizon, int64_t* doubles);
/* Global advantage statistics from every rank's (count, mean, M2) triple -- moments f64
 * [world][3] in rank order (all-gathered stats[5..7]) -- merged in rank order into
 * stats[0] count, [1] sum, [2] mean, [3] sum of squared deviations, [4] unbiased std (what the
 * train passes read: (adv - [2]) / ([4] + 1e-8)). */
int dxrl_pg_adv_combine(int32_t device, const double* moments, int32_t world, double* stats, void* stream);
/* One rank: dxrl_pg_adv_combine(stats + 5, world = 1).  phase must be 2; adv / count /
 * partial are unused (kept for ABI stability). */
int dxrl_pg_adv_finalize(int32_t device, int32_t phase, const float* adv, int64_t count, double* partial,
                         double* stats, void* stream);

/* ------------------------------------------------------------------------
 * Curriculum-scheduler feed (config C3; replaces the per-episode
 * CurriculumScheduler.update() calls of evaluation/component_ablation.py:160-170,
 * experiments/curriculum_scheduler.py:116-170 for a vectorised iteration).
 * Walks the rollout's episode-end codes (dxrl_pg_rollout_args.ep_code) of all
 * ranks in (end step, global env id) order and reports what the host scheduler
 * needs to replay the batch exactly.
 * ------------------------------------------------------------------------ */
#define DXRL_SCHED_MAX_CANDIDATES 64
typedef struct dxrl_sched_args {
    const uint16_t* codes;     /* u16 [world][T][N] episode-end codes, rank-major (all-gathered) */
    int32_t world, horizon;    /* ranks, T                                                 */
    int64_t num_envs;          /* N per rank                                               */
    int32_t window;            /* window_size (>= 1)                                       */
    int32_t max_candidates;    /* P <= DXRL_SCHED_MAX_CANDIDATES progressions still possible */
    double threshold;          /* success_rate_threshold                                   */
    int64_t min_episodes;      /* min_episodes_before_progression                          */
    int64_t episodes_before;   /* total_episodes before this batch (== len(episode_successes)) */
    const uint16_t* tail_in;   /* u16 [window] codes of the last tail_len_in episodes, oldest first */
    const int32_t* tail_len_in;   /* i32 [1] (device)                                      */
    uint16_t* tail_out;        /* u16 [window] the new tail (must not alias tail_in)       */
    int32_t* tail_len_out;     /* i32 [1] (device)                                         */
    void* scratch;             /* device scratch of dxrl_sched_scratch_bytes()             */
    int64_t scratch_bytes;
    int64_t* summary;          /* i64 [4 + 3 P] (device): [0] episodes, [1] steps, [2] successes,
                                  [3] candidates found (<= P), then per candidate in episode order:
                                  episode index k in the batch, steps through k, successes among
                                  the window ending at k                                        */
} dxrl_sched_args;
int dxrl_sched_scratch_bytes(int32_t world, int32_t horizon, int64_t num_envs, int32_t window, int64_t* bytes);
int dxrl_sched_scan(int32_t device, const dxrl_sched_args* args, void* stream);

/* The same feed with a compacted exchange between ranks (what a sharded run all-gathers instead
 * of the world x T x N codes).  Each rank packs its own codes [T][N]:
 *   header (episodes, tail length), per-step (episodes, steps, successes), its last `window`
 *   codes, and -- only while progressions are still possible (bits = 1) -- one success bit
 *   per episode;
 * = 4 (2 + 3 T + window / 2) bytes, + T N / 8 with bits.  The ranks all-gather the packs,
 * dxrl_sched_scan_packed walks them in (end step, global env id) order exactly as
 * dxrl_sched_scan walks the codes, and reports every candidate's steps only through the start
 * of its (step, rank) block plus where it lies (`where`); the owning rank adds the steps inside
 * the block (dxrl_sched_candidate_steps -> i64 [P], zero for others), the ranks SUM those P
 * values (all-reduce) and dxrl_sched_finish adds them into the summary.  The summary / tail
 * equal dxrl_sched_scan's on the all-gathered codes. */
int dxrl_sched_pack_words(int32_t horizon, int64_t num_envs, int32_t window, int32_t bits, int64_t* words);
int dxrl_sched_pack(int32_t device, const uint16_t* codes, int32_t horizon, int64_t num_envs, int32_t window,
                    int32_t bits, uint32_t* pack, void* stream);
typedef struct dxrl_sched_packed_args {
    const void* packs;         /* u32 [world][pack_words] all-gathered packs, rank order  */
    int64_t pack_words;        /* dxrl_sched_pack_words(horizon, num_envs, window, bits)  */
    int32_t bits;              /* the packs carry success bits (needed when max_candidates > 0) */
    int32_t world, horizon;
    int64_t num_envs;          /* N per rank                                              */
    int32_t window, max_candidates;
    double threshold;
    int64_t min_episodes, episodes_before;
    const uint16_t* tail_in;   /* as dxrl_sched_args                                      */
    const int32_t* tail_len_in;
    uint16_t* tail_out;
    int32_t* tail_len_out;
    void* scratch;             /* dxrl_sched_packed_scratch_bytes()                       */
    int64_t scratch_bytes;
    int64_t* summary;          /* as dxrl_sched_args (candidate steps: block prefix until finished) */
    int32_t* where;            /* i32 [P][3] per candidate: owning rank, end step, index in its block */
} dxrl_sched_packed_args;
int dxrl_sched_packed_scratch_bytes(int32_t world, int32_t horizon, int64_t num_envs, int32_t window,
                                    int64_t* bytes);
int dxrl_sched_scan_packed(int32_t device, const dxrl_sched_packed_args* args, void* stream);
int dxrl_sched_candidate_steps(int32_t device, const uint16_t* codes, int32_t horizon, int64_t num_envs,
                               int32_t rank, int32_t max_candidates, const int32_t* where, const int64_t* summary,
                               int64_t* partial, void* stream);
int dxrl_sched_finish(int32_t device, const int64_t* partial, int64_t* summary, void* stream);

typedef struct dxrl_pg_heads_args {
    const float* mu;           /* f32 [M][32] actor head output            */
    const float* values;       /* f32 [M] critic value                     */
    const float* act;          /* f32 [M][16]                              */
    const float* logp_old;     /* f32 [M]                                  */
    const float* adv;          /* f32 [M] raw GAE advantages               */
    const float* ret;          /* f32 [M] returns                          */
    const double* stats;       /* normalisation stats (mean [2], std [4])  */
    const float* params;       /* f32 master parameters (log_std)          */
    int64_t num_samples;       /* M (this rank)                            */
    double inv_total_samples;  /* 1 / (M summed over ranks)                */
    double clip_eps, vf_coef, ent_coef;
    void* dmu_rm;              /* bf16 [M][32]                             */
    void* dmu_fm;              /* bf16 [32][M]                             */
    void* dv_rm;               /* bf16 [M][32] (column 0)                  */
    void* dv_fm;               /* bf16 [32][M] (row 0)                     */
    float* dlogstd_partial;    /* f32 [ceil(M/256)][16]                    */
    double* loss_partial;      /* f64 [ceil(M/256)][4]                     */
    float* grads;              /* f32 master-layout gradients (log_std block written) */
} dxrl_pg_heads_args;

/* PPO-clip policy loss + value loss + entropy bonus: gradients at the heads. */
int dxrl_pg_heads(int32_t device, const dxrl_pg_heads_args* args, void* stream);
/* out[0] = sum(grads^2) (for global-norm clipping; all-reduce before Adam when sharded). */
int dxrl_pg_grad_sumsq(int32_t device, const float* grads, int64_t n, double* partial, double* out, void* stream);
int dxrl_pg_adam(int32_t device, float* params, const float* grads, float* m1, float* m2, int64_t n, double lr,
                 double beta1, double beta2, double eps, int64_t step, const double* gnorm2, double max_norm,
                 void* stream);
/* The whole optimiser step in two launches: grad-norm partials, then one kernel that finishes
 * the norm (k_sum_partials' order), applies clipped Adam (dxrl_pg_adam's arithmetic) and writes
 * the bf16 pack (dxrl_pg_pack_weights' layout) -- the updated master / moments go to the *_out
 * buffers (must not alias the inputs; the caller swaps the pairs).  n = dxrl_pg_sizes().params;
 * partial: f64 [512] scratch; gnorm2: f64 [1] (sum of squared grads, written). */
int dxrl_pg_optimizer_step(int32_t device, const float* params, const float* grads, const float* m1, const float* m2,
                           float* params_out, float* m1_out, float* m2_out, int64_t n, double lr, double beta1,
                           double beta2, double eps, int64_t step, double max_norm, double* partial, double* gnorm2,
                           void* packed, void* stream);
/* dxrl_pg_optimizer_step's second launch alone: the grad norm is finished from gnorm_blocks f64
 * partials the caller already holds (dxrl_pg_fused_pair_gnorm's, when one rank's reduction wrote
 * the whole gradient) instead of a k_sumsq pass over the gradient.  Same Adam / pack arithmetic;
 * the norm's f64 sum runs in another order, so it agrees with dxrl_pg_optimizer_step's to f64
 * rounding, not bit for bit.  New learner, no reference counterpart. */
int dxrl_pg_adam_step(int32_t device, const float* params, const float* grads, const float* m1, const float* m2,
                      float* params_out, float* m1_out, float* m2_out, int64_t n, double lr, double beta1, double beta2,
                      double eps, int64_t step, double max_norm, const double* gnorm_partial, int32_t gnorm_blocks,
                      double* gnorm2, void* packed, void* stream);

/* ---- fused one-pass learner step (csrc/dxrl_pg_fused.hip) ----------------------------
 * One launch per network replaces forward GEMMs + heads + backward GEMMs of the
 * layer-by-layer path (dxrl_gemm_bf16 / dxrl_pg_heads / dxrl_wgrad_bf16): per
 * 128-sample tile it runs the MLP forward, the PPO-clip (actor) or value (critic)
 * head and the backward pass out of LDS (db2 as fused column sums of dH2), then
 * dW2 = dH2^T H1 as one split-K contraction over dH2 (HBM).  H1 reaches it either
 * recomputed on chip from obs (h1_mode 0, rows % 32 == 0: no H1 traffic at all) or as
 * the h1 scratch copy this launch writes (h1_mode 1, or rows % 32 != 0).
 * train == 0 (critic only): forward pass writing values[rows] (GAE bootstrap pass). */
typedef struct dxrl_pg_fused_args {
    int32_t net;               /* 0 actor, 1 critic                                        */
    int32_t train;             /* 0 forward only (critic values), 1 forward + backward     */
    int64_t rows;              /* samples                                                  */
    const void* packed;        /* bf16 weight pack (dxrl_pg_pack_weights)                  */
    const float* params;       /* f32 master parameters (biases, log_std)                  */
    const void* obs;           /* bf16 [rows][64], column 45 = 1                           */
    const float* act;          /* actor: f32 [rows][16]                                    */
    const float* logp_old;     /* actor: f32 [rows]                                        */
    const float* adv;          /* actor: f32 [rows] raw GAE advantages                     */
    const float* ret;          /* critic: f32 [rows] returns                               */
    const double* stats;       /* actor: normalisation stats (mean [2], std [4])           */
    double inv_total_samples;  /* 1 / (samples summed over ranks)                          */
    double clip_eps, vf_coef, ent_coef;
    float* values;             /* forward mode: f32 [rows]                                 */
    void* h1;                  /* bf16 [rows][288] scratch (used by the H1 copy mode only)  */
    void* dh2;                 /* bf16 [rows][256] scratch                                 */
    float* partial;            /* f32 [grid + 17][dxrl_pg_fused_sizes().partial_floats]    */
    double* loss_partial;      /* f64 [grid][4]: actor writes 0,2,3, critic writes 1       */
    int32_t grid;              /* workgroups (one per CU: 256 on MI355X)                   */
    int32_t wgrad_splits;      /* split-K factor of the dW2 GEMM                           */
    float* wgrad_partial;      /* f32 [wgrad_splits + 16][256][288]                        */
    float* grads;              /* f32 master-layout gradients: W1/W2/W3 (+ log_std) blocks */
    int32_t h1_mode;           /* 0 recompute H1 for dW2 when rows % 32 == 0, 1 HBM copy    */
    /* Layer-2 activations computed once per weight version (round 6; both nullable):
       h2_out (forward mode): bf16 [rows][264] H2 of the critic, written by the values pass;
       h2_in (train mode): bf16 [rows][264] H2 of this net under the SAME weights -- the rollout's
       h2_tape for the actor, the values pass's h2_out for the critic -- read instead of
       recomputing layer 2 (bit-identical: same MFMA k order and tanh).  Columns 256..263 are
       padding (keep them finite, e.g. zero-initialised). */
    const void* h2_in;
    void* h2_out;
} dxrl_pg_fused_args;

int dxrl_pg_fused_sizes(int32_t* tile_rows, int64_t* partial_floats_per_block);
int dxrl_pg_fused(int32_t device, const dxrl_pg_fused_args* args, void* stream);
/* Both train passes of one learner step (a PPO minibatch, or the whole batch) with their
 * dW2 contractions in ONE k_wgrad_l1 launch (critic->wgrad_splits + actor->wgrad_splits
 * workgroups side by side) and every reduction of both networks in ONE launch.  Same
 * per-network arithmetic as two dxrl_pg_fused calls with those split counts; each pass needs
 * its own dh2 / partial / wgrad_partial buffers, h1_mode 0, rows % 32 == 0, splits > 16.
 * No reference counterpart (policies/simple_learner.py:73-95 is the update it replaces). */
int dxrl_pg_fused_pair(int32_t device, const dxrl_pg_fused_args* critic, const dxrl_pg_fused_args* actor,
                       void* stream);
/* dxrl_pg_fused_pair whose reduction also writes the global grad norm's partials: one f64 per
 * reduction block (*gnorm_blocks of them, dxrl_pg_gnorm_blocks(); gnorm_capacity >= that), each
 * the sum of squares of the gradient values the block stored.  The gradients are bit for bit
 * dxrl_pg_fused_pair's.  At one rank the pair writes the whole gradient, so
 * dxrl_pg_adam_step(gnorm_partial) replaces dxrl_pg_optimizer_step's k_sumsq launch; with a
 * gradient all-reduce in between, the partials are stale and the caller uses the latter. */
int dxrl_pg_fused_pair_gnorm(int32_t device, const dxrl_pg_fused_args* critic, const dxrl_pg_fused_args* actor,
                             double* gnorm_partial, int32_t gnorm_capacity, int32_t* gnorm_blocks, void* stream);
int dxrl_pg_gnorm_blocks(int32_t* blocks);

/* ------------------------------------------------------------------------
 * Evaluation episode programs:
 *   evaluation/evaluator.py:71-271      Evaluator.evaluate_episode / evaluate_heldout_set
 *   evaluation/robustness_tests.py:240-407 RobustnessTester.evaluate_with_noise / run_robustness_sweep
 * A LANE runs a chain of SEGMENTS back to back; a segment is one fresh env
 * instance (DexterousManipulationEnv(curriculum_config=row), so its first reset
 * draws the spawn position and later resets keep the object where it is,
 * manipulation_env.py:156-161), optionally wrapped in CombinedNoiseWrapper(obs
 * std, dyn std) (robustness_tests.py:140-211), running `num_episodes`
 * consecutive reset(seed) -> loop{select_action, step} episodes, each stopping
 * at terminated / truncated / max_steps with success = terminated
 * (evaluator.py:150-158, robustness_tests.py:288-303).  The policy is frozen
 * (evaluator.py:50-70: no update) and obs-independent, as every reference
 * policy is; its random stream runs on across the lane's segments, the noise
 * stream restarts with each segment's wrapper.
 *
 * Exact reference order = ONE lane whose segments are the driver's loop (the
 * global np.random stream is consumed serially); the vectorised form = one lane
 * per episode (or per noise level) with its own policy stream.
 * ------------------------------------------------------------------------ */
#define DXRL_EVAL_POLICY_SIMPLE 0    /* frozen SimpleLearner: clip(mean + f32(0 + s g), -1, 1)  (simple_learner.py:59-71) */
#define DXRL_EVAL_POLICY_HEURISTIC 1 /* clip(-0.5f + f32(-0.1 + 0.2 u), -1, 1)         (heuristic_policy.py:38-63) */
#define DXRL_EVAL_POLICY_RANDOM 2    /* Box.sample(): f32(-1 + 2 u)                     (random_policy.py:29-40)    */

typedef struct dxrl_eval_segment {
    int32_t curriculum_row;   /* row of the env's curriculum table                          */
    int32_t num_episodes;     /* consecutive episodes on this instance                      */
    int32_t first_episode;    /* record index of its first episode                           */
    int32_t reserved;
    double obs_noise_std;     /* wrapper observation noise (0 = off; consumes 45 normals per draw) */
    double dyn_noise_std;     /* wrapper dynamics noise (0 = off; 15 normals per step)       */
    int64_t noise_offset;     /* tape mode: first standard normal of this wrapper's stream    */
    int64_t noise_count;      /* tape mode: normals available from noise_offset               */
} dxrl_eval_segment;

typedef struct dxrl_eval_args {
    int32_t num_lanes;               /* <= env num_envs; lane i uses env slot i's weights    */
    int32_t policy;                  /* DXRL_EVAL_POLICY_*                                    */
    int32_t max_steps;               /* episode loop bound (evaluator.py:136)                */
    int32_t total_episodes;          /* record count (bounds check)                          */
    const int32_t* lane_segments;    /* device i32 [num_lanes + 1] CSR offsets into segments */
    const dxrl_eval_segment* segments; /* device                                            */
    const float* mean_action;        /* device f32 [num_lanes][15] (SIMPLE; NULL -> zeros)   */
    double exploration_noise;        /* SIMPLE sigma (simple_learner.py:28)                  */
    /* parity tapes (NULL -> device Philox streams) */
    const double* policy_tape;       /* f64 [num_lanes][policy_stride] raw draws: legacy gauss
                                        (SIMPLE) / next_double (HEURISTIC, RANDOM)           */
    int64_t policy_stride;
    const double* noise_tape;        /* f64 standard normals, addressed by segment offsets   */
    const double* reset_tape;        /* f64 [total_episodes][D+6] resolved reset draws       */
    uint64_t policy_seed, noise_seed, reset_seed; /* Philox keys of the device streams       */
    /* per-episode records [total_episodes] */
    double* ep_return;               /* episode_reward (f64, sequential sum)                 */
    int32_t* ep_length;              /* episode_steps                                        */
    uint8_t* ep_success;             /* terminated at the last step                          */
    uint8_t* ep_contacts;            /* num_contacts of the last step's info                 */
    uint8_t* contact_hist;           /* u8 [total_episodes][max_steps] per-step num_contacts
                                        (contact_history, evaluator.py:148-150; nullable)   */
    int32_t* policy_used;            /* i32 [num_lanes] policy draws consumed (nullable)     */
    int32_t* status;                 /* i32 [1] device error word: 1 = a tape ran out        */
    /* trajectories (nullable; failure_logger.py:242-297 EpisodeRecorder, evaluator.py:101-152):
       obs_traj f32 [total_episodes][max_steps + 1][45] -- the reset observation, then the
       observation after every step; act_traj f32 [total_episodes][max_steps][15] -- the policy's
       action of every step.  Rows past an episode's length are left untouched. */
    float* obs_traj;
    float* act_traj;
    /* device i32 [1] scratch owned by the caller: this launch's work-queue counter (zeroed on
       the stream by the call).  Required by the default (work-queue) kernel; give each launch
       that may run concurrently with another its own counter. */
    int32_t* work_queue;
} dxrl_eval_args;

int dxrl_evaluate(dxrl_env* env, const dxrl_eval_args* args, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DXRL_H_ */
