/*
 * salp.h — C ABI of the MI355X-native batched SALP simulator (libsalp.so).
 *
 * Drop-in boundary.  The reference (Avielstein/GRASP_LAB_SALP) exposes the hot
 * path only as Python objects:
 *
 *   SalpRobotEnv(render_mode, width, height, robot, num_obstacles, obstacle_radius)
 *       src/salp_robot_env.py:35          -> salp_create / SalpParams
 *   SalpRobotEnv.reset(seed, options) -> (obs, {})
 *       src/salp_robot_env.py:114-155     -> salp_reset / salp_reset_to
 *   SalpRobotEnv.step(action) -> (obs, reward, terminated, truncated, info)
 *       src/salp_robot_env.py:196-299     -> salp_step
 *   Robot(dry_mass, init_length, init_width, max_contraction, nozzle),
 *   Nozzle(length1, length2, length3, area, mass), Robot.set_environment,
 *   Nozzle.set_angles        src/robot.py:20-21, 261-262, 443-449, 50-60
 *                                         -> SalpParams fields
 *   Robot / Nozzle state attributes (src/robot.py:261-412)
 *                                         -> salp_get_state / salp_set_state
 *   SB3 VecEnv rollout collection around env.step (src/train_robot.py:26,
 *   src/train_robot_recurrent_ppo.py:65)  -> salp_rollout (rollout-buffer fill)
 *
 * The Python host layer (grasp_lab_salp_amd/) binds these with ctypes; the
 * reference-side binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every array argument is a caller-owned DEVICE pointer (e.g. a torch
 *    tensor's data_ptr()) on the handle's device; `stream` is a hipStream_t
 *    (NULL = the legacy default stream).  Calls only enqueue work: nothing
 *    synchronises and nothing allocates after salp_create.
 *  - Return value: 0 on success, a negative SALP_E* code on error; the
 *    message is available from salp_last_error(h) (h may be NULL for errors
 *    raised by salp_create).  No C++ exception crosses this boundary.
 *  - A handle is not thread-safe: one handle per GPU per process.
 *  - Physics is fp64 end to end (the reference is NumPy fp64); observations
 *    are float32 exactly as the reference returns them; rewards are fp64.
 */
#ifndef SALP_H
#define SALP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SALP_ABI_VERSION 13

#define SALP_MAX_OBSTACLES 4
#define SALP_OBS_DIM_MAX (6 + 2 * SALP_MAX_OBSTACLES)
/* info_out row: 7 reward components, 16 episode metrics, ep return, ep length,
 * has_metrics flag, terminal hit_obstacle flag (see SALP_INFO_* below). */
#define SALP_INFO_DIM 27

#define SALP_OK 0
#define SALP_EINVAL -1
#define SALP_EHIP -2
#define SALP_ENOMEM -3

/* Constructor arguments of the reference objects.  Constants that the
 * reference hard-codes (dt=0.01, drag/added-mass coefficients, the polynomial
 * cycle-time fits, masses of buoy/skin/tube) are not parameters there and are
 * not parameters here either. */
typedef struct SalpParams {
    /* Nozzle(length1, length2, length3, area, mass)   src/robot.py:20-21 */
    double nozzle_length1, nozzle_length2, nozzle_length3, nozzle_area, nozzle_mass;
    /* Robot(dry_mass, init_length, init_width, max_contraction, nozzle)
     *                                                  src/robot.py:261-262 */
    double dry_mass, init_length, init_width, max_contraction;
    /* Robot.set_environment(density)                  src/robot.py:443-449 */
    double density;
    /* Nozzle.set_angles(angle1, angle2) done by make_env before the env is
     * built (src/train_robot.py:16)                   src/robot.py:50-60 */
    double init_angle1, init_angle2;
    /* SalpRobotEnv(width, height, num_obstacles, obstacle_radius)
     *                                                  src/salp_robot_env.py:35 */
    double obstacle_radius;
    int32_t width, height, num_obstacles;
    int32_t max_cycles; /* timeout, hard-coded 500 at src/salp_robot_env.py:274 */
    /* Randomisation switches, all off in every reference script (0 = off):
     *   Robot.enable_dynamic_randomization  src/robot.py:436-438, 594-628
     *   Robot.enable_disturbances           src/robot.py:440-441, 796-800, 834-838
     *   SalpRobotEnv.enable_action_randomization / enable_observation_randomization /
     *   enable_latency                      src/salp_robot_env.py:157-194, 293-297
     * Draws come from the device Philox stream (grasp_lab_salp_amd/csrc/
     * salp_random.h), not NumPy's MT19937: distributional parity only. */
    int32_t dynamics_randomization, disturbances, action_randomization, observation_randomization,
        latency, reserved0;
} SalpParams;

typedef struct SalpEnv SalpEnv; /* opaque handle */

/* Rollout-buffer fill targets for salp_rollout (all device pointers, rows
 * indexed [slot][env], slot = completed-step counter of that env modulo
 * `capacity`).  Any pointer may be NULL to skip that output. */
typedef struct SalpRolloutBuffers {
    int64_t capacity;      /* slots per env                                  */
    float* obs;            /* [capacity][n_envs][obs_dim]  obs AFTER the step  */
    float* actions;        /* [capacity][n_envs][3]                            */
    float* rewards;        /* [capacity][n_envs]  (float32, SB3 buffer dtype)  */
    uint8_t* dones;        /* [capacity][n_envs]  bit0 terminated, bit1 truncated */
    int64_t* steps_done;   /* [n_envs] completed env-steps counter (in/out)    */
    int64_t max_steps;     /* >0: a lane starts no env-step once steps_done
                            * reaches it (fixed-length rollouts, n_steps)     */
    int32_t chunk;         /* ticks between env-step boundaries (0 = 64)      */
    int32_t reserved;
    float* obs_before;     /* [capacity][n_envs][obs_dim]  the observation the
                            * step's action was taken from (SB3 RolloutBuffer
                            * "obs"): the previous step's obs, or the reset obs
                            * after an episode end (ABI 4)                     */
} SalpRolloutBuffers;

/* ------------------------------------------------------------ lifecycle */
int salp_abi_version(void);
void salp_default_params(SalpParams* p); /* canonical make_env config */
int salp_create(const SalpParams* p, int64_t n_envs, uint64_t seed, int64_t env_id_offset,
                int device, SalpEnv** out);
int salp_destroy(SalpEnv* h);
const char* salp_last_error(const SalpEnv* h);
int64_t salp_num_envs(const SalpEnv* h);
int salp_obs_dim(const SalpEnv* h);

/* -------------------------------------------------------------- env API */
/* reset(): per masked env (mask NULL = all) draw target + obstacles from the
 * env's Philox stream, Robot.reset(), episode trackers; writes obs rows of
 * masked envs.  obs_out [n_envs][obs_dim] (NULL allowed). */
int salp_reset(SalpEnv* h, const uint8_t* mask, float* obs_out, void* stream);
/* reset() with the target / obstacles given by the caller (the reference
 * draws them from the global np.random; parity tests inject them).
 * targets [n][2], obstacles [n][SALP_MAX_OBSTACLES][2], n_obstacles [n]. */
int salp_reset_to(SalpEnv* h, const uint8_t* mask, const float* targets, const float* obstacles,
                  const int32_t* n_obstacles, float* obs_out, void* stream);
/* One SalpRobotEnv.step per env (one breathing cycle each).
 * actions [n][3] float32 in the action box; outputs may be NULL.
 * auto_reset != 0: envs that end are reset (SB3 VecEnv semantics); their
 * obs_out row is then the reset observation and terminal_obs_out [n][obs_dim]
 * receives the final observation.  info_out [n][SALP_INFO_DIM] fp64. */
int salp_step(SalpEnv* h, const float* actions, float* obs_out, double* reward_out,
              uint8_t* terminated_out, uint8_t* truncated_out, int auto_reset,
              float* terminal_obs_out, double* info_out, void* stream);
/* Synthetic random-action rollout, chained per lane: every env runs up to
 * `tick_budget` physics ticks (dt=0.01 each) in chunks of buf->chunk ticks,
 * completing as many env-steps as fit, with actions ~ U(action box) from
 * Philox(seed; env id, step index) and auto-reset (Philox targets/obstacles).
 * Env-steps end and start only at chunk boundaries (a lane waits < chunk
 * ticks); a cycle cut by the budget resumes on the next call.  Per-env results
 * do not depend on how the work is split. */
int salp_rollout(SalpEnv* h, int64_t tick_budget, const SalpRolloutBuffers* buf, void* stream);
/* Same random actions, lock-step: every env performs exactly n_steps
 * env-steps (one full cycle each) with auto-reset.  rewards_out [n] = sum. */
int salp_step_random(SalpEnv* h, int32_t n_steps, double* reward_sum_out, void* stream);

/* ------------------------------------------------ policy-in-the-loop collection
 * PPO's collect_rollouts (stable-baselines3 OnPolicyAlgorithm.collect_rollouts,
 * around the env.step calls of the reference's on-policy learner,
 * src/train_robot_recurrent_ppo.py:65, 85-107) inside the chained kernel: every env
 * runs `n_steps` env-steps back to back; at each env-step boundary the lane
 * evaluates the policy on the env's observation and draws its action there, so
 * no env waits for the slowest cycle of the batch between steps.
 *
 * Policy: SB3 MlpPolicy with net_arch pi=[64, 64], vf=[64, 64], tanh, a
 * state-independent log_std (diagonal Gaussian).  float32 weights packed in
 * one array (torch nn.Linear weights are [out][in]; the first layer's input
 * columns are zero-padded to SALP_OBS_DIM_MAX), offsets in floats:          */
#define SALP_POLICY_HIDDEN 64
#define SALP_POLICY_PI_W1 0
#define SALP_POLICY_PI_B1 (SALP_POLICY_PI_W1 + SALP_POLICY_HIDDEN * SALP_OBS_DIM_MAX)
#define SALP_POLICY_PI_W2 (SALP_POLICY_PI_B1 + SALP_POLICY_HIDDEN)
#define SALP_POLICY_PI_B2 (SALP_POLICY_PI_W2 + SALP_POLICY_HIDDEN * SALP_POLICY_HIDDEN)
#define SALP_POLICY_ACT_W (SALP_POLICY_PI_B2 + SALP_POLICY_HIDDEN)       /* [3][64] */
#define SALP_POLICY_ACT_B (SALP_POLICY_ACT_W + 3 * SALP_POLICY_HIDDEN)   /* [3] */
#define SALP_POLICY_LOG_STD (SALP_POLICY_ACT_B + 3)                     /* [3] */
#define SALP_POLICY_VF_W1 (SALP_POLICY_LOG_STD + 3)
#define SALP_POLICY_VF_B1 (SALP_POLICY_VF_W1 + SALP_POLICY_HIDDEN * SALP_OBS_DIM_MAX)
#define SALP_POLICY_VF_W2 (SALP_POLICY_VF_B1 + SALP_POLICY_HIDDEN)
#define SALP_POLICY_VF_B2 (SALP_POLICY_VF_W2 + SALP_POLICY_HIDDEN * SALP_POLICY_HIDDEN)
#define SALP_POLICY_VAL_W (SALP_POLICY_VF_B2 + SALP_POLICY_HIDDEN)       /* [1][64] */
#define SALP_POLICY_VAL_B (SALP_POLICY_VAL_W + SALP_POLICY_HIDDEN)       /* [1] */
#define SALP_POLICY_SIZE (SALP_POLICY_VAL_B + 1)

/* Per env-step of env i, row t (its t-th step of this call):
 *   obs[t][i]      the observation the action is taken on;
 *   actions[t][i]  a = mean + exp(log_std) * z, z ~ N(0, 1) from
 *                  Philox(noise_seed; global env id, step counter); the env
 *                  receives clamp(a, Box low, Box high) (SB3 clips, buffers a);
 *   values, log_probs: V(obs), log N(a; mean, std) summed over the 3 dims;
 *   episode_starts[t][i]: 1 if obs starts an episode (in: episode_start[i]);
 *   rewards[t][i]  float32 reward; + gamma * V(terminal obs) where the episode
 *                  was truncated, not terminated (SB3's timeout bootstrap);
 *                  0 and a fresh episode where the divergence guard fires
 *                  (|obs| > diverged_obs_abs, |reward| > diverged_reward_abs or
 *                  non-finite; guard off when diverged_obs_abs <= 0);
 * last_obs[i] is in/out: on entry the observation env i's first step of this
 * call is taken on (the reset observation, or the previous call's last_obs);
 * on return episode_start[i] (next step starts an episode) and last_obs[i]
 * (the obs after the last step, the reset obs where it ended an episode).
 * ep_stats[0..3] += (return, 1, target reached (terminated), length) per
 * episode that ended by the task's rules;
 * diverged[0] += envs reset by the guard. */
typedef struct SalpPolicyRollout {
    const float* weights;  /* [SALP_POLICY_SIZE] */
    uint64_t noise_seed;
    double gamma;
    double diverged_obs_abs;
    double diverged_reward_abs;
    int64_t n_steps;
    float* obs;            /* [n_steps][n_envs][obs_dim] */
    float* actions;        /* [n_steps][n_envs][3]        */
    float* rewards;        /* [n_steps][n_envs]           */
    float* episode_starts; /* [n_steps][n_envs]           */
    float* values;         /* [n_steps][n_envs]           */
    float* log_probs;      /* [n_steps][n_envs]           */
    float* episode_start;  /* [n_envs] in/out             */
    float* last_obs;       /* [n_envs][obs_dim] in/out    */
    double* ep_stats;      /* [4] accumulated             */
    int64_t* diverged;     /* [1] accumulated             */
} SalpPolicyRollout;
int salp_collect(SalpEnv* h, const SalpPolicyRollout* r, void* stream);

/* Launch order of the lock-step calls (salp_step, salp_step_random): a
 * launch lasts as long as its slowest wave.  mode 1: envs run sorted by the
 * predicted length of the cycle each is about to run (longest first): the
 * waves of short cycles finish early, which lets the chip clock the long ones
 * higher, and beyond one wave per SIMD the rounds pack; 0: env order;
 * -1 (default): sorted from 1 024 envs on.  Results per env are identical in
 * every mode. */
int salp_set_lockstep_order(SalpEnv* h, int mode);

/* Kernel of the chained calls (salp_rollout, salp_collect, salp_step_random
 * from 32 env-steps on; ABI 9).  mode 0: one env per lane (k_rollout); 1: each
 * env on two waves that split its physics tick and meet once per tick through
 * LDS (k_rollout_pair: twice the waves, so an env count that leaves SIMDs idle
 * with one env per lane fills the chip); 2 (round 6): two waves per env with
 * the tick split along its one-way dependences, the B wave's angle chain
 * following the A wave's forces through an LDS ring (k_rollout_split);
 * -1 (default): a two-wave kernel while n_envs <= 128 x compute units.  The
 * two-wave kernels have no randomised instance: with a randomisation switch
 * on the chained calls use k_rollout.  Results per env are identical in every
 * mode. */
int salp_set_rollout_kernel(SalpEnv* h, int mode);
/* Partner waits of k_rollout_pair that gave up (ABI 10): the two waves of an
 * env meet once per tick; a wave that polls for its partner ~56 ms in vain
 * stops waiting, so that the kernel always ends, and that env's results of the
 * launch are then invalid.  Reads (synchronising `stream`) and clears the
 * count of such waits since the previous call, over every launch of the
 * process; 0 is the only good answer (the Python layer raises otherwise).
 * k_step_wave (salp_step) also marks such an env invalid in place: its motion
 * state is set to NaN, the state of a diverged env, so a caller that never
 * reads this count still cannot take the unfinished cycle for a result.
 * Diagnostic with no reference counterpart. */
int salp_pair_timeouts(SalpEnv* h, uint64_t* count_out, void* stream);
/* Kernel of salp_step (ABI 11): -1 auto (default), 0 one env per lane
 * (k_step, lock-step), 1 one env per wave (k_step_wave: the wave's lanes
 * compute the geometry of 64 ticks at once, then run their dynamics; a cycle's
 * latency drops to about its steady ticks').  Auto: one env per wave up to
 * 1 024 envs (the per-env SalpRobotEnv.step, src/salp_robot_env.py:196-299,
 * and small vector envs).  Recording (salp_set_trace) always uses k_step.
 * Results per env are identical in every mode.  No reference counterpart. */
int salp_set_step_kernel(SalpEnv* h, int mode);

/* GAE / returns over a rollout buffer: stable_baselines3's
 * RolloutBuffer.compute_returns_and_advantage (stable-baselines3 >= 2.0,
 * requirements.txt:6-7), which RecurrentPPO runs with gamma 0.99 and
 * gae_lambda 0.95 (src/train_robot_recurrent_ppo.py:94-95).  All buffers are
 * float32 device arrays, [n_steps][n_envs] row-major as in SB3:
 * rewards, values, episode_starts (1.0 where the step began an episode);
 * last_values / last_dones [n_envs] are the value estimate and done flag after
 * the last step.  Outputs advantages, returns [n_steps][n_envs].  Float32 with
 * SB3's operation order and NumPy 2 promotion (float32(gamma),
 * float32(gamma * gae_lambda)): bit-identical to the NumPy code. */
int salp_gae(int64_t n_steps, int64_t n_envs, const float* rewards, const float* values,
             const float* episode_starts, const float* last_values, const float* last_dones,
             double gamma, double gae_lambda, float* advantages, float* returns, void* stream);

/* Fused PPO loss head (stable_baselines3 PPO.train's clipped surrogate, value
 * MSE and entropy for a diagonal Gaussian with state-independent log-std) and
 * its gradient, for one minibatch of B rows.  Device float32 arrays: mu [B][3]
 * (policy mean), log_std [3], value [B], actions [B][3], old_logp [B],
 * advantages [B], returns [B].  normalize_advantage: SB3's per-minibatch
 * (adv - mean) / (std + 1e-8).  workspace: SALP_PPO_WORKSPACE_DOUBLES doubles.
 * Outputs: out [8] = loss, pg_loss, vf_loss, entropy, clip_fraction,
 * d loss / d log_std [3]; dmu [B][3] = d loss / d mu; dvalue [B] = d loss /
 * d value.  Float32 row math with fp64 sums (agrees with the torch expression
 * to float32 rounding).  Not part of the reference's API: it is the loss of
 * the SB3 learner the reference trains with (grasp_lab_salp_amd/ppo.py). */
#define SALP_PPO_WORKSPACE_DOUBLES 2048
int salp_ppo_loss(int64_t batch, const float* mu, const float* log_std, const float* value,
                  const float* actions, const float* old_logp, const float* advantages, const float* returns,
                  double clip_range, double ent_coef, double vf_coef, int normalize_advantage,
                  double* workspace, float* out, float* dmu, float* dvalue, void* stream);

/* One PPO minibatch step of the built-in MlpPolicy, fused (stable_baselines3
 * PPO.train's inner loop for SB3's MlpPolicy with net_arch pi = vf = [64, 64],
 * tanh: forward, the loss of salp_ppo_loss, backward, clip_grad_norm_, Adam).
 * The policy's tensors, torch.nn.Linear row-major [out][in], in this order
 * (obs_dim D <= SALP_OBS_DIM_MAX): */
enum SalpMlpTensor {
    SALP_MLP_PI_W1,   /* [64][D] */
    SALP_MLP_PI_B1,   /* [64]    */
    SALP_MLP_PI_W2,   /* [64][64] */
    SALP_MLP_PI_B2,   /* [64]    */
    SALP_MLP_ACT_W,   /* [3][64] action mean head */
    SALP_MLP_ACT_B,   /* [3]     */
    SALP_MLP_LOG_STD, /* [3]     */
    SALP_MLP_VF_W1,   /* [64][D] */
    SALP_MLP_VF_B1,   /* [64]    */
    SALP_MLP_VF_W2,   /* [64][64] */
    SALP_MLP_VF_B2,   /* [64]    */
    SALP_MLP_VAL_W,   /* [1][64] value head */
    SALP_MLP_VAL_B,   /* [1]     */
    SALP_MLP_N_TENSORS
};
/* The flat gradient / Adam-state vectors hold the tensors back to back in
 * that order: salp_ppo_mlp_offset(D, t) floats in, salp_ppo_mlp_num_params(D)
 * in all. */
int64_t salp_ppo_mlp_num_params(int obs_dim);
int64_t salp_ppo_mlp_offset(int obs_dim, int tensor);
int64_t salp_ppo_mlp_workspace_doubles(int64_t batch, int obs_dim);
/* Gradient of the loss over rows idx[0..batch) of the rollout buffer
 * (obs [N][D], actions [N][3], old_log_prob, advantages, returns [N]) into
 * grads (flat, overwritten); stats [4] += pg_loss, vf_loss, entropy,
 * clip_fraction.  Deterministic (no atomics), float32 rows, fp64 sums. */
typedef struct SalpPpoMinibatch {
    int64_t batch;
    int32_t obs_dim;
    int32_t normalize_advantage;
    const int64_t* idx;
    const float* obs;
    const float* actions;
    const float* old_log_prob;
    const float* advantages;
    const float* returns;
    float* params[SALP_MLP_N_TENSORS];
    float* grads;
    double clip_range;
    double ent_coef;
    double vf_coef;
    double* workspace;     /* salp_ppo_mlp_workspace_doubles(batch, obs_dim) */
    float* stats;          /* [4] accumulated, or NULL */
    const double* adv_part; /* ABI 12: this minibatch's advantage partials from
                               salp_ppo_mlp_adv_partials, or NULL (computed here) */
    double* norm_part;     /* ABI 13: or NULL.  The squared norm's partials of the final gradient (one per
                              64 parameters), written by the reduction: pass SalpPpoAdam.workspace here and
                              set SalpPpoAdam.norm_ready when nothing changes grads between the two calls
                              (one rank; a multi-GPU learner's all-reduce does) */
} SalpPpoMinibatch;
int salp_ppo_mlp_grads(const SalpPpoMinibatch* m, void* stream);
/* The advantage normalisation's partial sums (sum, sum of squares in fp64;
 * SALP_PPO_ADV_PARTIAL_DOUBLES per minibatch) of n_minibatches consecutive
 * minibatches of `batch` rows each (minibatch k: idx[k * batch ...]), in one
 * launch, exactly as salp_ppo_mlp_grads computes them for one minibatch; pass
 * out + k * SALP_PPO_ADV_PARTIAL_DOUBLES as minibatch k's adv_part (ABI 12:
 * one launch per epoch instead of one per minibatch).  No reference
 * counterpart (SB3 PPO.train's advantage normalisation). */
#define SALP_PPO_ADV_PARTIAL_DOUBLES 512
int salp_ppo_mlp_adv_partials(int64_t batch, int64_t n_minibatches, const int64_t* idx, const float* advantages,
                              double* out, void* stream);
/* clip_grad_norm_(max_grad_norm; <= 0: no clipping) of the flat gradient,
 * then torch.optim.Adam (no weight decay / amsgrad) on the tensors; exp_avg
 * and exp_avg_sq are flat like grads, step [1] is Adam's step count (float32,
 * incremented here), grad_norm [1] (or NULL) receives the pre-clip norm.  A
 * multi-GPU learner all-reduces grads between the two calls. */
typedef struct SalpPpoAdam {
    int32_t obs_dim;
    int32_t norm_ready;    /* ABI 13: 1 = workspace already holds the norm partials of grads
                              (SalpPpoMinibatch.norm_part); 0 = computed here (k_mlp_norm) */
    float* params[SALP_MLP_N_TENSORS];
    const float* grads;
    float* exp_avg;
    float* exp_avg_sq;
    float* step;
    float* grad_norm;
    double lr;
    double beta1;
    double beta2;
    double eps;
    double max_grad_norm;
    double* workspace;     /* ABI 13: SALP_PPO_APPLY_WORKSPACE_DOUBLES, zero-filled once by the caller and
                              then left to these calls (the norm's partials and a block-arrival count):
                              clip + Adam run over many blocks (k_mlp_adam, after k_mlp_norm unless
                              norm_ready); NULL: one block does both (k_mlp_apply) */
} SalpPpoAdam;
#define SALP_PPO_APPLY_WORKSPACE_DOUBLES 256
int salp_ppo_mlp_apply(const SalpPpoAdam* a, void* stream);

/* The LSTM cell of RecurrentPPO's MlpLstmPolicy (sb3-contrib RecurrentPPO,
 * src/train_robot_recurrent_ppo.py:85-107; grasp_lab_salp_amd/recurrent_ppo.py),
 * elementwise part of one torch.nn.LSTM step with sb3-contrib's episode-start
 * reset: gates [rows][4 hidden] = x W_ih^T + b + (h keep) W_hh^T (i, f, g, o),
 * c_prev [rows][hidden], keep [rows] (1 - episode_start);
 * c = sigmoid(f) c_prev keep + sigmoid(i) tanh(g), h = sigmoid(o) tanh(c);
 * act [rows][4 hidden] receives the activated gates for the backward, which
 * turns dh (and dc, or NULL) into dgates and dc_prev.  float32, caller's
 * stream; not part of the reference's own API (its learner is sb3-contrib). */
int salp_lstm_cell_forward(int64_t rows, int32_t hidden, const float* gates, const float* c_prev, const float* keep,
                           float* h, float* c, float* act, void* stream);
int salp_lstm_cell_backward(int64_t rows, int32_t hidden, const float* act, const float* c_prev, const float* keep,
                            const float* c, const float* dh, const float* dc, float* dgates, float* dc_prev,
                            void* stream);
/* One step of a whole-sequence pass (the training pass of both LSTMs,
 * recurrent_ppo._LSTMPairSeqFn).  Forward: the cell of gates + gx (gx, the
 * input projection with the bias, may be NULL), and hk_next = h keep_next (the
 * next step's recurrent GEMM operand; keep_next and hk_next both NULL or
 * both set).  Backward: the cell's backward for dh = d_out + dhk_next keep_next
 * (dhk_next = d hk_next; dhk_next and keep_next both NULL or both set). */
int salp_lstm_step_forward(int64_t rows, int32_t hidden, const float* gates, const float* gx, const float* c_prev,
                           const float* keep, const float* keep_next, float* h, float* c, float* act, float* hk_next,
                           void* stream);
int salp_lstm_step_backward(int64_t rows, int32_t hidden, const float* act, const float* c_prev, const float* keep,
                            const float* c, const float* d_out, const float* dhk_next, const float* keep_next,
                            const float* dc, float* dgates, float* dc_prev, void* stream);

/* ------------------------------------------------ Robot / Nozzle level */
/* The reference's Robot API for callers that drive the robot directly,
 * without the task env (src/compare_trajectories.py:120-168,
 * src/robot.py:1103-1158): per env, in the reference's call order
 *   nozzle.set_yaw_angle(yaw); nozzle.solve_angles()   -> salp_nozzle_solve
 *   robot.set_control(contraction, coast_time, angles)  -> salp_robot_set_control
 *   robot.step_through_cycle()                          -> salp_robot_step_through_cycle
 * Python floats are float64; the *_f32 flags say that the argument is an
 * np.float32 instead (NumPy 2 then computes some of the geometry in float32,
 * as on the env path).  All arrays are device pointers with n_envs rows. */
/* Robot.reset() (src/robot.py:452-501); mask NULL = all envs */
int salp_robot_reset(SalpEnv* h, const uint8_t* mask, void* stream);
/* Nozzle.set_angles(angle1, angle2) (src/robot.py:50-60); angles [n][2] */
int salp_nozzle_set_angles(SalpEnv* h, const double* angles, void* stream);
/* Nozzle.set_yaw_angle(yaw) + Nozzle.solve_angles() (src/robot.py:62-98); yaw [n] */
int salp_nozzle_solve(SalpEnv* h, const double* yaw, int yaw_is_f32, void* stream);
/* Robot.set_control(contraction, coast_time, [angle1, angle2])
 * (src/robot.py:544-592); control [n][4] */
int salp_robot_set_control(SalpEnv* h, const double* control, int contraction_is_f32, void* stream);
/* Robot.step_through_cycle() (src/robot.py:740-777) */
int salp_robot_step_through_cycle(SalpEnv* h, void* stream);

/* Per-tick history recording (Robot.enable_history_recording, record=True:
 * the *_history lists of src/robot.py:687-738).  While a trace buffer is set,
 * salp_step and salp_robot_step_through_cycle write, for every env, sample 0
 * (the state before the cycle's first tick) and one sample per tick:
 *   rows[(t * SALP_TRACE_DIM + col) * n_envs + env],  t < max_samples
 * n_samples[env] receives the number of samples of the last cycle (ticks + 1;
 * more than max_samples means the tail was not recorded).  Force columns of
 * sample 0 are NaN (the reference's force histories are one shorter), and so
 * are its euler_angle_rate and nozzle_yaw (there the reference holds stale
 * values left by the previous cycle's last tick).  asymmetry_torque (always
 * [0, 0, 0.00*|v|] == 0) and position_front (= [length/2, 0, 0]) are not
 * recorded.  The bench paths (salp_rollout, salp_step_random) never record. */
typedef struct SalpTraceBuffer {
    int64_t max_samples;
    double* rows;          /* [max_samples][SALP_TRACE_DIM][n_envs] */
    int64_t* n_samples;    /* [n_envs] */
} SalpTraceBuffer;
/* buf NULL disables recording; the struct is copied, the arrays are not */
int salp_set_trace(SalpEnv* h, const SalpTraceBuffer* buf);

/* Switch the randomisation features of SalpParams on or off for subsequent
 * calls (the reference's enable_* methods can be called at any time). */
int salp_set_randomization(SalpEnv* h, int dynamics, int disturbances, int actions, int observations,
                           int latency);

/* --------------------------------------------------------- state access */
/* State is a struct-of-arrays of SALP_NUM_FIELDS fp64 rows of n_envs each:
 * state[field * n_envs + env].  Integer and float32 quantities are stored
 * exactly as doubles.  With every randomisation switch off the coefficient
 * fields hold the reference's means and the OU fields zero; the kernels then
 * use the constants and leave those fields alone, so a state written with
 * salp_set_state should keep them that way. */
int salp_num_fields(void);
const char* salp_field_name(int field);
int salp_trace_dim(void);   /* SALP_TRACE_DIM */
int salp_get_state(SalpEnv* h, double* state_out, void* stream);
int salp_set_state(SalpEnv* h, const double* state_in, void* stream);
/* Diagnostic: n_ticks physics ticks on every env with no env-step boundaries
 * (a cycle that ends simply continues in REST); times the tick body alone.
 * Leaves the envs in a state no reference call sequence produces. */
int salp_bench_ticks(SalpEnv* h, int32_t n_ticks, void* stream);
/* Device address of the handle's state buffer.  Its layout is internal
 * (field-major rows plus an env-major block of the fields only env-step
 * boundaries touch, grasp_lab_salp_amd/csrc/salp_device.h "state layout");
 * use salp_get_state / salp_set_state for the field-major view. */
int64_t salp_state_ptr(SalpEnv* h);
/* Device-side self-test of salp_math.h: out[r * n + i] for the rows
 * {0 sin, 1 cos, 2 tan, 3 atan2(x, y), 4 asin, 5 acos, 6 cube, 7 np_cosf,
 * 8 np_sinf, 9-10 sin and cos of the branch-free sincos, 11 x / y by the
 * tick's shared-reciprocal division, 12-13 sin and cos of the tick's yaw
 * function, 14-17 sin x, cos x, sin y, cos y of the tick's roll / pitch pair
 * function at (x, y), 18-20 the tick's world-frame rotation of (y, x, 1) by
 * the angles (x, y, x + y), 21 atan (select form), 22 atan (fdlibm's branches)},
 * x, y [n]; out [SALP_MATH_SELFTEST_ROWS][n]. */
#define SALP_MATH_SELFTEST_ROWS 23
int salp_math_selftest(const double* x, const double* y, int64_t n, double* out, void* stream);

/* State fields.  Names follow the reference attribute they hold. */
enum SalpField {
    /* Robot vectors (src/robot.py:358-374), body frame unless noted */
    SALP_F_V0 = 0, SALP_F_V1, SALP_F_V2,                  /* velocity */
    SALP_F_W0, SALP_F_W1, SALP_F_W2,                      /* angular_velocity */
    SALP_F_ACC0, SALP_F_ACC1, SALP_F_ACC2,                /* acceleration */
    SALP_F_ALPHA0, SALP_F_ALPHA1, SALP_F_ALPHA2,          /* angular_acceleration */
    SALP_F_ETA0, SALP_F_ETA1, SALP_F_ETA2,                /* euler_angle (world) */
    SALP_F_PW0, SALP_F_PW1, SALP_F_PW2,                   /* position_world */
    SALP_F_POS0, SALP_F_POS1, SALP_F_POS2,                /* position */
    SALP_F_ANG0, SALP_F_ANG1, SALP_F_ANG2,                /* angle */
    SALP_F_PPOS0, SALP_F_PPOS1, SALP_F_PPOS2,             /* prev_position */
    SALP_F_PANG0, SALP_F_PANG1, SALP_F_PANG2,             /* prev_angle */
    SALP_F_AVGV0, SALP_F_AVGV1, SALP_F_AVGV2,             /* avg_cycle_velocity */
    SALP_F_AVGW0, SALP_F_AVGW1, SALP_F_AVGW2,             /* avg_cycle_angular_velocity */
    /* body geometry / mass properties (src/robot.py:325-339) */
    SALP_F_LENGTH, SALP_F_WIDTH, SALP_F_VOLUME, SALP_F_PREV_VOLUME,
    SALP_F_COM, SALP_F_COM_RATE, SALP_F_COM_ACC,          /* x components (y,z == 0) */
    SALP_F_PREV_I0, SALP_F_PREV_I1, SALP_F_PREV_I2,       /* diag(prev_I) */
    /* NumPy dtype of length/width/volume (1 = np.float32, see DESIGN.md
     * §NEP 50) and of prev_water_volume */
    SALP_F_GEOM32, SALP_F_PVOL32,
    /* cycle (src/robot.py:311-322) */
    SALP_F_CYCLE_TIME, SALP_F_TIME, SALP_F_REFILL_TIME, SALP_F_JET_TIME, SALP_F_COAST_TIME,
    SALP_F_CONTRACTION, SALP_F_CONTRACT_RATE, SALP_F_RELEASE_RATE, SALP_F_PHASE, SALP_F_CYCLE,
    /* 1 if `contraction` is an np.float32 (always on the env path, where it
     * comes from the float32 action; 0 for a Python float passed to
     * Robot.set_control): selects float32 vs float64 body geometry */
    SALP_F_CONTR32,
    /* nozzle (src/robot.py:30-44) */
    SALP_F_ANGLE1, SALP_F_ANGLE2, SALP_F_PREV_ANGLE1, SALP_F_PREV_ANGLE2,
    SALP_F_YAW, SALP_F_PREV_YAW, SALP_F_TURN_TIME,
    /* env (src/salp_robot_env.py:114-155) */
    SALP_F_TARGET0, SALP_F_TARGET1,
    SALP_F_OBST0, SALP_F_OBST_END = SALP_F_OBST0 + 2 * SALP_MAX_OBSTACLES - 1,
    SALP_F_N_OBST, SALP_F_PREV_DIST, SALP_F_PREV_A2,
    /* episode trackers (src/salp_robot_env.py:145-153, 399-447) */
    SALP_F_EP_LEN, SALP_F_EP_RETURN, SALP_F_PATH_LEN, SALP_F_LAST_PX, SALP_F_LAST_PY,
    SALP_F_SUM_A0, SALP_F_SUM_A1, SALP_F_SUM_ABS_A2, SALP_F_SUM_VEL, SALP_F_INIT_DIST,
    SALP_F_SUM_R0, SALP_F_SUM_R_END = SALP_F_SUM_R0 + 6,
    /* in-flight env-step (action of the cycle being simulated) + RNG counters */
    SALP_F_ACT0, SALP_F_ACT1, SALP_F_ACT2, SALP_F_PENDING,
    SALP_F_STEP_COUNT, SALP_F_EPISODE,
    /* coefficients of the current cycle (src/robot.py:300-306 means, or the
     * Robot._randomize_parameters draw): discharge coefficient, drag force /
     * torque ratios, diag of the added-mass (rate) coefficient matrices */
    SALP_F_CD, SALP_F_DFR, SALP_F_DTR,
    SALP_F_AMF0, SALP_F_AMF1, SALP_F_AMF2, SALP_F_AMRF0, SALP_F_AMRF1, SALP_F_AMRF2,
    SALP_F_AMT0, SALP_F_AMT1, SALP_F_AMT2, SALP_F_AMRT0, SALP_F_AMRT1, SALP_F_AMRT2,
    /* OUDisturbance states (force, torque) and the randomisation counters */
    SALP_F_OUF0, SALP_F_OUF1, SALP_F_OUF2, SALP_F_OUT0, SALP_F_OUT1, SALP_F_OUT2,
    SALP_F_RNG_CTL, SALP_F_RNG_TICK,
    SALP_NUM_FIELDS
};

/* info_out columns */
enum SalpInfo {
    SALP_INFO_R_TRACK = 0, SALP_INFO_R_HEADING, SALP_INFO_R_SMOOTH, SALP_INFO_R_YAW,
    SALP_INFO_R_TIME, SALP_INFO_R_SIDESLIP, SALP_INFO_R_OBSTACLE,
    SALP_INFO_PATH_LENGTH, SALP_INFO_DIRECT_DISTANCE, SALP_INFO_PATH_EFFICIENCY,
    SALP_INFO_FINAL_DISTANCE, SALP_INFO_INITIAL_DISTANCE, SALP_INFO_AVG_COMPRESSION,
    SALP_INFO_AVG_COAST_TIME, SALP_INFO_AVG_NOZZLE_ANGLE, SALP_INFO_AVG_VELOCITY,
    SALP_INFO_AVG_R_TRACK, SALP_INFO_AVG_R_HEADING, SALP_INFO_AVG_R_SMOOTH, SALP_INFO_AVG_R_YAW,
    SALP_INFO_AVG_R_TIME, SALP_INFO_AVG_R_SIDESLIP, SALP_INFO_AVG_R_OBSTACLE,
    SALP_INFO_EP_RETURN, SALP_INFO_EP_LEN, SALP_INFO_HAS_METRICS, SALP_INFO_HIT_OBSTACLE
};

/* trace columns (src/robot.py:687-738 history names without "_history") */
enum SalpTraceCol {
    SALP_T_STATE = 0,                                   /* phase value */
    SALP_T_PW0, SALP_T_PW1, SALP_T_PW2,                 /* position_world */
    SALP_T_V0, SALP_T_V1, SALP_T_V2,                    /* velocity */
    SALP_T_ACC0, SALP_T_ACC1, SALP_T_ACC2,              /* acceleration */
    SALP_T_ETA0, SALP_T_ETA1, SALP_T_ETA2,              /* euler_angle */
    SALP_T_ETAR0, SALP_T_ETAR1, SALP_T_ETAR2,           /* euler_angle_rate */
    SALP_T_W0, SALP_T_W1, SALP_T_W2,                    /* angular_velocity */
    SALP_T_ALPHA0, SALP_T_ALPHA1, SALP_T_ALPHA2,        /* angular_acceleration */
    SALP_T_LENGTH, SALP_T_WIDTH,
    SALP_T_AREA0, SALP_T_AREA1, SALP_T_AREA2,
    SALP_T_VOLUME, SALP_T_MASS, SALP_T_MASS_RATE,       /* mass[0,0], mass_rate[0,0] */
    SALP_T_NOZZLE_YAW,                                  /* nozzle.current_yaw */
    SALP_T_I0, SALP_T_I1, SALP_T_I2,                    /* inertia_tensor (diag) */
    SALP_T_TCD0, SALP_T_TCD1, SALP_T_TCD2,              /* trans_drag_coefficient */
    SALP_T_RCD0, SALP_T_RCD1, SALP_T_RCD2,              /* rot_drag_coefficient */
    SALP_T_COM, SALP_T_COM_RATE, SALP_T_COM_ACC,        /* x components (y, z == 0) */
    SALP_T_FRONT_W0, SALP_T_FRONT_W1, SALP_T_FRONT_W2,  /* position_front_world */
    /* force values (NaN in sample 0) */
    SALP_T_JETV0, SALP_T_JETV1, SALP_T_JETV2,           /* jet_velocity */
    SALP_T_JETF0, SALP_T_JETF1, SALP_T_JETF2,           /* jet_force */
    SALP_T_JETT0, SALP_T_JETT1, SALP_T_JETT2,           /* jet_torque */
    SALP_T_DRAGF0, SALP_T_DRAGF1, SALP_T_DRAGF2,        /* drag_force */
    SALP_T_DRAGT0, SALP_T_DRAGT1, SALP_T_DRAGT2,        /* drag_torque */
    SALP_T_CORF0, SALP_T_CORF1, SALP_T_CORF2,           /* coriolis_force */
    SALP_T_CORT0, SALP_T_CORT1, SALP_T_CORT2,           /* coriolis_torque */
    SALP_T_AMF0, SALP_T_AMF1, SALP_T_AMF2,              /* added_mass_force */
    SALP_T_AMT0, SALP_T_AMT1, SALP_T_AMT2,              /* added_mass_torque */
    SALP_T_DEFT0, SALP_T_DEFT1, SALP_T_DEFT2,           /* deform_torque */
    SALP_T_ACCF0, SALP_T_ACCF1, SALP_T_ACCF2,           /* acceleration_force */
    SALP_TRACE_DIM
};
#define SALP_T_FIRST_FORCE SALP_T_JETV0

#ifdef __cplusplus
}
#endif
#endif /* SALP_H */
