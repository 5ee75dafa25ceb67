/*
 * merlin_hip.h -- C ABI of libmerlin_hip.so, the MI355X (gfx950) hot path of
 * PPO-2DGrid ("MERLIN"): batched MiniGrid step/reset dynamics, the occluded
 * 7x7 egocentric observation, reward/done rules, the RGB tile expansion, and
 * GAE(lambda) + advantage normalisation.
 *
 * Conventions
 *   - Plain C types only; every device pointer is caller-allocated (e.g. a
 *     torch tensor's data_ptr()) and every call is stream-ordered on `stream`
 *     (a hipStream_t passed as void*; NULL = the null stream).  Calls marked
 *     [sync] synchronise that stream.
 *   - The env context owns only per-env state (grid bitmasks, agent, RNG,
 *     episode accumulators) in device memory.
 *   - Every entry point returns 0 (MERLIN_OK) or a MERLIN_E* code; nothing
 *     throws across the ABI.  merlin_last_error() gives a thread-local message.
 *   - Not re-entrant per context; one host thread per device.
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   merlin_env_create    gym.make(env_id, size=..) + wrapper chain
 *                        src/scenario_creator/scenario_creator.py:35-57,
 *                        BaseCustomEnv.__init__ src/custom_envs/base_env.py:15-41
 *   merlin_env_seed      gymnasium Env.reset(seed=s) -> seeding.np_random(s)
 *                        (ppo/ppo_train.py:48 `env.reset(seed=base_seed + ep)`)
 *   merlin_env_reset     env.reset() src/ppo.py:35,65,96 -> MiniGridEnv.reset ->
 *                        <Difficulty>Env._gen_grid (medium_hard_env.py:12-45,
 *                        hard_env.py:11-73, easy/medium/hardest_env.py)
 *   merlin_env_step      env.step(action.item()) src/ppo.py:76 ->
 *                        ThreeActionWrapper.action (three_action_wrapper.py:16-17)
 *                        -> MiniGridEnv.step [+ StuckPenaltyWrapper.step
 *                        stuck_penalty_wrapper.py:29-57]; done = term or trunc
 *                        (src/ppo.py:77); auto-reset on done (src/ppo.py:93-98)
 *   obs codes            RGBImgPartialObsWrapper.observation -> get_pov_render
 *                        (gen_obs_grid + process_vis), selected at
 *                        scenario_creator.py:48
 *   merlin_obs_expand_*  Grid.render tile blit + ImgObsWrapper
 *                        (scenario_creator.py:50), PPO._obs_to_tensor
 *                        src/ppo.py:58-62, CNNActorCritic._format_obs
 *                        src/actor_critic.py:43-46 and the /255 of
 *                        CNNFeatureExtractor.forward src/actor_critic.py:20-21
 *   merlin_gae           PPO.compute_gae src/ppo.py:107-120
 *                        (== compute_gae_standard src/utils/utils_rl.py:11-29)
 *   merlin_adv_normalize (adv - adv.mean()) / (adv.std() + 1e-8) src/ppo.py:125
 *   merlin_conv1_lut_*   the first Conv2d(3,32,k8,s4)+ReLU of both CNNFeatureExtractor
 *                        towers (src/actor_critic.py:9-10,20-21) evaluated from the
 *                        tile codes, and its weight/bias gradient
 *   merlin_tower_*       the data-movement stages around the conv2/conv3 GEMMs of the
 *                        towers (actor_critic.py:11-14): conv1 -> conv2 im2col from codes,
 *                        conv2 bias+ReLU -> conv3 im2col, and their backward passes;
 *                        merlin_tower_conv2_lut_*: Conv2d(3,32,k8,s4)+ReLU+Conv2d(32,64,k4,s2)
 *                        of both towers (actor_critic.py:9-12) as table lookups from the
 *                        tile codes, and the table gradient
 *   merlin_tower_window_*, merlin_segment_sum: the same conv2 and the following
 *                        Conv2d(64,64,k3,s1)+ReLU (actor_critic.py:13-14) evaluated once per
 *                        distinct receptive-field window of an update, and the fixed-order
 *                        segmented sums of their backward pass (merlin/windows.py)
 *   merlin_tower_bias_relu / _relu_bwd / _head_bwd: the ReLU + bias epilogues of the
 *                        conv3 / fc1 GEMMs and the heads' backward (actor_critic.py:14-41)
 *
 * What the benched loop (bench.py, BASELINE cfg 2) calls, per rollout step: merlin_tower_codes_conv3_amax,
 * merlin_h3_gemm_nt_heads (cfg 12, heads only), merlin_env_act_step, merlin_env_refill; per update:
 * merlin_gae, merlin_adv_normalize, merlin_minibatch_patch_maps, and per optimizer step merlin_window_lut_*,
 * merlin_window_gemm_fwd / _bwd, merlin_tower_window_conv3_planes, merlin_h3_gemm_nt_heads (cfg 60),
 * merlin_ppo_loss*, merlin_tower_head_bwd_planes, merlin_h3_gemm_nt_planes (cfg 62),
 * merlin_h3_gemm_tn_gather_planes_a (cfg 20), merlin_segment_sum_* (R / S / dQ / dT2), merlin_stage_*,
 * merlin_clip_adam.  The rest serve the other drop-in paths -- the gym single env and the frame path (obs
 * expansion, conv1 / conv2 lookups per frame, im2col), the autograd window path, FOMAML (merlin_group_act) -- or
 * are ALTERNATE forms kept selectable for A/B and float64 precision tests: merlin_x6_* (fc1 in six bf16
 * products, rounds 2-3), merlin_h3_gemm_nt / _tn / _tn_planes / _nt_gather with the register-staged
 * configurations (round 4).  Probe-only configurations (kernel ablations that compute wrong results on purpose)
 * exist only in a -DMERLIN_PROBES build.
 */
#ifndef MERLIN_HIP_H
#define MERLIN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MERLIN_ABI_VERSION 3  /* 3: compact acting-table keys (round 5), plane-operand GEMMs */

#define MERLIN_OK 0
#define MERLIN_E_INVALID 1     /* bad argument / config */
#define MERLIN_E_HIP 2         /* a HIP runtime call failed */
#define MERLIN_E_DEVICE 3      /* device-side error flag raised (see merlin_env_errors) */
#define MERLIN_E_UNSUPPORTED 4 /* e.g. grid size > 32 */

/* difficulty ids (ScenarioCreator difficulties, src/config/scenario.yaml) */
#define MERLIN_EASY 0
#define MERLIN_MEDIUM 1
#define MERLIN_MEDIUMHARD 2
#define MERLIN_HARD 3
#define MERLIN_HARDEST 4

/* device error bits reported by merlin_env_errors */
#define MERLIN_DEVERR_BAD_ACTION 1u  /* action not in {0,1,2}: ThreeActionWrapper IndexError */
#define MERLIN_DEVERR_PLACE_OBJ 2u   /* place_obj max_tries exceeded: RecursionError */
#define MERLIN_DEVERR_SLOT_EMPTY 8u  /* a reset met an empty look-ahead slot with the step fallback off */
#define MERLIN_DEVERR_BAD_TILE 4u    /* merlin_tower_codes_conv3: a frame that is no observation (the agent tile (class
                                      * 4) missing at view cell (3, 6) or present elsewhere): merlin_tower_errors */

/* observation layouts for merlin_obs_expand_f32 */
#define MERLIN_LAYOUT_NCHW 0 /* [n][3][56][56]: what CNNActorCritic._format_obs hands the convs */
#define MERLIN_LAYOUT_NHWC 1 /* [n][56][56][3]: the RolloutBuffer / gym observation layout */

/* Observation codes: one 7x7 view per env = 49 tile classes (0 dark-empty,
 * 1 lit empty, 2 lit wall, 3 lit goal, 4 agent), 4 bits each, cell (vi,vj)
 * at nibble vj*7+vi, packed into MERLIN_OBS_WORDS uint32 words (32 B). */
#define MERLIN_OBS_WORDS 8
#define MERLIN_OBS_TILES 5
#define MERLIN_TILE_PX 8
#define MERLIN_VIEW 7

typedef struct merlin_env merlin_env;

typedef struct {
    int32_t num_envs;          /* envs in this context (this rank's shard) */
    int32_t size;              /* grid side, 5..32 (reference: 16, base_env.py:17) */
    int32_t difficulty;        /* MERLIN_* difficulty id */
    int32_t max_steps;         /* <= 0: 4*size^2 (base_env.py:32-33) */
    int32_t stuck_penalty;     /* 1: StuckPenaltyWrapper semantics (off in the reference chain) */
    int32_t max_stay;          /* StuckPenaltyWrapper.max_stay (default 3) */
    double penalty;            /* StuckPenaltyWrapper.penalty (default -0.1) */
    int32_t exploration_bonus; /* 1: +bonus on the first visit of a cell per episode */
    double bonus;
    int32_t reseed_each_reset; /* 1: every reset regenerates from the seeded RNG state, i.e.
                                  env.reset(seed=task_seed) on every episode as FOMAML's
                                  collect_trajectory does (src/fomaml.py:63,92) */
} merlin_env_config;

/* [host] Layout check for bindings that restate merlin_env_config (ctypes, cgo, ...): returns
 * sizeof(merlin_env_config) and writes the byte offset of its first min(n_fields,
 * MERLIN_ENV_CONFIG_FIELDS) fields, in declaration order, to offsets_host (nullable).
 * merlin_env_create reads all MERLIN_ENV_CONFIG_FIELDS fields: a binding must match. */
#define MERLIN_ENV_CONFIG_FIELDS 10
int64_t merlin_env_config_layout(int64_t *offsets_host, int32_t n_fields);

/* Library */
int merlin_version(void);
const char *merlin_last_error(void);
/* [host] the 5 tiles (uint8[5][8][8][3]) the library renders with, computed at
 * load time by the library's own restatement of minigrid's render_tile. */
int merlin_tile_atlas(uint8_t *out_host);

/* Env context */
int merlin_env_create(const merlin_env_config *cfg, merlin_env **out);
int merlin_env_destroy(merlin_env *env);
/* Seed env i with seeds_host[i] (numpy SeedSequence -> PCG64, as gymnasium
 * reset(seed=...)); takes effect at the next merlin_env_reset of that env. */
int merlin_env_seed(merlin_env *env, const uint64_t *seeds_host, int32_t n, void *stream);
/* Reset the envs whose mask_dev[i] != 0 (mask_dev NULL = all), writing their
 * observation codes to obs_dev[i][8]; others' obs rows are left untouched. */
int merlin_env_reset(merlin_env *env, const uint8_t *mask_dev, uint32_t *obs_dev, void *stream);
/* Advance all envs n_steps times.  Step t reads actions_dev[t*action_stride + i]
 * (int64, values 0 left / 1 right / 2 forward) and writes, at row t*num_envs+i:
 *   obs_dev[..][8]  observation after the step (after the auto-reset if done),
 *   reward_dev f32, terminated_dev u8, truncated_dev u8, done_dev f32 (term|trunc),
 *   ep_return_dev f64 / ep_length_dev i32 (the finished episode's totals; valid
 *   where done).  Any output pointer may be NULL.  autoreset=0 leaves a done env
 *   in its terminal state (gym semantics: the caller must reset it). */
int merlin_env_step(merlin_env *env, const int64_t *actions_dev, int32_t n_steps,
                    int64_t action_stride, uint32_t *obs_dev, float *reward_dev,
                    uint8_t *terminated_dev, uint8_t *truncated_dev, float *done_dev,
                    double *ep_return_dev, int32_t *ep_length_dev, int32_t autoreset,
                    void *stream);
/* The rollout's act -> env.step in one launch (src/ppo.py:73-76: ac.act(state) then env.step(action.item())):
 * the action of env i is drawn from the acting GEMM's head partials head_part float[2][n_parts][N][4] exactly as
 * merlin_act_draw draws it (log-softmax, argmax or the counter-keyed race keyed by seed, *epoch, step and
 * env_offset + i; biases added; action / logp / value written to action / logp / value, int64 / float / float[N]),
 * then stepped as merlin_env_step with n_steps = 1 and auto-reset.  Output pointers other than action / logp /
 * value may be NULL. */
int merlin_env_act_step(merlin_env *env, const float *head_part_dev, int32_t n_parts, const float *b_actor_dev,
                        const float *b_critic_dev, int32_t act_dim, int32_t deterministic, uint64_t seed,
                        const int64_t *epoch_dev, int64_t step, int64_t env_offset, int64_t *action_dev,
                        float *logp_dev, float *value_dev, uint32_t *obs_dev, float *reward_dev,
                        uint8_t *terminated_dev, uint8_t *truncated_dev, float *done_dev, double *ep_return_dev,
                        int32_t *ep_length_dev, void *stream);
/* FOMAML's acting step (src/fomaml.py:54-108: each task's fast_policy.act(state), src/actor_critic.py:48-56), one
 * frame per task g < groups, each task with its own weights (merlin/grouped_policy.py pack: towers 2g = actor,
 * 2g + 1 = critic): codes_dev int32[groups][8]; T2 float[2G][2720][64] + b2 [2G][64] (conv1 + conv2 tables);
 * W3t [2G][576][64] ((ky, kx, ci) x co) + b3 [2G][64]; W4p [2G][512][576] (fc1, columns (p3, co)) + b4 [2G][512];
 * Wa [G][act_dim][512] + ba [G][act_dim], Wc [G][512] + bc [G] (the heads).  Writes a3_ws [2G][576] (conv3's
 * output) and head_part float[2][8][G][4]: tower t, fc1 column chunk p (64 columns), the chunk's dot products of
 * relu(fc1) with the task's head weights (the biases added in chunk 0) -- the partials merlin_env_act_step reads
 * (with zero biases) to draw and step every task's env.  fp32.  shared_weights = 1: every task acts with ONE weight set
 * (the tensors hold one task's: T2 [2][2720][64], ..., Wa [1][act_dim][512]) -- the support rollout, where every fast
 * policy is still the meta policy (src/fomaml.py:164-171), reads 2 towers' weights instead of 2G copies. */
int merlin_group_act(const uint32_t *codes_dev, int32_t groups, const float *T2_dev, const float *b2_dev,
                     const float *W3t_dev, const float *b3_dev, const float *W4p_dev, const float *b4_dev,
                     const float *Wa_dev, const float *ba_dev, const float *Wc_dev, const float *bc_dev,
                     int32_t act_dim, float *a3_ws_dev, float *head_part_dev, int32_t shared_weights, void *stream);
/* Look-ahead maps (no reference counterpart: an implementation detail of the auto-reset above).
 * An env's next map depends only on its RNG stream, so it is generated ahead of time into a
 * per-env slot, and an auto-reset takes the slot instead of generating in the step.
 * merlin_env_reset refills every slot before it returns; merlin_env_step refills the used slots
 * every `every` step calls (default 16).  every = 0 hands the refills to the caller:
 * merlin_env_refill launches one on `stream` -- e.g. on a side stream after each step, joined
 * before the next step, so the (latency-bound) map generation overlaps the policy forward.  A
 * reset whose slot is empty generates its map in the step instead; results are identical
 * either way. */
int merlin_env_set_refill_interval(merlin_env *env, int32_t every);
int merlin_env_refill(merlin_env *env, void *stream);
/* step_fallback (default on): with refill interval 0, single-step launches are followed by the fallback pass that
 * generates the map of a reset whose slot was empty.  A caller that refills every used slot after EVERY step, before
 * the next one (PPO's rollout: merlin_env_refill on a side stream, joined), can never meet an empty slot and may turn
 * the pass off (one launch -- one graph node -- fewer per step); an empty slot then raises MERLIN_DEVERR_SLOT_EMPTY
 * (merlin_env_errors) and that step's results are invalid. */
int merlin_env_set_step_fallback(merlin_env *env, int32_t on);
/* The fully observable observation (FullyObsWrapper + ImgObsWrapper, src/scenario_creator/scenario_creator.py:45-50,
 * observation.fully_observable in src/config/scenario.yaml) of every env's current state: out_dev uint8[N][size][size]
 * [3], out[i][x][y] = minigrid Grid.encode's (object, color, state) of cell (x, y), the agent's cell (10, 0, dir).
 * observation.flatten (FlattenObservation, :52-53) is the same bytes read as uint8[N][size*size*3]. */
int merlin_env_full_obs(merlin_env *env, uint8_t *out_dev, void *stream);
/* [sync] copy env state to host: walls uint32[N][size] (bit x of row y = wall at
 * (x,y)); agent int32[N][8] = (x, y, dir, step_count, goal_x, goal_y, stay, 0);
 * rng uint64[N][5] = (state_hi, state_lo, inc_hi, inc_lo, has32<<32|buf32).
 * Any pointer may be NULL. */
int merlin_env_get_state(merlin_env *env, uint32_t *walls_host, int32_t *agent_host,
                         uint64_t *rng_host, void *stream);
/* [sync] read-and-clear the device error bits and the fallback-map counter. */
int merlin_env_errors(merlin_env *env, uint32_t *flags_host, uint32_t *fallbacks_host,
                      void *stream);
int merlin_env_num_envs(const merlin_env *env);
int merlin_env_size(const merlin_env *env);

/* Observation expansion: out[k] = RGB image of codes_dev[index_dev ? index_dev[k] : k],
 * k < n.  f32: values are tile bytes * scale (scale = 1/255 folds
 * CNNFeatureExtractor's /255), layout MERLIN_LAYOUT_*.  u8: NHWC bytes, exactly
 * the RGBImgPartialObsWrapper(tile_size=8) frame. */
int merlin_obs_expand_f32(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                          float *out_dev, float scale, int32_t layout, void *stream);
int merlin_obs_expand_u8(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                         uint8_t *out_dev, void *stream);

/* GAE over [T][N] (row t, env i at t*N+i), truncation treated as terminal
 * (done = term or trunc).  stats_dev (nullable) receives double[3] =
 * (count, sum adv, sum adv^2) of this call's advantages -- the per-rank
 * partial that multi-GPU callers all-reduce before merlin_adv_normalize. */
int merlin_gae(const float *reward_dev, const float *value_dev, const float *done_dev,
               const float *last_value_dev, float *adv_dev, float *ret_dev, int32_t T, int32_t N,
               double gamma, double lam, double *stats_dev, void *stream);
/* out[k] = (adv[k] - mean) / (std_unbiased + 1e-8) with mean/std from
 * stats_dev = (count, sum, sum of squares); out may alias adv. */
int merlin_adv_normalize(const float *adv_dev, int64_t n, const double *stats_dev, float *out_dev,
                         void *stream);

/* conv1 from tile codes (both towers at once).  tables_dev: float[towers][32][4][20]
 * = P[co][slot=(dy,dx)][class*4 + quarter], the conv1 weights contracted with the
 * /255-scaled atlas (see csrc/merlin_conv1.hip); bias_dev float[towers][32].
 * out_dev float[towers][n][32][13][13] = relu(conv1(frame_k)) with frame_k the frame
 * of codes_dev[index_dev ? index_dev[k] : k]. */
int merlin_conv1_lut_fwd(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                         const float *tables_dev, const float *bias_dev, int32_t towers,
                         float *out_dev, void *stream);
/* Backward: dz = grad * (act > 0) with act/grad float[towers][n][32][13][13];
 * writes dtables_dev float[towers][32][4][20] and dbias_dev float[towers][32]
 * (overwritten, not accumulated). */
int merlin_conv1_lut_bwd(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                         const float *act_dev, const float *grad_dev, int32_t towers,
                         float *dtables_dev, float *dbias_dev, void *stream);

/* Tower stages (towers = 1 or 2; n frames; K orders are (ky, kx, ci)).
 * conv2_im2col_fwd: A2[t][k*25 + p2][(ky*4+kx)*32 + ci] = relu(conv1 of frame k)[ci]
 *   at (2*oy+ky, 2*ox+kx), p2 = oy*5+ox; tables/bias as merlin_conv1_lut_fwd.
 * conv2_im2col_bwd: dtables/dbias of that map given dA2 (same layout); the ReLU mask
 *   is recomputed from the tables.
 * conv3_im2col_fwd: A3[t][k*9 + p3][(ky*3+kx)*64 + ci] = relu(Z2[t][k*25 + (oy+ky)*5
 *   + ox+kx][ci] + b2[t][ci]), p3 = oy*3+ox.
 * conv3_col2im_bwd: dZ2 = [Z2 + b2 > 0] * col2im(dA3). */
int merlin_tower_conv2_im2col_fwd(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                                  const float *tables_dev, const float *bias_dev, int32_t towers,
                                  float *A2_dev, void *stream);
int merlin_tower_conv2_im2col_bwd(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                                  const float *tables_dev, const float *bias_dev,
                                  const float *dA2_dev, int32_t towers, float *dtables_dev,
                                  float *dbias_dev, void *stream);
int merlin_tower_conv3_im2col_fwd(const float *Z2_dev, const float *b2_dev, int64_t n,
                                  int32_t towers, float *A3_dev, void *stream);
int merlin_tower_conv3_col2im_bwd(const float *dA3_dev, const float *Z2_dev, const float *b2_dev,
                                  int64_t n, int32_t towers, float *dZ2_dev, void *stream);
/* Same, writing dZ2 chunk-major, dZ2c[t][ci/4][k*25 + p2][ci%4] (the histogram's input),
 * and absmax_dev[0] = float bits of max |dZ2| (the histogram's fixed-point scale). */
int merlin_tower_conv3_col2im_bwd_chunked(const float *dA3_dev, const float *Z2_dev,
                                          const float *b2_dev, int64_t n, int32_t towers,
                                          float *dZ2c_dev, uint32_t *absmax_dev, void *stream);

/* conv1 + conv2 as table lookups (csrc/merlin_conv2lut.hip has the derivation).
 * tables_dev float[towers][rows][64], rows = merlin_tower_conv2_lut_rows() = 2720:
 *   row = base(type) + 4*v + j for conv2 tap (ky, kx), type = (ky&1, kx&1) with bases
 *   0 / 20 / 120 / 220 for (0,0) / (0,1) / (1,0) / (1,1), j = 2*(ky>>1) + (kx>>1), and v
 *   the classes of the tiles the tap's conv1 position covers, in base 5 (row-major tiles).
 *   Row content: W2[:, :, ky, kx] applied to relu(conv1) of that tile combination.
 * lut_fwd: Z2[t][k*25 + p2][co] = sum over the 16 taps of tables[t][row(tap, p2, frame k)][co]
 *   (conv2 of relu(conv1(frame k)), no conv2 bias), frame k = codes[index ? index[k] : k].
 * lut_bwd: dtables[t][row][co] = sum of dZ2 over the (k, p2) that read row at some tap, for
 *   frame k = codes_dev[k] (the minibatch's own rows, no index), given dZ2 chunk-major and its
 *   max |dZ2| (float bits, >= the true max) as written by
 *   merlin_tower_conv3_col2im_bwd_chunked; summed in 64-bit fixed point (exact,
 *   order-independent), overwritten, not accumulated.  A non-finite max gives NaN. */
int merlin_tower_conv2_lut_rows(void);
int merlin_tower_conv2_lut_fwd(const uint32_t *codes_dev, const int64_t *index_dev, int64_t n,
                               const float *tables_dev, int32_t towers, float *Z2_dev,
                               void *stream);
int merlin_tower_conv2_lut_bwd(const uint32_t *codes_dev, int64_t n, const float *dZ2c_dev,
                               const uint32_t *absmax_dev, int32_t towers, float *dtables_dev,
                               void *stream);
/* Grouped form (one weight set per group of frames: FOMAML's per-task policies, src/fomaml.py:158-212).
 * towers = 2 * groups; frames codes[g * group_frames + i] (i < group_frames) belong to group g and are
 * evaluated by towers 2g (actor) and 2g+1 (critic) only, with their own tables:
 * lut_fwd_grouped: Z2[2g + c][i*25 + p2][co] for the n = groups * group_frames frames;
 * lut_bwd_grouped: dtables[2g + c] from dZ2c[2g + c] (chunk-major, group_frames frames per tower, as
 *   merlin_tower_conv3_col2im_bwd_chunked writes it for n = group_frames, towers = 2 * groups);
 *   slabs_dev: caller-owned scratch of merlin_tower_conv2_lut_slab_bytes(towers, group_frames) bytes. */
int merlin_tower_conv2_lut_fwd_grouped(const uint32_t *codes_dev, int64_t n, int64_t group_frames,
                                       const float *tables_dev, int32_t towers, float *Z2_dev, void *stream);
int64_t merlin_tower_conv2_lut_slab_bytes(int32_t towers, int64_t group_frames);
int merlin_tower_conv2_lut_bwd_grouped(const uint32_t *codes_dev, int64_t group_frames, const float *dZ2c_dev,
                                       const uint32_t *absmax_dev, int32_t towers, float *dtables_dev,
                                       void *slabs_dev, void *stream);

/* Receptive-field windows (csrc/merlin_window.hip; the plan is built by merlin/windows.py).
 * window_lut:   Z2w[t][w][co] = sum over the 16 taps of tables[t][rows[w][tap]][co]
 *               (rows int32[n_windows][16]: conv2 table rows as merlin_tower_conv2_lut_fwd's)
 * window_conv3: Y3[t][k*9 + p3][co] = relu(b3[t][co] + sum over tap = ky*3 + kx of
 *               Q[t][wid[g*25 + (oy+ky)*5 + ox+kx]][tap][co]), g = groups ? groups[k] : k,
 *               p3 = oy*3 + ox; Q float[towers][n_windows][9][64], wid int32[*][25]
 * segment_sum:  out[t][key[e]][:] = sum over the nnz entries e (keys ascending) of
 *               src[t][row(e)][:], each destination summed in entry order (no atomics);
 *               row(e) = idx[e], or with slot_dev slot[idx[e] / sub] * sub + idx[e] % sub,
 *               entries whose slot is -1 skipped.  Items of item_len entries; fix_dev
 *               int32[n_fix][4] = (dst, first item, last item, carry slot in the first item)
 *               for destinations spanning items; carry_dev float[towers][ceil(nnz /
 *               item_len)][2][64] scratch.  out float[towers][out_rows][64] is overwritten
 *               (rows without entries = 0), or with accumulate != 0 the sums are added to it
 *               (a list split by source block into several calls sums in call order). */
int merlin_tower_window_lut(const int32_t *rows_dev, int64_t n_windows, const float *tables_dev,
                            int32_t towers, float *Z2w_dev, void *stream);
/* The live-patch maps of every minibatch of an update (merlin/windows.py WindowPlan._bulk_minibatches): group g
 * (group_keys[g] = minibatch m * n_frames + frame; group_offsets[m] = first group of minibatch m), position p3 ->
 * patch k = kid[frame * 9 + p3]: kmap[m * n_patches + k] = k (preset to -1 by the caller), rmap[...] = one row
 * j * 9 + p3 of m holding k (scratch, no preset), rep_row[g * 9 + p3] = that row (conv3's patch representatives). */
int merlin_minibatch_patch_maps(const int32_t *kid_dev, const int64_t *group_keys_dev, int64_t n_groups,
                                int64_t n_frames, const int64_t *group_offsets_dev, int32_t n_patches, int32_t *kmap_dev,
                                int32_t *rmap_dev, int32_t *rep_row_dev, void *stream);
/* window_lut with conv2's bias and ReLU applied as the rows are written: a2w[t][w] = relu(Z2w[t][w] + b2[t]). */
int merlin_tower_window_lut_bias_relu(const int32_t *rows_dev, int64_t n_windows, const float *tables_dev,
                                      int32_t towers, const float *b2_dev, float *a2w_dev, void *stream);
int merlin_tower_window_conv3(const float *Q_dev, int64_t n_windows, const int32_t *wid_dev,
                              const int64_t *groups_dev, int64_t n, const float *b3_dev,
                              int32_t towers, float *Y3_dev, void *stream);
/* conv3 of the acting path from a table over every 3x3 tile window an observation can hold:
 * Qall_dev float[towers][merlin_tower_all_windows() = 4^9 + 3 * 4^8 = 458,752][9][64] (Q of
 * merlin_tower_window_conv3 for the window with compact key k: a window away from the agent's view cell (3, 6) =
 * its 9 tile classes 0..3 in base 4, tile (0,0) most significant; a window at conv2 position (4, wx), wx = 1..3,
 * which holds the agent's tile (class 4) at local (2, 3 - wx) = 4^9 + (wx - 1) 4^8 + its other 8 classes in
 * base 4 -- merlin/windows.py compact_window_keys; built once per rollout, merlin/actor_critic.py rollout_pack);
 * Y3[t][k*9 + p3][co] = relu(b3[t][co] + sum over the 9 taps of Qall[t][id of frame k's window at
 * p3 + tap][tap][co]) for frames codes_dev[k] (8 words of tile-class nibbles, merlin_env_step). */
int64_t merlin_tower_all_windows(void);
int merlin_tower_codes_conv3(const uint32_t *codes_dev, int64_t n, const float *Qall_dev,
                             const float *b3_dev, int32_t towers, float *Y3_dev, void *stream);
/* Same, with amax_dev (or NULL): atomicMax of max |Y3| per tower as float bits into amax_dev[t] (zeroed by the
 * caller), the operand scale of the acting path's fc1 on merlin_h3_gemm_nt. */
int merlin_tower_codes_conv3_amax(const uint32_t *codes_dev, int64_t n, const float *Qall_dev,
                                  const float *b3_dev, int32_t towers, float *Y3_dev, uint32_t *amax_dev,
                                  void *stream);
/* tower_errors: the device error flags the tower kernels raised on this device since the last call
 * (MERLIN_DEVERR_BAD_TILE from merlin_tower_codes_conv3: a frame whose compact table key is not its window), then
 * clears them; synchronises `stream` (PPO reads it once per rollout, with merlin_env_errors). */
int merlin_tower_errors(uint32_t *flags, void *stream);
/* Same, also writing relu_bits_dev uint64[towers][n*9]: bit co of row (k*9 + p3) = Y3 > 0 there; amax_dev
 * (or NULL): atomicMax of max |Y3| per tower as float bits into amax_dev[t] (zeroed by the caller), the operand
 * scale of fc1's f16 two-plane GEMMs (merlin_h3_gemm_*). */
int merlin_tower_window_conv3_bits(const float *Q_dev, int64_t n_windows, const int32_t *wid_dev,
                                   const int64_t *groups_dev, int64_t n, const float *b3_dev,
                                   int32_t towers, float *Y3_dev, uint64_t *relu_bits_dev, uint32_t *amax_dev,
                                   void *stream);
/* merlin_tower_window_conv3_bits (relu_bits_dev may be NULL here) computing each distinct 5x5-tile patch once:
 * rows (k, p3) whose frames hold the same patch at p3 read the same windows, so only the representative rows
 * (rep_row_dev[r] == r; rep_row_dev int32[n*9]: for every row r = k*9 + p3 of this call, a row of this call holding
 * the same patch, itself a representative) are computed; a second launch copies the other rows from theirs: their
 * Y3 rows with copy bit 0, their mask words with copy bit 1 (copy = 3: the same outputs as _bits; without a bit
 * the non-representative rows stay unwritten, for consumers that read rows through rep_row_dev); copy bit 2: the
 * copies only, after a call that computed the representatives (e.g. on another stream). */
int merlin_tower_window_conv3_reuse(const float *Q_dev, int64_t n_windows, const int32_t *wid_dev,
                                    const int64_t *groups_dev, int64_t n, const float *b3_dev,
                                    int32_t towers, float *Y3_dev, uint64_t *relu_bits_dev, uint32_t *amax_dev,
                                    const int32_t *rep_row_dev, int32_t copy, void *stream);
/* window_conv3_planes: window_conv3_reuse with copy = 0 (representatives only; the bits of the other rows are read
 * through rep_row by merlin_segment_sum_mask_rows) writing Y3 as its h3 planes (Y3_planes [t][n*9][8][2][8] f16, the
 * fp32 Y3's byte layout) for fc1's plane-operand GEMMs.  The plane scale of tower t comes from a bound on max Y3
 * computed first from Q: bound[t] (written, float bits) = max over c of relu(b3[t][c] + sum over taps of
 * max_w Q[t][w][tap][c]) >= every Y3 value; colmax_ws uint32[towers * 64 * 576] is scratch (per-block column maxima). */
int merlin_tower_window_conv3_planes(const float *Q_dev, int64_t nw, const int32_t *wid_dev, const int64_t *groups_dev,
                                     int64_t n, const float *b3_dev, int32_t towers, void *Y3_planes_dev,
                                     uint64_t *relu_bits_dev, const int32_t *rep_row_dev, uint32_t *colmax_ws_dev,
                                     uint32_t *bound_dev, void *stream);
int merlin_segment_sum(const float *src_dev, int64_t src_rows, const int32_t *idx_dev,
                       const int32_t *key_dev, int64_t nnz, const int32_t *slot_dev, int32_t sub,
                       int64_t item_len, const int32_t *fix_dev, int64_t n_fix, int32_t towers,
                       float *out_dev, int64_t out_rows, float *carry_dev, int32_t accumulate,
                       void *stream);
/* merlin_segment_sum with options.  mask_dev (or NULL): each source row is multiplied by a ReLU
 * mask of the same row (src where mask > 0, else 0: the ReLU backward of a forward output,
 * fused into the gather); float[towers][src_rows][64], or with MERLIN_SEG_MASK_BITS
 * uint64[towers][src_rows] (bit ch = channel ch > 0, as merlin_tower_window_conv3_bits writes).
 * flags: MERLIN_SEG_ACCUMULATE as accumulate != 0 above; MERLIN_SEG_NO_FILL leaves the rows of
 * destinations without any (unskipped) entry untouched instead of zeroing them (the caller
 * knows which rows are live, e.g. merlin/windows.py's patch sums). */
#define MERLIN_SEG_ACCUMULATE 1
#define MERLIN_SEG_NO_FILL 2
#define MERLIN_SEG_MASK_BITS 4
/* bits 8..10: which pass of conv3's backward this is (1 R, 2 S, 3 dQ, 4 dT2; 0 generic) -- it only
 * names the kernel instantiation, so profiles tell the passes apart; the sums are the same */
#define MERLIN_SEG_ROLE_SHIFT 8
#define MERLIN_SEG_ROLE_MASK (7 << MERLIN_SEG_ROLE_SHIFT)
int merlin_segment_sum_masked(const float *src_dev, const void *mask_dev, int64_t src_rows,
                              const int32_t *idx_dev, const int32_t *key_dev, int64_t nnz,
                              const int32_t *slot_dev, int32_t sub, int64_t item_len,
                              const int32_t *fix_dev, int64_t n_fix, int32_t towers, float *out_dev,
                              int64_t out_rows, float *carry_dev, int32_t flags, void *stream);
/* merlin_segment_sum_masked that also marks the destinations it sums into: mark_dev int32[out_rows]
 * (or NULL), mark[key(e)] = key(e) for every entry e not skipped; rows of other keys keep what the
 * caller put there (-1).  The marks are a slot map (sub 1) for a following pass that reads these
 * rows, so it skips the rows no entry was summed into (with MERLIN_SEG_NO_FILL they are never
 * written: merlin/fast_step.py's band sums of conv3's backward). */
int merlin_segment_sum_marked(const float *src_dev, const void *mask_dev, int64_t src_rows,
                              const int32_t *idx_dev, const int32_t *key_dev, int64_t nnz,
                              const int32_t *slot_dev, int32_t sub, int64_t item_len,
                              const int32_t *fix_dev, int64_t n_fix, int32_t towers, float *out_dev,
                              int64_t out_rows, float *carry_dev, int32_t flags, int32_t *mark_dev,
                              void *stream);
/* merlin_segment_sum_marked with the destinations that span items finished inside the launch (no second fix-up
 * launch): head_fix_dev int32[n_items] = the fix row (the item) at which item i's first destination started when it
 * continues into item i, else -1; counters_dev int32[n_fix] zero before the first call (the launch leaves them zero).
 * Requires one fix row per item (n_fix = ceil(nnz / item_len), as merlin/windows.py SegmentPlan builds it).  The
 * item that completes a row adds the row's partial sums in the fix-up pass's order: the same bits as
 * merlin_segment_sum_marked.  Both NULL: that function. */
int merlin_segment_sum_fused(const float *src_dev, const void *mask_dev, int64_t src_rows,
                             const int32_t *idx_dev, const int32_t *key_dev, int64_t nnz,
                             const int32_t *slot_dev, int32_t sub, int64_t item_len,
                             const int32_t *fix_dev, int64_t n_fix, int32_t towers, float *out_dev,
                             int64_t out_rows, float *carry_dev, int32_t flags, int32_t *mark_dev,
                             const int32_t *head_fix_dev, int32_t *counters_dev, void *stream);
/* merlin_segment_sum_fused with the mask's bit words read through a row map: the mask of source row r is
 * mask[t][mask_rows[r]] (conv3's patch representatives, merlin_tower_window_conv3_reuse with copy = 0: rows of one
 * patch share their ReLU mask and only the representatives' words are written). */
int merlin_segment_sum_mask_rows(const float *src_dev, const void *mask_dev, int64_t src_rows, const int32_t *idx_dev,
                                 const int32_t *key_dev, int64_t nnz, const int32_t *slot_dev, int32_t sub,
                                 int64_t item_len, const int32_t *fix_dev, int64_t n_fix, int32_t towers, float *out_dev,
                                 int64_t out_rows, float *carry_dev, int32_t flags, int32_t *mark_dev,
                                 const int32_t *head_fix_dev, int32_t *counters_dev, const int32_t *mask_rows_dev,
                                 void *stream);

/* Acting tail (src/actor_critic.py:48-55 act, src/ppo.py:69-71): z float[2][n][hidden] = fc1's
 * pre-activation of the actor / critic tower, b4 float[2][hidden]; h = relu(z + b4); logits =
 * w_actor float[act_dim][hidden] . h0 + b_actor, value = w_critic float[hidden] . h1 + b_critic[0];
 * action int64[n] = argmax(logits) when deterministic, else a Categorical(logits) draw (exponential
 * races on a counter-based generator keyed by seed, *epoch_dev (NULL = 0; bump it to redraw in
 * a replayed graph), step and the global env index env_offset + k, so data-parallel shards draw
 * what one process over the concatenated envs draws); logp float[n] = log_softmax(logits)[action],
 * value float[n].  hidden % 4 == 0, act_dim <= 8.  Non-finite logits (where the reference's
 * Categorical(logits) raises) give action -1, which merlin_env_step flags as
 * MERLIN_DEVERR_BAD_ACTION. */
int merlin_act_heads(const float *z_dev, const float *b4_dev, int64_t n, int32_t hidden,
                     const float *w_actor_dev, const float *b_actor_dev, const float *w_critic_dev,
                     const float *b_critic_dev, int32_t act_dim, int32_t deterministic, uint64_t seed,
                     const int64_t *epoch_dev, int64_t step, int64_t env_offset, int64_t *action_dev,
                     float *logp_dev,
                     float *value_dev, void *stream);

/* PPO minibatch loss (src/ppo.py:136-150), per distinct frame u < n_frames of the minibatch:
 *   logits float[n_frames][act_dim] (act_dim <= 8), value float[n_frames]; the frame's samples
 *   are order[offs[u] .. offs[u+1]) (int32 CSR, offs[n_frames] = n_samples, every frame owns
 *   >= 1 sample), frame_of int64[n_samples] maps a sample to its frame (frame_of[order[k]] =
 *   the u whose range holds k), and sample i reads actions / logp_old / adv / ret at
 *   sample_index[i] (int64; NULL = i).  With logp = log_softmax(logits), ratio = exp(logp[a] -
 *   logp_old),
 *   loss = -mean(min(ratio*A, clamp(ratio, 1-clip_eps, 1+clip_eps)*A)) + vf_coef*mean((v-R)^2)
 *          - ent_coef*mean(entropy)
 * writes loss float[1], dlogits float[n_frames][act_dim] and dvalue float[n_frames] = d loss /
 * d (logits, value) summed over each frame's samples (fixed order; torch.min / clamp
 * subgradients), and adds (-mean(min(...)), mean((v-R)^2), mean(entropy), mean(logp_old -
 * logp), mean(|ratio-1| > clip_eps)) to stats double[5] (NULL: not written).  workspace double[
 * merlin_ppo_loss_workspace(n_samples)].  An action outside [0, act_dim) makes the loss NaN.
 * bias_actor float[act_dim] / bias_critic float[1] (NULL = 0) are added to logits / value
 * first, and dbias_actor / dbias_critic (NULL: not written) get their gradients. */
int64_t merlin_ppo_loss_workspace(int64_t n_samples);
int merlin_ppo_loss(const float *logits_dev, const float *value_dev, const float *bias_actor_dev,
                    const float *bias_critic_dev, int64_t n_frames, int32_t act_dim, const int32_t *offs_dev,
                    const int32_t *order_dev, const int64_t *frame_of_dev, int64_t n_samples,
                    const int64_t *sample_index_dev, const int64_t *actions_dev, const float *logp_old_dev,
                    const float *adv_dev, const float *ret_dev, double clip_eps, double vf_coef, double ent_coef,
                    float *dlogits_dev, float *dvalue_dev, float *dbias_actor_dev, float *dbias_critic_dev,
                    float *loss_dev, double *stats_dev, double *workspace_dev, void *stream);
/* merlin_ppo_loss plus grad_absmax_dev uint32[9] (or NULL): atomicMax of max over the frames of |dlogits[u][j]|
 * into [j] (j < act_dim) and of max |dvalue[u]| into [8], as float bits (the caller zeroes it) -- the bound
 * merlin_tower_head_bwd_planes derives dz's plane scale from. */
int merlin_ppo_loss_absmax(const float *logits_dev, const float *value_dev, const float *bias_actor_dev,
                           const float *bias_critic_dev, int64_t n_frames, int32_t act_dim, const int32_t *offs_dev,
                           const int32_t *order_dev, const int64_t *frame_of_dev, int64_t n_samples,
                           const int64_t *sample_index_dev, const int64_t *actions_dev, const float *logp_old_dev,
                           const float *adv_dev, const float *ret_dev, double clip_eps, double vf_coef,
                           double ent_coef, float *dlogits_dev, float *dvalue_dev, float *dbias_actor_dev,
                           float *dbias_critic_dev, float *loss_dev, double *stats_dev, double *workspace_dev,
                           uint32_t *grad_absmax_dev, void *stream);

/* Tower GEMM epilogues (csrc/merlin_head.hip): towers = 1 or 2, `rows` per tower; cols (hidden)
 * a multiple of 4 dividing 1024 (4 x a divisor of 256).  Column sums use a per-device library
 * workspace: calls on one device must be stream-ordered with each other.
 * bias_relu: z[t][r][c] = relu(z[t][r][c] + bias[t][c]) in place (NaN propagates), after a
 *            plain GEMM (conv3 / fc1 of CNNFeatureExtractor / the heads, actor_critic.py:9-41)
 * relu_bwd:  dz = [y > 0] * dy (dz may alias dy), dbias[t][c] = sum over r of dz[t][r][c]
 * head_bwd:  the heads' backward through fc1's ReLU (actor_critic.py:30-41): h float[2][n][hidden]
 *            = relu(fc1) of the actor / critic tower, dlogits float[n][act_dim], dvalue float[n],
 *            w_actor float[act_dim][hidden], w_critic float[hidden] ->
 *            dz[0][k] = [h0 > 0] * (dlogits[k] . w_actor), dz[1][k] = [h1 > 0] * dvalue[k] * w_critic,
 *            dbias float[2][hidden] = sum_k dz[t][k], dw_actor = dlogits^T h0, dw_critic = dvalue^T h1
 *            (fixed-order sums; act_dim <= 8); amax_dev (or NULL): atomicMax of max |dz| per tower as float
 *            bits into amax_dev[0..1] (zeroed by the caller; merlin_h3_gemm_*'s operand scale). */
int merlin_tower_bias_relu(float *z_dev, const float *bias_dev, int64_t rows, int32_t cols, int32_t towers,
                           void *stream);
int merlin_tower_relu_bwd(const float *y_dev, const float *dy_dev, float *dz_dev, int64_t rows, int32_t cols,
                          int32_t towers, float *dbias_dev, void *stream);
/* colsum: out float[towers][cols] = sum over r < rows of x[t * tower_stride + r * row_stride + c]
 * (fixed order; strides in floats, multiples of 4): the conv3 bias gradient from the per-window tap-0
 * rows of dQ (merlin/windows.py). */
int merlin_tower_colsum(const float *x_dev, int64_t rows, int32_t cols, int64_t row_stride, int64_t tower_stride,
                        int32_t towers, float *out_dev, void *stream);
int merlin_tower_head_bwd(const float *h_dev, const float *dlogits_dev, const float *dvalue_dev,
                          const float *w_actor_dev, const float *w_critic_dev, int64_t n, int32_t hidden,
                          int32_t act_dim, float *dz_dev, float *dbias_dev, float *dw_actor_dev,
                          float *dw_critic_dev, uint32_t *amax_dev, void *stream);
/* head_bwd_planes: head_bwd with dz written as its h3 planes dz_planes [2][n][hidden/8][2][8] f16 (merlin_h3_split's
 * layout, 4 B per value) instead of fp32, scaled by the power of two from a bound on max |dz| known before the pass:
 * dz_bound_dev[t] (written, float bits) = max over k of sum_j grad_absmax[j] |w_actor[j][k]| (tower 0) /
 * grad_absmax[8] |w_critic[k]| (tower 1), grad_absmax_dev from merlin_ppo_loss_absmax.  dz_bound_dev is then the
 * operand scale of the planes for merlin_h3_gemm_nt_planes / merlin_h3_gemm_tn_gather_planes_a.  hidden a multiple
 * of 8 dividing 1024. */
int merlin_tower_head_bwd_planes(const float *h_dev, const float *dlogits_dev, const float *dvalue_dev,
                                 const float *w_actor_dev, const float *w_critic_dev, int64_t n, int32_t hidden,
                                 int32_t act_dim, void *dz_planes_dev, float *dbias_dev, float *dw_actor_dev,
                                 float *dw_critic_dev, const uint32_t *grad_absmax_dev, uint32_t *dz_bound_dev,
                                 void *stream);
/* heads_fwd: the two heads (actor_critic.py:41-46, Linear(512, act_dim) / Linear(512, 1)) on h
 * float[2][n][hidden] = relu(fc1) of the actor / critic tower: logits float[n][act_dim] = h0 w_actor^T
 * (+ b_actor), value float[n] = h1 . w_critic (+ b_critic); biases may be NULL (not added).  hidden 512,
 * act_dim <= 8; one fixed summation order (every call the same bits). */
int merlin_tower_heads_fwd(const float *h_dev, int64_t n, int32_t hidden, const float *w_actor_dev,
                           int32_t act_dim, const float *w_critic_dev, const float *b_actor_dev,
                           const float *b_critic_dev, float *logits_dev, float *value_dev, void *stream);

/* fc1 (src/actor_critic.py:31-41, Linear(576, 512) of both towers) on the bf16 matrix cores in fp32
 * (csrc/merlin_gemm.hip): every fp32 operand value x is used as three bf16 planes x0 + x1 + x2 == x
 * (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)), and a product as the six plane products
 * with i + j <= 2 (the terms left out are below one fp32 rounding), summed per 32-deep k step and
 * added to the fp32 running sum once.  Replaces the three fp32 GEMMs of CNNActorCritic's fc1 in
 * PPO.update (forward src/actor_critic.py:40, backward through autograd at src/ppo.py:153-155).
 * The weights are passed as "x6 planes", bf16 [R][C/8][3][8] (per group of 8 values three 16-byte
 * chunks, planes 0, 1, 2; merlin_x6_split); the activations as plain fp32, split while staged.
 * split / join: n fp32 values (n % 8 == 0) <-> their planes (6 bytes per value).
 * gemm_nt:  C[t][m][n] = sum_k A[t][m][k] B[t][n][k], A fp32 [M][K], B planes [N][K] (K % 32 == 0;
 *           tower strides in values), + bias[t][n] and ReLU when bias != NULL; cfg selects the tile
 *           (0: 256x128, 1: 128x192, 2: 128x128, 3: 256x64; N a multiple of the tile width).
 * gemm_tn:  out[t][m][n] = sum_k A[t][k][m] B[t][k][n], A fp32 [Kd][M], B fp32 [Kd][N] (M, N multiples
 *           of the tile: cfg 0 / 2: 128x192, 1: 128x64), the k range cut into <= splits slabs
 *           (slab float[merlin_x6_tn_slab_floats(...)]) summed in slab order. */
int merlin_x6_split(const float *x_dev, int64_t n, void *planes_dev, void *stream);
int merlin_x6_join(const void *planes_dev, int64_t n, float *x_dev, void *stream);
int merlin_x6_gemm_nt(const float *A_dev, const void *B_dev, int64_t M, int32_t N, int32_t K, int32_t towers,
                      int64_t a_stride, int64_t b_stride, const float *bias_dev, float *C_dev, int64_t c_stride,
                      int32_t cfg, void *stream);
int64_t merlin_x6_tn_slab_floats(int32_t M, int32_t N, int32_t towers, int32_t splits);
int merlin_x6_gemm_tn(const float *A_dev, const float *B_dev, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                      int64_t a_stride, int64_t b_stride, int32_t splits, float *slab_dev, float *out_dev, int32_t cfg,
                      void *stream);

/* fc1 (src/actor_critic.py:31-41) on the f16 matrix cores in fp32-class two-plane form (csrc/merlin_h3.hip, the
 * default of PPO.update's fc1 GEMMs): every operand x is scaled by a per-tower power of two 2^e (from its max |x|:
 * max |x| 2^e in [2^14, 2^15)) and used as two f16 planes h = f16(x'), l = f16((x' - h) 2^11); a product as the three
 * plane products h h, h l, l h (fp32 accumulation, the lo sum scaled by 2^-11 once), the result scaled back by
 * 2^-(eA + eB).  Error per output below the fp32 GEMM's (hipBLASLt) on the same operands (tests/test_gpu_h3.py).
 * Replaces the same three fp32 GEMMs as merlin_x6_* (forward src/actor_critic.py:40, backward src/ppo.py:153-155).
 * amax:  amax_dev[t] = float bits of max |x| over tower t's n values (x + t * stride; n, stride % 4 == 0); with n = 0
 *        it zeroes amax_dev[0 .. towers) (any count up to 2^20, by a kernel: safe inside a captured graph).
 * split: weight planes f16 [t][n/8][2][8] (per group of 8 values a hi and a lo 16-byte chunk), scaled by the
 *        exponent of amax_dev[t]; 4 bytes per value.
 * gemm_nt: C[t][m][n] = sum_k A[t][m][k] B[t][n][k], A fp32 [M][K] with its amax, B planes [N][K] (K % 32 == 0;
 *          tower strides in values), + bias[t][n] and ReLU when bias != NULL; cfg: 0 256x128, 1 128x192,
 *          2 128x128, 3 128x256 (N a multiple of the tile width), 10..13 the same tiles with the split interleaved
 *          into the MFMAs (K >= 64).  a_planes_dev (nullable): receives A's planes as the kernel makes them
 *          ([t][M][K/8][2][8] f16, A's byte layout and tower stride) for a later gemm_tn_planes.
 * gemm_tn: out[t][m][n] = sum_k A[t][k][m] B[t][k][n], both fp32 with their amax (cfg 0 / 1: 128x192 tiles, M % 128,
 *          N % 192), the k range cut into <= splits slabs (slab float[merlin_x6_tn_slab_floats(...)]) summed in slab
 *          order.
 * gemm_tn_planes: the same product over operands already in plane form (the a_planes output of gemm_nt for the same
 *          tensor and amax), strides in values.
 * gemm_nt_gather / gemm_tn_gather: gemm_nt (cfg 10..13) / gemm_tn (cfg 0..2) with the fp32 operand A / B read by
 *          64-value chunks through a row map: row r's chunk j (values 64 j .. 64 j + 63) is row rows_dev[r * K / 64 + j]
 *          (NT; TN: r * N / 64 + j) of the operand seen as [*][64] (tower stride as before; K or N % 64 == 0, K <= 576):
 *          conv3's rows through their patch representatives (merlin_tower_window_conv3_reuse with copy < 1). */
int merlin_h3_amax(const float *x_dev, int64_t n, int32_t towers, int64_t stride, uint32_t *amax_dev, void *stream);
int merlin_h3_split(const float *x_dev, int64_t n, int32_t towers, const uint32_t *amax_dev, void *planes_dev,
                    void *stream);
int merlin_h3_gemm_nt(const float *A_dev, const uint32_t *amax_a_dev, const void *B_dev, const uint32_t *amax_b_dev,
                      int64_t M, int32_t N, int32_t K, int32_t towers, int64_t a_stride, int64_t b_stride,
                      const float *bias_dev, float *C_dev, int64_t c_stride, void *a_planes_dev, int32_t cfg,
                      void *stream);
int merlin_h3_gemm_tn(const float *A_dev, const uint32_t *amax_a_dev, const float *B_dev, const uint32_t *amax_b_dev,
                      int64_t Kd, int32_t M, int32_t N, int32_t towers, int64_t a_stride, int64_t b_stride,
                      int32_t splits, float *slab_dev, float *out_dev, int32_t cfg, void *stream);
int merlin_h3_gemm_tn_planes(const void *A_planes_dev, const uint32_t *amax_a_dev, const void *B_planes_dev,
                             const uint32_t *amax_b_dev, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                             int64_t a_stride, int64_t b_stride, int32_t splits, float *slab_dev, float *out_dev,
                             int32_t cfg, void *stream);
int merlin_h3_gemm_nt_gather(const float *A_dev, const uint32_t *amax_a_dev, const void *B_dev,
                             const uint32_t *amax_b_dev, int64_t M, int32_t N, int32_t K, int32_t towers,
                             int64_t a_stride, int64_t b_stride, const float *bias_dev, float *C_dev, int64_t c_stride,
                             const int32_t *a_rows_dev, int32_t cfg, void *stream);
/* gemm_nt_heads: the update's fc1 forward (both towers, bias + ReLU, cfg 10 / 12 / 13, a_rows_dev nullable as in
 *          gemm_nt_gather) with the policy / value heads (src/actor_critic.py:41-46) folded into the epilogue: per
 *          row, merlin_h3_heads_parts(N, cfg) partial dot products of h with head_w0 [n_actions][N] (tower 0, the
 *          actor; n_actions <= 4) and head_w1 [N] (tower 1, the critic), head_partials_dev float
 *          [2][parts][M][4]; merlin_heads_combine sums them in order: logits [M][n_actions], value [M] (no biases).
 *          C_dev may be NULL (towers' h not written; merlin_act_draw then finishes the acting step). */
int merlin_h3_gemm_nt_heads(const float *A_dev, const uint32_t *amax_a_dev, const void *B_dev,
                            const uint32_t *amax_b_dev, int64_t M, int32_t N, int32_t K, int64_t a_stride,
                            int64_t b_stride, const float *bias_dev, float *C_dev, int64_t c_stride,
                            const int32_t *a_rows_dev, const float *head_w0_dev, int32_t n_actions,
                            const float *head_w1_dev, float *head_partials_dev, int32_t cfg, void *stream);
int32_t merlin_h3_heads_parts(int32_t N, int32_t cfg);
/* gemm_nt_planes: gemm_nt with A already in plane form too (A_planes [t][M][K/8][2][8] f16 scaled by amax_a_dev's
 *          exponent, e.g. merlin_tower_head_bwd_planes' dz), both operands staged into LDS by DMA (csrc/merlin_h3p.hip):
 *          cfg 60 128x256 / 62 128x192 tiles, K = 512 or 576, bias as gemm_nt.  Same products and order as gemm_nt
 *          on the fp32 A with the same scale: the same bits.  Measured alternates (round 6, not on the benched path):
 *          63 = 62 on a 4-stage ring; 66 = 62 with its MFMAs product-major (the same bits); 65 / 68 / 69 = one
 *          accumulator per tile (the lo planes rescaled in registers: another summation, held to float64 like the
 *          rest) on 256x192 / 256x256 (4 waves) / 192x192 tiles.
 * gemm_tn_gather_planes_a: gemm_tn_gather with A already in plane form (strides in values). */
int merlin_h3_gemm_nt_planes(const void *A_planes_dev, const uint32_t *amax_a_dev, const void *B_dev,
                             const uint32_t *amax_b_dev, int64_t M, int32_t N, int32_t K, int32_t towers,
                             int64_t a_stride, int64_t b_stride, const float *bias_dev, float *C_dev, int64_t c_stride,
                             int32_t cfg, void *stream);
/* gemm_nt_heads_planes: gemm_nt_heads (cfg 10 / 12 / 13, gathered rows, bias + ReLU, C_dev required) with A's
 *          gathered rows already h3 planes (merlin_tower_window_conv3_planes): staged as copies, no split; head_*
 *          NULL: h only.  With the planes of the same values and scale: gemm_nt_heads' bits.
 * gemm_tn_gather_planes: gemm_tn_gather with both operands as planes (dz from merlin_tower_head_bwd_planes, the
 *          gathered B from merlin_tower_window_conv3_planes). */
int merlin_h3_gemm_nt_heads_planes(const void *A_planes_dev, const uint32_t *amax_a_dev, const void *B_dev,
                                   const uint32_t *amax_b_dev, int64_t M, int32_t N, int32_t K, int64_t a_stride,
                                   int64_t b_stride, const float *bias_dev, float *C_dev, int64_t c_stride,
                                   const int32_t *a_rows_dev, const float *head_w0_dev, int32_t n_actions,
                                   const float *head_w1_dev, float *head_partials_dev, int32_t cfg, void *stream);
int merlin_h3_gemm_tn_gather_planes(const void *A_planes_dev, const uint32_t *amax_a_dev, const void *B_planes_dev,
                                    const uint32_t *amax_b_dev, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                                    int64_t a_stride, int64_t b_stride, int32_t splits, float *slab_dev,
                                    float *out_dev, const int32_t *b_rows_dev, int32_t cfg, void *stream);
int merlin_h3_gemm_tn_gather_planes_a(const void *A_planes_dev, const uint32_t *amax_a_dev, const float *B_dev,
                                      const uint32_t *amax_b_dev, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                                      int64_t a_stride, int64_t b_stride, int32_t splits, float *slab_dev,
                                      float *out_dev, const int32_t *b_rows_dev, int32_t cfg, void *stream);
/* The acting tail (merlin_act_heads' log-softmax, argmax or draw, action / logp / value) from the partials of a
 * merlin_h3_gemm_nt_heads call with C_dev = NULL (the acting path: h itself is never written), biases added here. */
int merlin_act_draw(const float *partials_dev, int32_t parts, int64_t n, const float *b_actor_dev,
                    const float *b_critic_dev, int32_t n_actions, int32_t deterministic, uint64_t seed,
                    const int64_t *epoch_dev, int64_t step, int64_t env_offset, int64_t *action_dev, float *logp_dev,
                    float *value_dev, void *stream);
int merlin_heads_combine(const float *partials_dev, int32_t parts, int64_t M, int32_t n_actions, float *logits_dev,
                         float *value_dev, void *stream);
int merlin_h3_gemm_tn_gather(const float *A_dev, const uint32_t *amax_a_dev, const float *B_dev,
                             const uint32_t *amax_b_dev, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                             int64_t a_stride, int64_t b_stride, int32_t splits, float *slab_dev, float *out_dev,
                             const int32_t *b_rows_dev, int32_t cfg, void *stream);

/* The conv1 / conv2 tables of both towers and their adjoint (the parameter-only part of PPO.update's
 * minibatch step, merlin/fast_step.py WeightStage; replaces CNNActorCritic.conv2_tables and its autograd
 * backward, src/actor_critic.py:9-14 conv1 / conv2), csrc/merlin_stage.hip.  Per tower t < towers (1..2):
 * W1 f32[t][32][3][8][8], b1 f32[t][32], W2 f32[t][64][32][4][4] (the conv weights, towers stacked), atlas
 * f32[5][3][8][8] (the tile atlas / 255), idx int16[680][4] (the conv1-table entries of each tile
 * combination, CNNActorCritic._lut2_h1_index order).  Forward: HT f32[t][680][32] (relu(conv1) of every
 * combination, kept for the backward), T2 f32[t][2720][64].  Backward from dT2 f32[t][2720][64]: dH
 * f32[t][680][32] (scratch), dW1 / db1 / dW2 in the layouts of W1 / b1 / W2; koff int16[81] / kv int16[2720]
 * = the combinations v of each table entry k (CSR, (v, e) order).  Fixed-order sums (bitwise reproducible).
 * The backward keeps partial sums in a per-device library workspace: calls on one device run one at a time
 * (one stream, or ordered streams). */
/* The window GEMM's backward (Q = a2w W3r, conv3 per window; src/actor_critic.py:13 conv3 + the ReLU of conv2,
 * replacing CNNActorCritic's bmm / split-K bmm / relu backward in merlin/fast_step.py), csrc/merlin_winbwd.hip.
 * Per tower t < towers: a2w f32[t][nw][64] (relu(conv2) of the windows), dQ f32[t][nw][576], W3r f32[t][64][576] ->
 * da2w = [a2w > 0] * (dQ W3r^T) f32[t][nw][64], db2 = column sums of da2w f32[t][64], dW3r = a2w^T dQ
 * f32[t][64][576]; db3 (nullable) = column sums of dQ's first 64 columns f32[t][64] (tap 0: conv3's bias gradient).
 * exact-f32 MFMA products and sums, fixed order (bitwise reproducible).  work: scratch of at least
 * merlin_window_gemm_bwd_work(towers, nw) floats (-1: invalid arguments). */
int merlin_window_gemm_fwd(const float *a2w_dev, const float *W3r_dev, int32_t towers, int64_t nw, float *Q_dev,
                           void *stream);  /* Q = a2w W3r f32[t][nw][576], exact-f32 MFMA, fixed order */
int64_t merlin_window_gemm_bwd_work(int32_t towers, int64_t nw);
int merlin_window_gemm_bwd(const float *a2w_dev, const float *dQ_dev, const float *W3r_dev, int32_t towers, int64_t nw,
                           float *da2w_dev, float *db2_dev, float *dW3r_dev, float *db3_dev, float *work_dev,
                           int64_t work_floats, void *stream);
int merlin_stage_tables_fwd(const float *W1_dev, const float *b1_dev, const float *W2_dev, const float *atlas_dev,
                            const int16_t *idx_dev, int32_t towers, float *HT_dev, float *T2_dev, void *stream);
int merlin_stage_tables_bwd(const float *W2_dev, const float *HT_dev, const float *dT2_dev, const float *atlas_dev,
                            const int16_t *koff_dev, const int16_t *kv_dev, int32_t towers, float *dH_dev,
                            float *dW1_dev, float *db1_dev, float *dW2_dev, void *stream);

/* Optimizer step of PPO.update (src/ppo.py:153-156: clip_grad_norm_(params, max_norm) then
 * Adam.step(), replacing torch.nn.utils.clip_grad_norm_ + torch.optim.Adam(fused=True).step()) over
 * n_tensors (1..32) float32 parameter tensors, csrc/merlin_optim.hip.  params / grads / exp_avg /
 * exp_avg_sq / steps are host arrays of device pointers (steps: each tensor's Adam step counter,
 * float32[1], advanced by one), numel[i] > 0.  The gradients are scaled in place by
 * min(max_norm / (||g||_2 + 1e-6), 1) as clip_grad_norm_ does; norm_out (float32[1], NULL: not
 * written) gets ||g||_2 before clipping.  Adam: torch's fused arithmetic (no weight decay, amsgrad
 * or maximize).  workspace double[merlin_clip_adam_workspace(n_tensors, numel)]. */
int64_t merlin_clip_adam_workspace(int32_t n_tensors, const int64_t *numel);
int merlin_clip_adam(int32_t n_tensors, float *const *params, float *const *grads, float *const *exp_avg,
                     float *const *exp_avg_sq, float *const *steps, const int64_t *numel, double lr, double beta1,
                     double beta2, double eps, float max_norm, float *norm_out, double *workspace, void *stream);

#ifdef __cplusplus
}
#endif
#endif
