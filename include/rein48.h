/*
 * rein48.h -- C-ABI of the MI355X-native 2048 environment (librein48.so).
 *
 * The reference (nevertiree/Rein48) has no FFI: its environment is the Python class
 * game/GameClient.py:Game, consumed duck-typed by main.py:39-48, algorithm/a3c/a3c.py:182-204
 * and algorithm/ddpg/ddpg.py:22-29. Each entry point below names the reference member it
 * replaces. The Python side binds them with ctypes (rein48_amd/_lib.py; INTEGRATION.md shows
 * the stub a reference maintainer would add).
 *
 * Conventions
 *   - A board is int8[16], row-major (cell (r,c) at 4*r+c). Cell value e: 0 = empty,
 *     e > 0 = tile 2^e (the reference stores the raw value 2^e in list[list[int]]).
 *   - Every array argument is a DEVICE pointer on the env's GPU, owned by the caller;
 *     nothing is allocated inside step/reset. Boards are bound with r48_env_bind_boards.
 *   - `stream` is a hipStream_t (NULL = default stream); calls are asynchronous on it.
 *   - Every function returns R48_OK (0) or a negative R48_E* status; the message for the
 *     calling thread is in r48_last_error(). The reference raises ValueError for a bad
 *     action (GameClient.py:254); batched kernels cannot raise, so a bad action byte
 *     leaves that board unchanged and is counted in the env's device error counter
 *     (r48_env_error_count).
 *   - Action codes: 0 UP, 1 DOWN, 2 LEFT, 3 RIGHT (GameClient.py:140,182,206,230).
 */
#ifndef REIN48_H
#define REIN48_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define R48_OK 0
#define R48_EINVAL (-1)   /* bad argument (null pointer, size, unbound boards, ...) */
#define R48_EHIP (-2)     /* a HIP runtime call failed */
#define R48_ENOMEM (-3)

/* step / create flags */
#define R48_AUTO_RESET 1u      /* a board that is done after the step is reset (reset rule) */
#define R48_RANDOM_POLICY 2u   /* actions drawn in-kernel (control/rand.py:9-11) and written back */
#define R48_MERGE_REWARD 4u    /* reward = merged tile values (opt-in; reference reward is 0) */

/* Version of the Philox-mode draw contract (which Philox words decide action, spawn and reset;
 * DESIGN.md section 7, restated in oracle/r48_oracle.c). A seed replays the same trajectories
 * only under the same version: version 3 (round 4) draws the step words from Philox4x32-7
 * (resets keep Philox4x32-10), version 2 (round 2) drew them from Philox4x32-10 and counts the
 * spawn rank over the blanks in the line order of the action, version 1 counted them row-major.
 * The injected-draw path (r48_env_step_with_draws) is the reference's row-major rule under every
 * version. */
#define R48_DRAW_CONTRACT 3

typedef struct r48_env r48_env;

/* Game.__init__ (GameClient.py:19-29) for a batch: an env of n_boards boards on `device`.
 * `board_offset` is the global id of board 0 (shard offset); Philox draws are keyed by
 * (seed, global board id), so a sharded run is identical to an unsharded one. */
int r48_env_create(r48_env **out, int device, int64_t n_boards, uint64_t seed, int64_t board_offset);
int r48_env_destroy(r48_env *env);

/* Game.state_matrix (GameClient.py:17,34,45): bind the caller's int8[n_boards][16] device
 * buffer (16-byte aligned) as the boards the env steps in place. */
int r48_env_bind_boards(r48_env *env, int8_t *boards);
int8_t *r48_env_boards(const r48_env *env);
int64_t r48_env_size(const r48_env *env);

/* Philox counters: the step counter advances once per r48_env_step, the reset counter once
 * per r48_env_reset. Exposed for checkpoint/resume and parity tests. */
int r48_env_get_counters(const r48_env *env, uint32_t *step, uint32_t *reset);
int r48_env_set_counters(r48_env *env, uint32_t step, uint32_t reset);

/* Game.reset (GameClient.py:33-38): zero the board, then ONE spawn (random_fill_grid,
 * :102-127). mask (uint8[n], nullable = all boards) selects the boards to reset. */
int r48_env_reset(r48_env *env, const uint8_t *mask, void *stream);

/* Synthetic start boards (bench input; no reference counterpart): every cell
 * empty w.p. 1/2, else exponent ~ U{1..max_exp} (max_exp in 1..17), from Philox keyed by
 * (seed, global board id) -- independent of sharding and of the counters, which it leaves as
 * they are. */
int r48_env_fill_random(r48_env *env, uint32_t max_exp, void *stream);

/* Game.reset with injected draws: rank[i] picks the blank (row-major, modulo the blank
 * count), four[i] != 0 spawns a 4 instead of a 2. */
int r48_env_reset_with_draws(r48_env *env, const uint8_t *mask, const uint8_t *rank,
                             const uint8_t *four, void *stream);

/* Game.step (GameClient.py:40-51) for every board: update_matrix (:129-254), spawn only if
 * the board changed (:48-49), then has_game_over on the spawned board (:51, :65-100).
 *   actions  int8[n]: read; with R48_RANDOM_POLICY drawn in-kernel (uniform over 0..3,
 *            control/rand.py:9-11) and written back when non-NULL.
 *   done     uint8[n] (nullable): has_game_over after the step (before any auto-reset).
 *   changed  uint8[n] (nullable): the reference's has_changed.
 *   reward   int32[n] (nullable): 0 (GameClient.py:138), or merged values with R48_MERGE_REWARD.
 *   score    int32[n] (nullable): tile-value sum after the step (main.py:48), before auto-reset.
 * flags: R48_AUTO_RESET | R48_RANDOM_POLICY | R48_MERGE_REWARD. Spawn draws come from
 * Philox4x32-10 keyed by (seed, board id) with the step counter, which then advances (the
 * rank counts the blanks in the line order of the move: uniform over the blanks like
 * random_fill_grid's row-major pick; oracle/r48_oracle.c orc_spawn_lines).
 * Ordering: every call on an env reads and writes its boards and advances its host-side step
 * counter at launch, so calls on one env must be ordered (one stream, or streams the caller
 * orders); different envs are independent. */
int r48_env_step(r48_env *env, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed,
                 int32_t *reward, int32_t *score, void *stream);

/* n_steps consecutive r48_env_step calls with the same arguments (outputs hold the last step's
 * values; the step counter advances by n_steps) in ONE kernel launch: boards are independent, so
 * every board stays in registers for all n_steps steps and is written back once, with the last
 * step's output planes -- bit-identical to n_steps r48_env_step calls, at a fraction of the HBM
 * traffic (34 B per board per call instead of per step). With given actions the same action
 * bytes apply at every step (a bad byte counts n_steps errors). n_steps >= 0. */
int r48_env_step_n(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done,
                   uint8_t *changed, int32_t *reward, int32_t *score, void *stream);

/* Game.step with the spawn draws injected (parity mode, reproduces a reference trajectory
 * given the reference's randint/uniform draws): rank[i] modulo the post-move blank count,
 * four[i] != 0 -> 4. No auto-reset, no step-counter advance. */
int r48_env_step_with_draws(r48_env *env, const int8_t *actions, const uint8_t *rank,
                            const uint8_t *four, uint32_t flags, uint8_t *done, uint8_t *changed,
                            int32_t *reward, void *stream);

/* The two halves of Game.step for callers that draw the spawn on the host after seeing
 * the move (the drop-in single-board Game uses the global Python `random`, exactly like
 * GameClient.py:121,125):
 *   r48_env_move : update_matrix only (:129-254) -> changed, n_blank (blank count after move)
 *   r48_env_spawn: random_fill_grid with injected draws where mask[i] != 0, then
 *                  has_game_over for every board -> done. */
int r48_env_move(r48_env *env, const int8_t *actions, uint32_t flags, uint8_t *changed,
                 uint8_t *n_blank, int32_t *reward, void *stream);
int r48_env_spawn(r48_env *env, const uint8_t *mask, const uint8_t *rank, const uint8_t *four,
                  uint8_t *done, void *stream);

/* Game.step of ONE board (the drop-in Game, GameClient.py:40-51) in one launch and one result
 * read: board = 16 exponent cells (host memory, copied into the kernel arguments), action 0..3.
 * One wave moves the board and, for every blank rank r (row-major, GameClient.py:109-114) and
 * tile (f = 0: 2, f = 1: 4), spawns it and evaluates has_game_over (:74-93), so the caller draws
 * the spawn with its own RNG (randint over the blank count, :121; uniform > 0.1, :125) after the
 * launch and picks candidate 2r + f. out (device memory, 16-byte aligned,
 * r48_game_step1_out_bytes() bytes): int8 [32][16] candidate boards; uint8 [512] changed (when 0
 * every candidate is the unchanged board, no spawn); uint8 [513] blank count after the move;
 * uint32 [516] game-over mask, bit 2r + f for candidate 2r + f. Replaces r48_env_move +
 * r48_env_spawn (two launches and two host round trips) for the single-board drop-in. */
int r48_game_step1(const int8_t *board, int32_t action, uint8_t *out, void *stream);
int r48_game_step1_out_bytes(void);

/* Pinned, device-mapped, coherent host memory (hipHostMalloc) for small results a kernel writes
 * straight to the host (the drop-in Game's r48_game_step1 `out`): returns the host pointer and
 * stores the device-side pointer in *device_ptr; NULL on failure. r48_host_free releases it. */
void *r48_host_alloc(int64_t bytes, void **device_ptr);
int r48_host_free(void *host_ptr);

/* Random-policy rollout (README.md:19 "random-policy data generation on GPU"; the
 * main.py:36-42 loop batched): n_steps Philox-mode steps with R48_RANDOM_POLICY |
 * R48_AUTO_RESET, boards held in registers across steps. Per step t it writes
 * actions[t*n + i] and done[t*n + i] (both nullable); equal to n_steps calls of
 * r48_env_step with those flags. */
int r48_env_rollout(r48_env *env, int32_t n_steps, int8_t *actions, uint8_t *done, void *stream);

/* main.py:48 score = np.sum(state_matrix): tile-value sum per board into int32[n]. */
int r48_env_score(r48_env *env, int32_t *out, void *stream);

/* Number of bad action bytes seen since the last clear (synchronises the stream). */
int r48_env_error_count(r48_env *env, int64_t *out, void *stream);
int r48_env_clear_errors(r48_env *env, void *stream);

/* ---- stateless value-domain helpers: the reference's @staticmethods on arbitrary integer
 * tiles (GameClientTest.py uses values such as 1 and non-square 4x1 / 1x4 matrices) ----
 * boards int32[n][16] of raw tile values (row-major 4x4; a smaller matrix is zero-padded on
 * the side AWAY from the move, which leaves its lines unchanged by construction).        */

/* Game.update_matrix (GameClient.py:129-254): in place; changed uint8[n]; actions int8[n]. */
int r48_values_move(int32_t *boards, const int8_t *actions, int64_t n, uint8_t *changed,
                    int64_t *reward, void *stream);
/* Game.has_table_filled (:96-100) / Game.has_game_over (:65-94) over rows x cols
 * (1..4 each) top-left sub-matrices; outputs uint8[n], each nullable. */
int r48_values_check(const int32_t *boards, int64_t n, int32_t rows, int32_t cols,
                     uint8_t *filled, uint8_t *over, void *stream);

/* Any board shape (Game(table_matrix_size) for sizes > 4, GameClient.py:19-27): boards
 * int32[n][rows][cols] of raw values, rows and cols in 1..R48_GRID_MAX.
 * r48_values_move_grid = update_matrix (:129-254), in place, changed uint8[n] (nullable);
 * r48_values_check_grid = has_table_filled (:96-100) / has_game_over (:65-94). */
#define R48_GRID_MAX 4096
int r48_values_move_grid(int32_t *boards, int64_t n, int32_t rows, int32_t cols, const int8_t *actions,
                         uint8_t *changed, void *stream);
int r48_values_check_grid(const int32_t *boards, int64_t n, int32_t rows, int32_t cols, uint8_t *filled,
                          uint8_t *over, void *stream);

/* ---- A3C pieces around the env step (algorithm/a3c/a3c.py) ---- */
#define R48_FEAT_VALUES 0     /* raw tile values 2^e, as a3c.py:37-39,139 feed the network */
#define R48_FEAT_EXPONENTS 1  /* the exponent e (a normalised input for the corrected mode) */
#define R48_F32 0
#define R48_BF16 1

/* Network input from boards: out[n][16] float32 or bf16 (16-byte aligned). */
int r48_board_features(const int8_t *boards, int64_t n, int32_t mode, int32_t out_dtype, void *out,
                       void *stream);

/* LocalAgent.choose_action (a3c.py:89-93) batched: softmax over logits float[n][4], then the
 * first action whose cumulative probability exceeds u (np.random.choice semantics), u from
 * Philox4x32-10(key = seed, counter = {gid0+i, ctr, 0xA3C}) with 24 bits. Optional outputs
 * logp[i] = log p[a_i] and entropy[i] = -sum_k p_k log(p_k + 1e-5) (a3c.py:114). */
int r48_sample_actions(const float *logits, int64_t n, uint64_t seed, int64_t gid0, uint32_t ctr,
                       int8_t *actions, float *logp, float *entropy, void *stream);

/* Worker._get_target_value_list (a3c.py:246-256) for n segments at once, time-major:
 * rewards/out float[T][n], lengths int32[n] (segment length, 1..T), bootstrap float[n].
 * drop_last != 0: out[len-1] = bootstrap, out[t] = r_t + gamma*out[t+1] (the reference, whose
 * last reward never enters); drop_last == 0: the textbook n-step return. out[t] = 0 for
 * t >= len. */
int r48_discounted_returns(const float *rewards, const int32_t *lengths, const float *bootstrap,
                           int32_t T, int64_t n, float gamma, int32_t drop_last, float *out,
                           void *stream);

/* Per-segment constants of the A3C loss (losses.segment_stats; a3c.py:99-123) for n segments of
 * lengths[i] (1..T) steps, time-major [T][n]: B[i] = max(lengths[i], 1); with td_sum (nullable):
 * td_sum[i] = sum over t < lengths[i] of targets[t][i] - values[t][i]; counts float[n][4] (16-byte
 * aligned) = per-segment action counts over t < lengths[i]. Replaces the masked sums and the
 * scatter-add of the tensor form (fp32 sums in step order). */
int r48_a3c_segment_stats(const float *values, const float *targets, const int8_t *actions, const int32_t *lengths,
                          int32_t T, int64_t n, float *B, float *td_sum, float *counts, void *stream);
/* The fused update's per-row weights over [T][n]: wn = (m / B[i]) * (1 / n) with m = t < lengths[i];
 * cm (nullable, the reference loss) = ((td_sum[i] / ((4 B[i]) B[i])) m) * (1 / n) -- the operation
 * order (and fp32 reciprocal) of the tensor form in rein48_amd/a3c/trainer.py, bit-identical to it. */
int r48_a3c_row_weights(const int32_t *lengths, const float *B, const float *td_sum, int32_t T, int64_t n, float *wn,
                        float *cm, void *stream);
/* The update's per-board pass in one launch (the fused update's inputs without any [T][n] weight rows):
 * targets float[T][n] exactly as r48_discounted_returns (same arguments), and per segment
 * seg float[n][4] = {w0, c0, L, 0} (16-byte aligned; L = clamp(lengths[i], 0, T) as int32 bits) with
 * w0 = (1 / B) (1 / n) and c0 = (td_sum / ((4 B) B)) (1 / n), B = max(L, 1) -- r48_a3c_row_weights' wn
 * and cm at every row t < L, bit for bit given the same td_sum. counts (nullable, 16-byte aligned;
 * the reference loss): float[n][4] action counts over t < L, as r48_a3c_segment_stats, and c0 from
 * td_sum = sum over t < L of targets - values (values float[T][n], actions int8[T][n] needed then),
 * summed from t = L - 1 down (the returns scan's order); without counts c0 = 0. */
int r48_a3c_segments(const float *rewards, const float *values, const int8_t *actions, const int32_t *lengths,
                     const float *bootstrap, int32_t T, int64_t n, float gamma, int32_t drop_last, float *targets,
                     float *seg, float *counts, void *stream);

/* tf.train.RMSPropOptimizer(lr) (a3c.py:264-265; TF1 semantics: ms slot starts at ONES, eps
 * inside the sqrt, momentum 0 by default) over one flat float32 parameter buffer of n values. */
int r48_rmsprop_tf1(float *var, const float *grad, float *ms, float *mom, int64_t n, float lr,
                    float decay, float momentum, float eps, void *stream);

/* Fused 2-layer CNN policy inference (config 3; rein48_amd/a3c/nets.py:ActorCriticCNN, the
 * conv trunk of algorithm/ddpg/actor.py:51-85 with actor/critic heads) on bf16 MFMA:
 * boards int8[n][16] -> logits float[n][4] and value float[n] (each nullable), and, when
 * actions != NULL, the choose_action draw of r48_sample_actions (same Philox contract) into
 * actions int8[n]; boards_out (nullable, 16-byte aligned): a copy of the input boards (the
 * rollout's trajectory snapshot, a3c.py:203-209). wfrag: 33 x 64 x 8 bf16 weight fragments (conv1,
 * conv2, and the heads laid out for 16x16x32 MFMAs) and
 * bias: 104 floats, both packed by rein48_amd/a3c/fused.py:pack_cnn (16-byte aligned). mode:
 * R48_FEAT_VALUES/EXPONENTS. */
int r48_cnn_policy_forward(const int8_t *boards, int64_t n, const void *wfrag, const float *bias,
                           int32_t mode, float *logits, float *value, int8_t *actions, int8_t *boards_out,
                           uint64_t seed, int64_t gid0, uint32_t ctr, void *stream);

/* The whole fused A3C rollout (configs 3-4; rein48_amd/a3c/trainer.py A3CTrainer.rollout, the
 * batched a3c.py:194-212 loop) in ONE launch: for each of n_steps steps, every board goes through
 * the policy of r48_cnn_policy_forward (same weights/bias packing and mode, action draw with
 * policy_seed, counter sample_ctr + t, board id gid0 + i) and then the env step of r48_env_step
 * with those actions (Philox key env_seed, step counter env_step + t, board id gid0 + i; no
 * auto-reset; R48_MERGE_REWARD in flags for the merge reward). boards int8[n][16] (16-byte
 * aligned) are read at the start and hold the final boards at the end; traj_boards
 * int8[n_steps + 1][n][16] receives the pre-step board of every step and the final board;
 * actions int8[n_steps][n], done uint8[n_steps][n], reward float[n_steps][n] (nullable; the merge
 * reward as fp32, exact below 2^24, 0 without R48_MERGE_REWARD), lengths
 * int32[n] (nullable): 1 + the first step that ended done, else n_steps (a3c.py:201); values
 * float[n_steps][n] (nullable): the critic value of every pre-step board, as r48_cnn_policy_forward's
 * `value` output (the reference loss's value pass, a3c.py:218-223, read from the rollout). Results
 * equal n_steps x (r48_cnn_policy_forward + r48_env_step) bit for bit; the caller advances the
 * env's step counter by n_steps (r48_env_set_counters). */
int r48_cnn_rollout(int8_t *boards, int64_t n, int32_t n_steps, const void *wfrag, const float *bias, int32_t mode,
                    int8_t *traj_boards, int8_t *actions, uint8_t *done, float *reward, int32_t *lengths,
                    float *values, uint64_t policy_seed, int64_t gid0, uint32_t sample_ctr, uint64_t env_seed, uint32_t env_step,
                    uint32_t flags, void *stream);

/* The reference's own network, fused (rein48_amd/a3c/nets.py:ActorCriticMLP = a3c.py:136-169: actor
 * 16 -> 64 ReLU6 -> 4 ReLU, critic 16 -> 64 ReLU6 -> 1, fp32) on the VALU, one board per lane.
 * w: float[r48_mlp_weight_floats()] packed by rein48_amd/a3c/fused.py:pack_mlp (16-byte aligned).
 * r48_mlp_policy_forward: boards int8[n][16] -> logits float[n][4] (post-ReLU, a3c.py:153) and
 * value float[n] (each nullable) and, when actions != NULL, the choose_action draw of
 * r48_sample_actions (same Philox contract) into actions int8[n]. mode: R48_FEAT_VALUES/EXPONENTS.
 * Replaces NetworkTool.get_network_output + LocalAgent.choose_action (a3c.py:89-93,136-169). */
int32_t r48_mlp_weight_floats(void);
int r48_mlp_policy_forward(const int8_t *boards, int64_t n, const float *w, int32_t mode, float *logits,
                           float *value, int8_t *actions, uint64_t seed, int64_t gid0, uint32_t ctr, void *stream);
/* The whole A3C rollout with the MLP in ONE launch: arguments, outputs and counters exactly as
 * r48_cnn_rollout, with the policy of r48_mlp_policy_forward; values (nullable) = the critic value of
 * every pre-step board. Equals n_steps x (r48_mlp_policy_forward + r48_env_step) bit for bit. */
int r48_mlp_rollout(int8_t *boards, int64_t n, int32_t n_steps, const float *w, int32_t mode, int8_t *traj_boards,
                    int8_t *actions, uint8_t *done, float *reward, int32_t *lengths, float *values,
                    uint64_t policy_seed, int64_t gid0, uint32_t sample_ctr, uint64_t env_seed, uint32_t env_step,
                    uint32_t flags, void *stream);

/* Fused A3C update for the reference MLP (fp32; the per-row loss of r48_cnn_train_grad below, here
 * through the logits' ReLU): arguments as r48_cnn_train_grad with the MLP weight blob w of
 * r48_mlp_policy_forward; grad float[2504] (16-byte aligned) receives the gradient in FlatParams
 * order (a1.w [64][16] | a1.b | a2.w [4][64] | a2.b | c1.w | c1.b | c2.w | c2.b = 2,501 floats),
 * then the actor and critic losses. workspace: r48_mlp_train_workspace_floats(rows) 4-byte words
 * (16-byte aligned; the per-wave records of the hot and the exact-decision pass and the hot pass's
 * per-wave lists of flagged tiles). Deterministic (fixed-order reduction). Replaces
 * NetworkTool.get_loss_value + compute_gradients (a3c.py:99-123, 73-80). */
int64_t r48_mlp_train_workspace_floats(int64_t rows);
int r48_mlp_train_grad(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                       const float *targets, const float *wn, const float *cm, const float *counts, float beta,
                       int32_t mode, const float *w, float *workspace, float *grad, void *stream);
/* The same with per-board weights: seg float[n_boards][4] of r48_a3c_segments (16-byte aligned) instead
 * of wn / cm -- row r = t n_boards + b weighs seg[b].w0 (and seg[b].c0) when t < seg[b].L, else 0;
 * the reference loss when counts != NULL. Equals r48_mlp_train_grad on the expanded rows bit for bit. */
int r48_mlp_train_grad_seg(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                           const float *targets, const float *seg, const float *counts, float beta, int32_t mode,
                           const float *w, float *workspace, float *grad, void *stream);

/* Fused A3C update for the CNN (configs 3-4; rein48_amd/a3c/losses.py restating a3c.py:99-123):
 * the gradient of (actor + critic) over `rows` training states w.r.t. every ActorCriticCNN
 * parameter, in one pass with no activation written to memory. boards int8[rows][16], actions
 * int8[rows], targets / wn float[rows] (wn = mask / (segment length * n)); reference-mode actor
 * loss when cm != NULL: cm float[rows] (= coef * mask / n) and counts float[n_boards][4] (row r
 * belongs to board r % n_boards); textbook otherwise. wfrag: 65 x 64 x 8 bf16 fragments and bias
 * 104 floats from rein48_amd/a3c/fused.py:pack_cnn_train. workspace: r48_cnn_train_workspace_floats()
 * floats; grad: r48_cnn_train_grad_floats() floats = dW2[64][128] | db2[64] | dW1[32][5] (col 4 =
 * bias) | dWh[5][257] (col 256 = bias) | actor loss | critic loss. Deterministic. */
int r48_cnn_train_grad(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                       const float *targets, const float *wn, const float *cm, const float *counts,
                       float beta, int32_t mode, const void *wfrag, const float *bias, float *workspace,
                       float *grad, void *stream);
/* The same with per-board weights (seg of r48_a3c_segments, as r48_mlp_train_grad_seg; n_boards < 2^31):
 * bit for bit r48_cnn_train_grad on the expanded rows. */
int r48_cnn_train_grad_seg(const int8_t *boards, int64_t rows, int64_t n_boards, const int8_t *actions,
                           const float *targets, const float *seg, const float *counts, float beta, int32_t mode,
                           const void *wfrag, const float *bias, float *workspace, float *grad, void *stream);
int64_t r48_cnn_train_workspace_floats(void);
int64_t r48_cnn_train_grad_floats(void);

/* ---- Transition store for replay-based training (config 5; algorithm/ddpg/replay.py) ----
 * HBM-resident, structure of arrays, 38 B per transition: state int8[16], action int8,
 * reward float, next_state int8[16], done uint8. State pointers must be 16-byte aligned. */
typedef struct r48_replay r48_replay;
#define R48_REPLAY_RING 0u        /* overwrite the oldest; sample uniformly WITH replacement */
#define R48_REPLAY_FILL_DRAIN 1u  /* Replay (replay.py:8-47): store drops once max_size is held
                                   * (:18-21); sample = random.sample WITHOUT replacement (a
                                   * permutation when batch == size), or the whole buffer in
                                   * insertion order if batch > size (:23-34),
                                   * then clear() (:26, :45-47) */

/* Replay.__init__(replay_size) (replay.py:10-13): `capacity` slots on `device`. Draws are
 * Philox4x32-10 keyed by `seed` with a per-sample counter. */
int r48_replay_create(r48_replay **out, int device, int64_t capacity, uint32_t mode, uint64_t seed);
int r48_replay_destroy(r48_replay *rep);
int64_t r48_replay_capacity(const r48_replay *rep);
/* cur_size (replay.py:12), the ring's next slot, the sample counter (checkpoint/resume). */
int r48_replay_get_counters(const r48_replay *rep, int64_t *size, int64_t *head, uint32_t *sample_ctr);
int r48_replay_set_counters(r48_replay *rep, int64_t size, int64_t head, uint32_t sample_ctr);
/* Device planes, for zero-copy readers: state/next_state [capacity][16], action, reward, done. */
int r48_replay_planes(const r48_replay *rep, int8_t **state, int8_t **action, float **reward,
                      int8_t **next_state, uint8_t **done);
/* Replay.clear (replay.py:45-47). */
int r48_replay_clear(r48_replay *rep);
/* Replay.store (replay.py:18-21) for n transitions at once (device arrays; reward and done
 * nullable = 0). *stored = how many were kept (FILL_DRAIN drops past capacity; RING keeps the
 * newest min(n, capacity)). */
int r48_replay_store(r48_replay *rep, const int8_t *state, const int8_t *action, const float *reward,
                     const int8_t *next_state, const uint8_t *done, int64_t n, int64_t *stored,
                     void *stream);
/* Replay.sample (replay.py:23-27) into device arrays of `batch` rows (each nullable; index =
 * the slot of each row). *count = rows written (FILL_DRAIN: min(batch, size)). */
int r48_replay_sample(r48_replay *rep, int64_t batch, int8_t *state, int8_t *action, float *reward,
                      int8_t *next_state, uint8_t *done, int64_t *index, int64_t *count, void *stream);
/* Gather the given slots (index int64[n], each in [0, size)); out-of-range indices produce
 * zero rows and are counted in r48_replay_error_count. */
int r48_replay_gather(r48_replay *rep, const int64_t *index, int64_t n, int8_t *state, int8_t *action,
                      float *reward, int8_t *next_state, uint8_t *done, void *stream);
int r48_replay_error_count(const r48_replay *rep, uint64_t *count);

/* ---- Value-based training around the env (config 5: ResNet-10 Q-network + replay) ----
 * No reference code exists for these (README.md:15-17 names ResNet + BN + ReLU for 2048; the
 * only replay anchor is algorithm/ddpg/replay.py). */
/* One-hot input planes: out[n][16][18] (position-major, plane e = exponent 0..17), f32/bf16. */
int r48_board_onehot(const int8_t *boards, int64_t n, int32_t out_dtype, void *out, void *stream);
/* Epsilon-greedy over q float[n][4] (16-byte aligned): Philox4x32-10(key = seed, counter =
 * {gid lo, gid hi, ctr, 0xD0E}), u = (w0 >> 8) / 2^24; u < eps -> action w1 >> 30, else the
 * first argmax. */
int r48_egreedy_actions(const float *q, int64_t n, float eps, uint64_t seed, int64_t gid0, uint32_t ctr,
                        int8_t *actions, void *stream);
/* TD target y[i] = R + gamma * (1 - done[i]) * q_next_target[i][a*], a* = argmax of
 * q_next_online[i] (double DQN) or of q_next_target[i] when q_next_online is NULL; R = reward[i],
 * or log2(1 + reward[i]) (fp32, as torch.log2(1.0 + r)) when log2_reward != 0 -- the trainer's
 * reward transform folded in. done nullable (= 0). Q arrays float[n][4], 16-byte aligned. */
int r48_td_target(const float *reward, const uint8_t *done, const float *q_next_target,
                  const float *q_next_online, int64_t n, float gamma, int32_t log2_reward, float *y, void *stream);

/* Huber loss (smooth L1, beta 1) of the update: d = q[i][action[i]] - y[i]; out[0] = mean loss,
 * out[1] = mean q[i][action[i]]; dq[i][a] = clamp(d, -1, 1) / n for a = action[i], else 0 (the
 * gradient of the mean loss). q, dq float[n][4] 16-byte aligned; workspace float[512].
 * Deterministic (fixed-order sums). Replaces trainer.py's gather + F.smooth_l1_loss + backward. */
int r48_huber_grad(const float *q, const int8_t *action, const float *y, int64_t n, float *dq, float *out,
                   float *workspace, void *stream);

/* Adam (torch.optim.Adam: bias-corrected, eps outside the square root) over one flat fp32
 * parameter buffer of n floats (n % 4 == 0, all four buffers 16-byte aligned), step = the 1-based
 * step count t: m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
 * param -= lr / (1 - b1^t) * m / (sqrt(v / (1 - b2^t)) + eps). One launch. Replaces the flat
 * optimizer step of rein48_amd/dqn/trainer.py's Adam on the GPU. */
int r48_adam(float *param, const float *grad, float *m, float *v, int64_t n, float lr, float beta1, float beta2,
             float eps, int64_t step, void *stream);

/* ---- The ResNet-10 update's 3x3 convolutions on the 4x4 grid (csrc/r48_conv.hip) ----
 * Channels-last bf16 activations [boards][16 cells][C], 64 output channels, 32 or 64 input
 * channels; only the 100 in-grid (cell, tap) pairs are computed. Replace the structured dense
 * GEMMs of nets.py:ResNet10Q._conv (hipBLASLt) in the update. */
/* The finish of the training-mode BN that a conv's output feeds (forward: r48_conv3x3_stats_finish,
 * r48_conv3x3_bn_in) or whose backward reduction a data-gradient conv sums (r48_conv3x3_bn_grad),
 * done in the conv itself by the workgroup that writes the last statistics record, so that no
 * finish launch sits between the conv and the BN's apply pass. Forward: save = float[2C] {mean,
 * invstd} of the conv's output over `rows`, coef = float[2C] {a = gamma invstd, b = beta - mean a},
 * running_mean / running_var (nullable together) updated with momentum and the unbiased variance;
 * beta, gamma as the BN's. Backward: save is read (the forward's), coef = float[3C] {a, cc, d} of
 * dx = a g + cc x + d, dgamma / dbeta (nullable) = invstd sum g (x - mean), sum g. The statistics
 * buffer's last float is the arrival counter: it must be 0 before the first such call (the finishing
 * workgroup resets it), and one buffer serves one such launch at a time (launches on one stream). C = 64
 * (the update's convs). */
typedef struct r48_bn_finish_args {
    const float *gamma;
    const float *beta;
    float *running_mean;
    float *running_var;
    float *save;
    float *coef;
    float *dgamma;
    float *dbeta;
    int64_t rows;
    float momentum;
    float eps;
} r48_bn_finish_args;
/* One-hot input planes for the training stem: out bf16 [n][16][32] (plane e = exponent 0..17,
 * planes 18..31 zero), 16-byte aligned. */
int r48_board_onehot32(const int8_t *boards, int64_t n, void *out, void *stream);
/* y[b][p][co] = bias[co] + sum over taps t in the grid, ci of W[co][ci][t] x[b][p + off(t)][ci]
 * (+ add[b][p][co]) (the forward conv; with the flipped, transposed taps the data gradient).
 * wfrag: 9 x 4 x (cin/32) MFMA A fragments of 1 KiB (rein48_amd/dqn/conv.py pack_conv); bias fp32
 * [64] or NULL; add bf16 [boards][16][64] or NULL (cin 64 only: a basic block's input gradient
 * summed in the epilogue). stats (NULL, or float[r48_conv_stats_floats()]; not with add): the
 * per-channel sum and sum of squares of the bf16 outputs, one record [S1 64][S2 64] per CU, for
 * r48_bn_forward_stats. All pointers 16-byte aligned. The statistics buffer's last float is the
 * arrival counter of the finishing forms (r48_bn_finish_args). */
int64_t r48_conv_stats_floats(void);
/* r48_conv3x3 with stats (no add) and the finish of the BN that its output feeds (fin, required):
 * the BN's apply pass follows as r48_bn_apply. */
int r48_conv3x3_stats_finish(const void *x, int64_t boards, int32_t cin, const void *wfrag, const float *bias, void *y,
                             float *stats, const r48_bn_finish_args *fin, void *stream);
/* The update's forward conv with the PREVIOUS layer's training-mode BN + ReLU folded into its operand
 * load (rein48_amd/dqn/train_step.py): x bf16 [boards][16][64] is that BN's input (the previous conv's
 * output); coef float[128] = (a[64], b[64]) from r48_bn_finish; residual (nullable) the block's identity
 * input. The conv consumes z = relu(a x + b (+ residual)) -- the arithmetic and rounding of
 * r48_bn_forward_stats' apply -- and also writes z into z_out and its ReLU mask (one byte per 8
 * channels, bit k = z > 0) into mask_out; y and stats as r48_conv3x3 with stats (required). Replaces
 * nets.py's BatchNorm + ReLU (+ identity) followed by the next conv (README.md:15-17). */
int r48_conv3x3_bn_in(const void *x, int64_t boards, const void *wfrag, const float *bias, const float *coef,
                      const void *residual, void *z_out, uint8_t *mask_out, void *y, float *stats,
                      const r48_bn_finish_args *fin, void *stream);
/* A data-gradient conv (64 -> 64 channels, wfrag from pack_conv_dgrad; + add as r48_conv3x3) whose
 * output dx is the gradient reaching a training-mode BN + ReLU, with that BN's backward reduction
 * fused in the epilogue: bn_part (float[r48_conv_stats_floats()]) gets per-CU records [sum g 64]
 * [sum g (bn_x - mean) 64], g = dx . bn_mask, bn_x the BN's input, mean = bn_save[0..63] -- the
 * input of r48_bn_backward_part. add_mask (NULL, or with add: [boards][16][8] bytes, bit k of byte
 * j = channel 8 j + k): the added term is add . [mask bit] -- a basic block's identity-path
 * gradient formed from the gradient at the block's output ReLU and that ReLU's forward mask. fin
 * (nullable; bn_save == fin->save): that BN's backward finish in the conv, the apply pass following
 * as r48_bn_backward_apply. r48_conv3x3_bn_in's fin (nullable) finishes the BN of ITS output. */
int r48_conv3x3_bn_grad(const void *dy, int64_t boards, const void *wfrag, const void *add, const uint8_t *add_mask,
                        void *dx, const void *bn_x, const uint8_t *bn_mask, const float *bn_save, float *bn_part,
                        const r48_bn_finish_args *fin, void *stream);
int r48_conv3x3(const void *x, int64_t boards, int32_t cin, const void *wfrag, const float *bias, const void *add,
                void *y, float *stats, void *stream);
/* dw fp32 [64][cin][3][3] = sum over boards and in-grid cells of dy[b][p][co] x[b][p + off(t)][ci];
 * workspace of r48_conv_wgrad_workspace_floats(cin) floats (per-workgroup records, summed in a
 * fixed order: deterministic). */
int64_t r48_conv_wgrad_workspace_floats(int32_t cin);
int r48_conv3x3_wgrad(const void *dy, const void *x, int64_t boards, int32_t cin, float *workspace, float *dw,
                      void *stream);
/* Every fragment set of the update's convs in one launch: weights = DEVICE array of 9 fp32
 * pointers (stem [64][18][3][3], conv1..8 [64][64][3][3]); fwd (bf16, 16-byte aligned) gets the
 * stem's 36 fragments then conv1..8's 72 each (the r48_conv3x3 wfrag of each layer, pack_conv
 * layout), dgrad gets conv1..8's data-gradient fragments (72 each, pack_conv_dgrad layout). */
int r48_conv_pack_resnet(const float *const *weights, void *fwd, void *dgrad, void *stream);
/* The Q head Linear(1024 -> 4) of the update (nets.py: linear(h, head.weight, head.bias, bf16)
 * .float(), replacing its three hipBLASLt GEMMs): h bf16 [boards][1024] (channels-last cells x
 * channels), w bf16 [4][1024], bias fp32 [4] (used bf16-rounded); q fp32 [boards][4] holds the
 * bf16-rounded outputs. Backward: dq fp32 [boards][4] (used bf16-rounded, as the gradient of the bf16
 * output) -> dh bf16 [boards][1024] and dw fp32 [4 * 1024 + 4] (weight rows, then the bias
 * gradient; bf16-rounded, fixed-order sums). All pointers 16-byte aligned. */
int r48_q_head_forward(const void *h, int64_t boards, const void *w, const float *bias, float *q, void *stream);
int64_t r48_q_head_workspace_floats(void);
int r48_q_head_backward(const float *dq, const void *h, int64_t boards, const void *w, void *dh, float *workspace,
                        float *dw, void *stream);

/* Fused ResNet-10 Q-network inference on bf16 MFMA (rein48_amd/dqn/nets.py:ResNet10Q with
 * C = 64, 4 basic blocks, eval-mode BN folded): boards int8[n][16] (16-byte aligned) -> q
 * float[n][4] (nullable, 16-byte aligned) and, when actions != NULL, the epsilon-greedy draw of
 * r48_egreedy_actions (same Philox contract) into actions int8[n]. wblob
 * (r48_resnet_q_blob_bytes() bytes, 16-byte aligned: every layer incl. the head as
 * v_mfma_f32_16x16x32_bf16 fragments) is packed by r48_resnet_pack or
 * rein48_amd/dqn/fused.py:pack_resnet. */
int r48_resnet_q_forward(const int8_t *boards, int64_t n, const void *wblob, float *q, int8_t *actions,
                         float eps, uint64_t seed, int64_t gid0, uint32_t ctr, void *stream);
int64_t r48_resnet_q_blob_bytes(void);
/* The packing of rein48_amd/dqn/fused.py:pack_resnet in one launch (eval-mode BN folded, bf16
 * fragments): ptrs is a DEVICE array of 56 float pointers -- for conv L = 0..8 (stem, conv1..8):
 * weight [co][ci][3][3], bias [co], BN gamma, beta, running mean, running var (gamma NULL: no BN)
 * -- then head weight [4][1024] and head bias [4]. Same layout as pack_resnet; the BN scale is
 * computed with correctly rounded f32 division and sqrt (may differ from PyTorch's in the last
 * ulp). */
int r48_resnet_pack(const float *const *ptrs, float bn_eps, void *wblob, void *stream);

/* Structured 3x3 (pad 1) conv weight on the 4x4 grid for the ResNet's GEMM form
 * (rein48_amd/dqn/nets.py dense_conv_weight): w float[co][ci][3][3] -> dense[16 co][16 ci] (f32 or
 * bf16, 16-byte aligned), block (P, Q) = w[:, :, dr + 1, dc + 1] where input cell Q = P + 4 dr + dc
 * is an in-grid neighbour of output cell P, else zero. Needs 16 ci % 8 == 0. The gradient maps
 * gdense[16 co][16 ci] (f32 or bf16) back to gw float[co][ci][3][3] (fixed summation order). */
int r48_struct_conv_weight(const float *w, int32_t co, int32_t ci, int32_t out_dtype, void *dense, void *stream);
int r48_struct_conv_weight_grad(const void *gdense, int32_t co, int32_t ci, int32_t in_dtype, float *gw,
                                void *stream);

/* Training-mode BatchNorm fused with ReLU and the basic block's identity add, for the ResNet-10
 * update (rein48_amd/dqn/nets.py, bn.py; replaces torch.nn.BatchNorm1d + F.relu + add on
 * channels-last bf16 activations). x, residual, y, dy, dx, dresidual: bf16 [rows][C], 16-byte
 * aligned, C in {32, 64, 128}; gamma, beta, running statistics, dgamma, dbeta: float[C].
 * Forward: y = relu?(gamma (x - mean) invstd + beta (+ residual)) with the batch statistics over
 * rows (biased variance), running_mean/var (nullable together) updated with `momentum` and the
 * unbiased variance, save = float[2 C] {mean, invstd} for the backward. Backward: given dy
 * (gradient of y) and the saved y (ReLU mask, when relu) -> dx, dgamma, dbeta (nullable) and
 * dresidual (nullable: the gradient reaching the residual input). workspace: float[
 * r48_bn_workspace_floats(rows, C)], not shared between calls in flight. Deterministic.
 * mask (nullable): uint8[rows][C / 8], bit k of byte (r, j) = (y[r][8 j + k] > 0); the forward
 * writes it, and the backward reads it instead of y when given (y may then be NULL). */
int64_t r48_bn_workspace_floats(int64_t rows, int32_t C);
int r48_bn_forward(const void *x, const void *residual, int64_t rows, int32_t C, const float *gamma,
                   const float *beta, float *running_mean, float *running_var, float momentum, float eps,
                   int32_t relu, float *save, float *workspace, void *y, uint8_t *mask, void *stream);
/* The forward from statistics a producer already summed (r48_conv3x3 `stats`: nblk records of
 * unshifted [S1 C][S2 C] sums over x): finish (mean, invstd, running statistics) + apply, as
 * r48_bn_forward without its statistics pass over x. */
int r48_bn_forward_stats(const float *part, int32_t nblk, const void *x, const void *residual, int64_t rows, int32_t C,
                         const float *gamma, const float *beta, float *running_mean, float *running_var,
                         float momentum, float eps, int32_t relu, float *save, float *workspace, void *y, uint8_t *mask,
                         void *stream);
/* The finish of r48_bn_forward_stats alone (no apply pass): from the nblk per-block sums `part` a
 * producer wrote (r48_conv3x3 stats), the batch mean / invstd into save[2C], the apply coefficients
 * (a = gamma invstd, b = beta - mean a) into coef[2C], and the running statistics (nullable). */
int r48_bn_finish(const float *part, int32_t nblk, int64_t rows, int32_t C, const float *gamma, const float *beta,
                  float *running_mean, float *running_var, float momentum, float eps, float *save, float *coef,
                  void *stream);
/* The backward (with ReLU mask) from sums a producer already reduced (r48_conv3x3_bn_grad: nblk
 * records of [sum g C][sum g (x - mean) C], g = dy . mask): finish + apply, as r48_bn_backward
 * without its reduction pass over dy and x. */
int r48_bn_backward_part(const float *part, int32_t nblk, const void *dy, const uint8_t *mask, const void *x,
                         int64_t rows, int32_t C, const float *gamma, const float *save, float *workspace, void *dx,
                         void *dresidual, float *dgamma, float *dbeta, void *stream);
int r48_bn_backward(const void *dy, const void *y, const uint8_t *mask, const void *x, int64_t rows, int32_t C,
                    const float *gamma, const float *save, int32_t relu, float *workspace, void *dx, void *dresidual,
                    float *dgamma, float *dbeta, void *stream);
/* The apply passes alone, from coefficients a finishing conv wrote (r48_bn_finish_args coef):
 * forward y = relu?(a x + b (+ residual)) (+ mask as r48_bn_forward), coef float[2C]; backward
 * dx = a g + cc x + d with g = dy . mask, coef float[3C]. */
int r48_bn_apply(const void *x, const void *residual, int64_t rows, int32_t C, const float *coef, int32_t relu, void *y,
                 uint8_t *mask, void *stream);
int r48_bn_backward_apply(const void *dy, const uint8_t *mask, const void *x, int64_t rows, int32_t C, const float *coef,
                          void *dx, void *stream);

/* Thread-local message of the last failed call on this thread ("" if none). */
const char *r48_last_error(void);
/* "rein48 <version> gfx950" */
const char *r48_version(void);

#ifdef __cplusplus
}
#endif

#endif /* REIN48_H */
