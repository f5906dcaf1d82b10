/*
 * splendor_amd.h — C ABI of the MI355X-native Splendor engine (libsplendor_amd.so).
 *
 * Drop-in boundary for the reference's Game plug-in surface as it is used on the
 * self-play hot path (kuboyoo/alphazero-general-ori):
 *   Game API          Game.py:14-162, implemented by SplendorGame.py:11-86
 *   rules engine      SplendorLogicNumba.Board (@jitclass), SplendorLogicNumba.py:84-774
 * The reference binds these from Python one board at a time through Numba's jitclass
 * boxing; this library exposes the same operations BATCHED over B boards held in device
 * memory (HBM), stream-ordered, with no allocation in any hot call. The Python host
 * mirror (alphazero-general-ori_amd/splendor/SplendorGame.py) binds it with ctypes.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers owned by the caller unless noted.
 *   - state: B boards x S bytes, S = 7*R, R = 32 + 10n + n^2 (the reference's int8 (R,7)
 *     observation, row-major, identical bytes to board.tobytes(), SplendorGame.py:63-64).
 *   - mask: B x 7 uint64; bit (a % 64) of word (a / 64) is action a (0..408).
 *   - player arrays are int8 (0..n-1); a NULL player pointer means "player 0 everywhere".
 *   - chance: either explicit uniforms (u != NULL: board b consumes u[b*u_stride + k],
 *     k = 0,1,.. in the reference's draw order) or counter-based Philox4x32-10 with
 *     key = seed and counter = (k, board_base + b, stream, 'SPLD').
 *   - hip_stream: a hipStream_t (NULL = default stream).
 *   - Return value: 0 ok; SPL_EINVAL bad argument; SPL_EDEVICE HIP launch/runtime error.
 *     Per-board errors found on device (action out of range) are OR-ed into *err when
 *     err != NULL (device int32), so hot calls never synchronise.
 */
#ifndef SPLENDOR_AMD_H
#define SPLENDOR_AMD_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define SPL_ABI_VERSION 1
#define SPL_ACTIONS 409
#define SPL_MASK_WORDS 7
#define SPL_EINVAL (-1)
#define SPL_EDEVICE (-2)
#define SPL_ERR_BAD_ACTION 1

typedef struct spl_ctx spl_ctx;

int spl_abi_version(void);

/* Board(num_players) rule constants (SplendorLogicNumba.py:86-98): n in {2,3,4};
 * token_limit = NUM_TOKEN_LIMIT (default 10; Board.setNumTokenLim, :214-215). */
int spl_ctx_create(int n_players, int token_limit, spl_ctx **out);
int spl_ctx_destroy(spl_ctx *ctx);
/* observation_size (SplendorLogicNumba.py:26-27): rows R; bytes per board 7*R */
int spl_state_rows(const spl_ctx *ctx);
int spl_state_bytes(const spl_ctx *ctx);

/* Board.init_game (SplendorLogicNumba.py:222-246) / SplendorGame.getInitBoard
 * (SplendorGame.py:17-19). Writes B fresh boards; player_out (nullable) set to 0.
 * Draws: 12 cards x 2 uniforms, then n+1 noble draws (partial Fisher-Yates). */
int spl_init(const spl_ctx *ctx, int B, int8_t *state, int8_t *player_out,
             const double *u, int u_stride, uint64_t seed, uint32_t stream,
             uint32_t board_base, void *hip_stream);

/* SplendorGame.getValidMoves (SplendorGame.py:35-37) -> Board.valid_moves
 * (SplendorLogicNumba.py:251-265). */
int spl_valid_moves(const spl_ctx *ctx, int B, const int8_t *state, const int8_t *player,
                    uint64_t *mask_out, void *hip_stream);

/* SplendorGame.getNextState (SplendorGame.py:30-33) -> Board.make_move
 * (SplendorLogicNumba.py:267-289), in place on `state`. deterministic=1 is the in-tree
 * transition (no deck draws, MCTS.py:228). next_player_out nullable. */
int spl_step(const spl_ctx *ctx, int B, int8_t *state, const int8_t *player,
             const int16_t *action, int8_t *next_player_out, int deterministic,
             const double *u, int u_stride, uint64_t seed, uint32_t stream,
             uint32_t board_base, int32_t *err, void *hip_stream);

/* SplendorGame.getGameEnded (SplendorGame.py:39-41) -> Board.check_end_game
 * (SplendorLogicNumba.py:320-334). out: B x n float32. */
int spl_game_ended(const spl_ctx *ctx, int B, const int8_t *state, float *out,
                   void *hip_stream);

/* SplendorGame.getCanonicalForm (SplendorGame.py:51-57) -> Board.swap_players
 * (SplendorLogicNumba.py:338-347). out may equal state. */
int spl_canonical(const spl_ctx *ctx, int B, const int8_t *state, const int8_t *player,
                  int8_t *out, void *hip_stream);

/* SplendorGame.getScore / getRound (SplendorGame.py:43-49): out B x n int32 / B int32 */
int spl_score(const spl_ctx *ctx, int B, const int8_t *state, int32_t *out, void *hip_stream);
int spl_round(const spl_ctx *ctx, int B, const int8_t *state, int32_t *out, void *hip_stream);

/* In-tree transition of MCTS.get_next_best_action_and_canonical_state (MCTS.py:222-237):
 * child = swap_players(make_move(copy(parent), a, 0, deterministic=True)). */
int spl_tree_step(const spl_ctx *ctx, int B, const int8_t *parent, const int16_t *action,
                  int8_t *child, int32_t *err, void *hip_stream);

/* One fused random-policy self-play step per board (BASELINE config 2; the move loop of
 * Coach.executeEpisode, Coach.py:71-100, with a uniform random policy):
 *   canonical -> valid mask -> action = k-th legal, k = floor(U(seed,b,step,0)*count)
 *   -> make_move(real board, player, chance draws 1,2) -> check_end -> if ended: re-init
 *   (draws 3..) and player=0, games_done[b] += 1.
 * Outputs mask (B x 7), action (B), ended (B x n), all per step. */
int spl_rollout_step(const spl_ctx *ctx, int B, int8_t *state, int8_t *player,
                     uint64_t *mask_out, int16_t *action_out, float *ended_out,
                     int32_t *games_done, uint64_t seed, uint32_t step, uint32_t board_base,
                     void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
