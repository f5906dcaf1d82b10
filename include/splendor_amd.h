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
 *     key = seed: uniform k is half (k & 1) of the block at counter
 *     (k >> 1, board_base + b, stream, 'SPLD'), 53 bits from words (0,1) or (2,3).
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

#define SPL_ABI_VERSION 11
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
/* Board.setNumTokenLim (SplendorLogicNumba.py:214-215; Arena.py:116 handicap games) */
int spl_ctx_set_token_limit(spl_ctx *ctx, int token_limit);
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

/* SplendorGame.getSymmetries (SplendorGame.py:59-61) -> Board.get_symmetries
 * (SplendorLogicNumba.py:349-395) for E examples (state E x S, pi E x 409 f32, valid E x 7
 * u64). Outputs K = 10 + 2n variant slots per example in the reference's order: identity,
 * 3 tiers x 3 card permutations, then per player up to 2 reserve permutations;
 * present[E][K] = 1 for emitted slots (reserve permutations depend on #reserved cards). */
int spl_symmetries(const spl_ctx *ctx, int E, const int8_t *state, const float *pi,
                   const uint64_t *valid, int8_t *out_state, float *out_pi, uint64_t *out_valid,
                   uint8_t *present, void *hip_stream);

/* One fused random-policy self-play step per board (BASELINE config 2; the move loop of
 * Coach.executeEpisode, Coach.py:71-100, with a uniform random policy):
 *   canonical -> valid mask -> action = k-th legal, k = floor(U(seed,b,step,0)*count)
 *   -> make_move(real board, player, chance draws 1,2) -> check_end -> if ended:
 *   games_done[b] += 1 = g and re-init with the deal of game g: draws 0..28 of stream
 *   0x80000000 | g (so deals can be drawn ahead of the game end; steps < 2^31), player=0.
 * games_done is required (it keys the deals). Outputs mask (B x 7), action (B), ended
 * (B x n), all per step. */
int spl_rollout_step(const spl_ctx *ctx, int B, int8_t *state, int8_t *player,
                     uint64_t *mask_out, int16_t *action_out, float *ended_out,
                     int32_t *games_done, uint64_t seed, uint32_t step, uint32_t board_base,
                     void *hip_stream);

/* K consecutive spl_rollout_step calls (steps step0 .. step0+K-1) in one launch: each
 * workgroup keeps its boards on chip for all K moves, so board bytes cross HBM once per
 * launch. Per-move outputs are stacked by move: mask_out [K][B][7] (may be NULL),
 * action_out [K][B], ended_out [K][B][n]; state, player and games_done hold the result
 * after move K. Bit-identical to K spl_rollout_step calls. */
int spl_rollout_run(const spl_ctx *ctx, int B, int K, int8_t *state, int8_t *player,
                    uint64_t *mask_out, int16_t *action_out, float *ended_out,
                    int32_t *games_done, uint64_t seed, uint32_t step0, uint32_t board_base,
                    void *hip_stream);


/* ===================================================================== MCTS
 * Device-resident batched PUCT search (MCTS.py), one tree per board/game, B trees.
 * The reference's MCTS(game, nnet, args).getActionProb(canonicalBoard, temp=1,
 * force_full_search) (MCTS.py:45-97) maps to:
 *     spl_mcts_set_roots(roots)                 -- re-root (tree persists when keep_tree)
 *     repeat until every tree spent its budget:
 *         spl_mcts_select(leaf_state, leaf_mask, leaf_valid)   -- MCTS.search descent
 *         <network on leaf_state/leaf_mask -> pi[B][409], v[B][n]> (nnet.predict, :138)
 *         spl_mcts_backup(leaf_mask, pi, v)     -- expansion + backup (:134-176)
 *     spl_mcts_root_stats(counts, qsa, probs, q) -- :61-97 (temp = 1)
 * Every tree runs exactly one simulation per select/backup pair, so each tree's search
 * is the reference's sequential search. Trees own device memory allocated at create. */
typedef struct spl_mcts spl_mcts;
typedef struct {
    int num_sims;            /* numMCTSSims (main.py:110) */
    int ratio_full;          /* ratio_fullMCTS: fast search = num_sims / ratio_full */
    double prob_full;        /* prob_fullMCTS: P(full search) (MCTS.py:54) */
    double cpuct;            /* cpuct */
    double fpu;              /* fpu (>0: parent-relative; <=0: absolute) (MCTS.py:203) */
    int forced_playouts;     /* forced playouts + policy-target pruning (MCTS.py:56,69-74) */
    double dirichlet_alpha;  /* > 0 enables root noise at step 0 of full searches */
    double dirichlet_temp;   /* temperature[0]: softmax before noise (MCTS.py:142) */
    int temp_threshold;      /* tempThreshold (Coach.py:82-83), self-play only */
    int node_cap;            /* maximum node slots of one tree (its transposition table and
                                node page table are sized for it) */
    int edge_cap;            /* maximum edge units of one tree (its edge page table). Edges are
                                stored in two tiers of 8-byte units: every edge one unit (prior,
                                action) in its node's run, and an edge with statistics (Nsa,
                                Qsa, child link) 3 more in its node's visit block */
    uint64_t seed;           /* Philox key for search/self-play randomness */
    uint32_t board_base;     /* global id of tree 0 (multi-GPU sharding) */
    int selfplay;            /* 1: trees play games (spl_mcts_reset_games / spl_mcts_commit) */
    int out_cap;             /* self-play: finished-example queue capacity (examples) */
    int node_boards;         /* 1: keep every node's canonical board (8 x rows bytes per node
                                slot), so a descent through linked edges skips the in-tree
                                transition (getNextState, MCTS.py:155-157) — the descent then
                                runs one transition per simulation instead of one per level */
    long long pool_nodes;    /* node slots shared by all B trees (0: B x node_cap) */
    long long pool_edges;    /* edge units shared by all B trees (0: B x edge_cap). Trees draw
                                node pages (64 slots) and edge pages (2048 units) from these
                                pools on demand and return them when garbage is collected, so
                                memory follows the sum of the live trees, not B x the largest */
} spl_mcts_config;

int spl_mcts_create(const spl_ctx *ctx, int B, const spl_mcts_config *cfg, spl_mcts **out);
int spl_mcts_destroy(spl_mcts *m);
/* HBM bytes of the whole search arena: the shared node / edge pools, per tree its page
 * tables, transposition table (power of two >= node_cap / 0.7) and path, + self-play buffers. plan_bytes: the same figure before creating it (pool
 * sizing by the caller); device_bytes: of a created arena. */
long long spl_mcts_plan_bytes(const spl_ctx *ctx, int B, const spl_mcts_config *cfg);
long long spl_mcts_device_bytes(const spl_mcts *m);
/* roots: B canonical boards (device). keep_tree: look the root up in the persistent
 * transposition table and keep its subtree (exact GC of unreachable nodes). */
int spl_mcts_set_roots(spl_mcts *m, const int8_t *roots, int keep_tree, int force_full,
                       void *hip_stream);
/* same, for the trees with active[t] != 0 only (active: B u8, device; NULL = all). Inactive
 * trees keep their tree untouched and get no search budget: Arena's per-player MCTS
 * objects (Arena.py:94-160) search only on their own turns. */
int spl_mcts_set_roots_active(spl_mcts *m, const int8_t *roots, const uint8_t *active, int keep_tree,
                              int force_full, void *hip_stream);
/* Arena move choice (the Arena players of Coach.py:152-153: np.argmax(getActionProb(x, temp=0)[0]),
 * MCTS.py:87-92): per active tree, the action with the largest (pruned) root count, ties
 * broken uniformly by Philox (cfg.seed, board_base + t, ST_BEST | stream, draw 0) with
 * ST_BEST = 6 << 24 and stream < 2^24 (the caller's game id base and ply), written to
 * action[t] (B i16, device). */
int spl_mcts_pick_best(spl_mcts *m, const uint8_t *active, uint32_t board_base, uint32_t stream,
                       int16_t *action, void *hip_stream);
/* leaf_state: B x S int8, leaf_mask: B x 7 u64, leaf_valid: B u8 (1 = needs the network) */
int spl_mcts_select(spl_mcts *m, int8_t *leaf_state, uint64_t *leaf_mask, uint8_t *leaf_valid,
                    void *hip_stream);
/* select + the trees whose leaf needs the network listed segment by segment (ABI 11):
 * segment j = trees 64 j .. 64 j + 63; leaf_count (device, ceil(B / 64) i32, 16-byte aligned)
 * holds each segment's number of such trees and leaf_index (device, B i32) their ids at
 * leaf_index[64 j .. 64 j + leaf_count[j]) in no particular order; the list is the segments'
 * entries in segment order. Pair with spl_nn_forward_indexed so the network runs on those
 * leaves only (terminal leaves and idle trees need no evaluation: ~30 % of all trees per
 * iteration at BASELINE config 3's steady state). (ABI 10 kept one compact list and one count:
 * every 64-tree workgroup then took its place with a returning atomic on one counter.) */
int spl_mcts_select_compact(spl_mcts *m, int8_t *leaf_state, uint64_t *leaf_mask, uint8_t *leaf_valid,
                            int32_t *leaf_index, int32_t *leaf_count, void *hip_stream);
/* pi: B x 409 f32 (policy over all actions, as predict returns), v: B x n f32 */
int spl_mcts_backup(spl_mcts *m, const uint64_t *leaf_mask, const float *pi, const float *v,
                    void *hip_stream);
/* spl_mcts_backup for the trees whose leaf is of the given kinds only (bit 0: NN leaves, the
 * expansion + backup of MCTS.py:134-176; bit 1: terminal leaves, :125-131 then :169-176).
 * Trees are independent, so a caller may back up the terminal leaves on a second stream
 * while the network evaluates the NN leaves (their backup needs no pi / v: NULL allowed). */
#define SPL_LEAF_NN 1
#define SPL_LEAF_TERMINAL 2
/* kinds | SPL_BACKUP_DEFER_GC (self-play handles, ABI 10): no collection launch for the trees
 * whose simulation was withdrawn (a leaf that did not fit); the caller runs spl_mcts_commit
 * before the next select, and the collection it launches takes them. The self-play driver
 * backs up this way: one k_gc launch per iteration instead of two (~5 us, empty at steady
 * state). Without it, or without a commit before the next select, collect as before. */
#define SPL_BACKUP_DEFER_GC 4
int spl_mcts_backup_kind(spl_mcts *m, const uint64_t *leaf_mask, const float *pi, const float *v, int kinds,
                         void *hip_stream);
/* counts B x 409 i64 (root visit counts Nsa), qsa B x 409 f64 (-42 = unvisited), probs
 * B x 409 f64 (temp = 1), q B x n f64, adjusted B x 409 i64 (counts after policy-target
 * pruning, MCTS.py:69-74; = counts without forced playouts); any may be NULL */
/* ps: B x 409 f32, the root's stored priors Ps (nodes_data[s][2], MCTS.py:147/176: after
 * root Dirichlet noise when it was applied), 0 for illegal actions and for trees without a
 * root. */
int spl_mcts_root_priors(spl_mcts *m, float *ps, void *hip_stream);
int spl_mcts_root_stats(spl_mcts *m, int64_t *counts, double *qsa, double *probs, double *q,
                        int64_t *adjusted, void *hip_stream);
/* ---- self-play (Coach.executeEpisode, Coach.py:50-100), selfplay=1 only ----
 * reset_games: deal B new games (Board.init_game via Philox) and start their searches.
 * commit: for every tree whose search budget is spent, play the move on device:
 *   pi = root visit counts (pruned if forced playouts), record (board, player, pi, valids,
 *   q) if it was a full search, sample the action with temperature 2 before tempThreshold
 *   moves and 0.2 after (Coach.py:19-33, 82-83), getNextState with chance, getGameEnded;
 *   on game end write every example of the game with winner = roll(r, -player) and
 *   score difference (Coach.py:89-98) to the example queue and deal a new game; re-root
 *   the tree at the next canonical board (exact GC) and draw the next search type. */
int spl_mcts_reset_games(spl_mcts *m, void *hip_stream);
/* restart_games: like reset_games for the games with restart[t] != 0 only (restart: B u8,
 * device): each abandons its current game (examples staged for it are discarded; nothing
 * is written to the example queue) and is dealt its next game (game number + 1), with a
 * fresh tree. Call between iterations. Not in the reference (its episodes run one after
 * another): the batched driver uses it to spread B games that started together over the
 * phases of a game (bench warm-up). */
int spl_mcts_restart_games(spl_mcts *m, const uint8_t *restart, void *hip_stream);
int spl_mcts_commit(spl_mcts *m, void *hip_stream);
/* copy up to `max` finished examples to caller buffers (state E x S i8, pi E x 409 f32,
 * valid E x 7 u64, winner E x n f32, scdiff E x n i32, q E x n f32, meta E x 4 i32 =
 * (global board id, game number, example index in game, player)), write the count to
 * *n_out (device int32) and empty the queue (examples beyond `max` are dropped). Any
 * output pointer may be NULL. */
/* out (device, 2 x i32): [0] finished examples waiting in the queue, [1] examples dropped
 * so far because the queue (out_cap) was full when their game ended or a drain asked for
 * fewer than were queued. Self-play arenas only. */
int spl_mcts_counters(spl_mcts *m, int32_t *out, void *hip_stream);
/* out (device, 4 x i32): free node pages, free edge pages, node / edge page requests that
 * found the pool empty so far (each such leaf was withdrawn for collection or counted as
 * unexpanded in its tree's header). pool_pages (host): pages in the node / edge pools and
 * their sizes (node slots / edges per page). */
int spl_mcts_pool_state(spl_mcts *m, int32_t *out, void *hip_stream);
int spl_mcts_pool_pages(const spl_mcts *m, long long *out4);   /* pages, pages, NPG, units/page */
int spl_mcts_drain_examples(spl_mcts *m, int8_t *state, float *pi, uint64_t *valid,
                            float *winner, int32_t *scdiff, float *q, int32_t *meta, int max,
                            int32_t *n_out, void *hip_stream);
/* copies the B per-tree headers (208 bytes each, layout in splendor/mcts.py) to `out` */
int spl_mcts_headers(spl_mcts *m, int32_t *out, void *hip_stream);

/* out B x 4 i32 per tree: node slots used, edge slots used, live nodes (the root and every
 * node whose round exceeds the root's: what garbage collection keeps, MCTS.py:79-85) and
 * their edges. Capacity planning diagnostic (tools/tree_sizes.py). */
int spl_mcts_tree_sizes(spl_mcts *m, int32_t *out, void *hip_stream);

/* predict input conversion (GenericNNetWrapper.py:160-161): int8 boards [B][R][7] -> f32
 * written transposed as x[B][7][R] (SplendorNNet.py:129 layout), packed mask -> bool bytes
 * (valid may be NULL) */
int spl_nn_input(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask,
                 float *x, uint8_t *valid, void *hip_stream);
/* deterministic hash-prior network (see oracle or_fake_predict): parity tests and
 * tree-only throughput runs. spl_hash_eval = mode 0 (spread priors, values in [-1, 1));
 * mode 1: peaked priors, values near +-1 (deep trees like the random-init SplendorNNet's) */
int spl_hash_eval(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask,
                  float *pi, float *v, void *hip_stream);
int spl_hash_eval_mode(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask,
                       float *pi, float *v, int mode, void *hip_stream);

/* ===================================================================== network
 * SplendorNNet inference (SplendorNNet.py:56-159 in eval mode; GenericNNetWrapper.predict
 * :141-168 minus the host round trip) as one fused kernel: int8 boards [B][R][7] + packed
 * masks [B][7] -> pi [B][409] = softmax(masked logits, invalid -> -1e8) and v [B][n] =
 * tanh(value head). f32 arithmetic on bf16 MFMAs, every f32 operand split exactly into three
 * bf16 parts (six products per chunk, the largest in its own f32 accumulator): the per-column
 * layers on v_mfma_f32_32x32x16_bf16, the per-leaf layers on v_mfma_f32_16x16x32_bf16
 * (DESIGN.md §4).
 *
 * packed_weights: spl_nn_packed_floats(n) floats, 16-byte aligned, the eval-mode network
 * with BatchNorms folded (splendor/nnet.py pack_weights). For each of the 13 linear layers
 * (N outputs, K inputs) in the order dense2d_1[0], dense2d_1[3], partialgpool_1 dense,
 * dense2d_3, dense1d_4, partialgpool_4 dense, dense1d_5[0], dense1d_5[3], partialgpool_5
 * dense, output_layers_PI[0], [1], output_layers_V[0], [1]:
 *     Kp = K rounded up to 8; NT = ceil(N / T)
 *     first 4 layers (T = 32, v_mfma_f32_32x32x2_f32, K in 2 halves of S = Kp / 2):
 *         weights [NT][S/4][64][4]: element (nt, q, l, j) = W[32 nt + l % 32][4 q + j + (l / 32) S]
 *     other 9 (T = 16, v_mfma_f32_16x16x4_f32, Kp a multiple of 16, k groups interleaved):
 *         weights [NT][Kp/16][64][4]: element (nt, q, l, j) = W[16 nt + l % 16][16 q + 4 (l / 16) + j]
 *     (0 outside N x K)
 *     bias    [T NT] (0-padded)
 * then the per-board-column BatchNorm affines of dense2d_1 and partialgpool_1:
 * s1[7], t1[7], sp1[7], tp1[7] (y = x * s + t); then, from the next 16-byte boundary, the
 * 13 layers again as exact three-part bf16 splits (w = hi + mid + lo by truncation) for the
 * bf16-MFMA form of those layers: the first 5 (the per-column layers and dense1d_4, whose
 * weights are the A operand of v_mfma_f32_32x32x16_bf16) per layer [4][Kp16/16][3][64][8] bf16 (Kp16 = K rounded
 * up to 16), element (nt, c, p, l, j) = part p of W[32 nt + l % 32 - o][16 c + 8 (l / 32) + j]
 * (o = 8 for partialgpool_1, whose outputs follow its 8 pooled channels, else 0; 0 outside),
 * two bf16 per float slot; then the other 8 layers the same way for 16x16x32: per layer
 * [NT16][Kp32/32][3][64][8] bf16 (NT16 = ceil(N / 16), Kp32 = K rounded up to 32), element
 * (nt, c, p, l, j) = part p of W[16 nt + l % 16][32 c + 8 (l / 16) + j]. The f32 copies of the
 * 13 layers stay in the layout (the biases are read from them). Returns the float count or
 * SPL_EINVAL. */
int spl_nn_packed_floats(int n_players);
int spl_nn_forward(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                   const float *packed_weights, float *pi, float *v, void *hip_stream);
/* the same network on the rows listed by leaf_index / leaf_count only, in the segmented form
 * spl_mcts_select_compact writes (B = the number of trees: ceil(B / 64) segment counts,
 * leaf_count 16-byte aligned): boards, masks and outputs of row r = every listed leaf_index
 * entry; other rows of pi / v are left untouched. */
int spl_nn_forward_indexed(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                           const int32_t *leaf_index, const int32_t *leaf_count, const float *packed_weights,
                           float *pi, float *v, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
