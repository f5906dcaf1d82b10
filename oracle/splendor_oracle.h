/*
 * splendor_oracle.h — CPU restatement of the reference Splendor hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the HIP product
 * (alphazero-general-ori_amd/csrc) and the timed CPU baseline in bench.py. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product never links, imports or calls it.
 *
 * Pinning: every function below is checked bit-exactly against golden vectors that
 * tests/golden/make_golden.py records from the reference itself (executed in the build
 * container from /root/reference text with the in-memory patches listed there).
 *
 * Reference semantics followed (file:line in /root/reference):
 *   state layout / copy_state          SplendorLogicNumba.py:291-303
 *   init_game                          SplendorLogicNumba.py:222-246
 *   valid_moves                        SplendorLogicNumba.py:251-265 (+ helpers :476-680)
 *   make_move                          SplendorLogicNumba.py:267-289 (+ helpers :400-768)
 *   check_end_game / judge / get_score SplendorLogicNumba.py:320-334, :306-318, :217-220
 *   swap_players                       SplendorLogicNumba.py:338-347
 *   get_symmetries                     SplendorLogicNumba.py:349-395
 *   MCTS.search / getActionProb        MCTS.py:45-177, pick_highest_UCB MCTS.py:199-219
 */
#ifndef SPLENDOR_ORACLE_H
#define SPLENDOR_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define OR_ACTIONS 409

int  or_rows(int n);                                   /* 32 + 10n + n^2 */
/* chance draws: u[] is consumed in order; *used receives the count. */
void or_init(int n, int8_t *state, const double *u, int *used);
void or_valid_moves(int n, const int8_t *state, int player, uint8_t *mask /*409*/);
int  or_make_move(int n, int8_t *state, int action, int player, int deterministic,
                  const double *u, int *used);
void or_check_end(int n, const int8_t *state, float *out /*n*/);
void or_swap_players(int n, int8_t *state, int k);
int  or_get_score(int n, const int8_t *state, int player);
int  or_get_round(const int8_t *state);
/* card table access for table pinning: writes (cost row, gain row) = 14 bytes */
void or_card(int tier, int color, int k, int8_t *out14);
/* in-tree transition (MCTS.py:222-237): copy, make_move(a,0,det=1), swap(next) */
int  or_tree_step(int n, const int8_t *parent, int action, int8_t *child);
/* symmetries (SplendorLogicNumba.py:349-395). Writes up to 1+9+2n variants; returns count. */
int  or_symmetries(int n, const int8_t *state, const float *pi, const uint8_t *valids,
                   int8_t *out_states, float *out_pi, uint8_t *out_valids);

/* counter-based chance source shared with the device: Philox4x32-10 */
void   or_philox4x32(uint32_t key0, uint32_t key1, const uint32_t ctr[4], uint32_t out[4]);
double or_uniform(uint64_t seed, uint32_t board, uint32_t stream, uint32_t draw);

/* deterministic stand-in network used for search parity (see make_golden.py) */
uint64_t or_state_hash(const int8_t *state, int bytes);
void or_fake_predict(int n, const int8_t *state, const uint8_t *valids, float *pi, float *v);
/* hash network mode: 0 spread priors / values (default), 1 peaked priors (w/max w)^256 and
 * values near +-1 (deep trees, see the .c) */
void or_set_fake_mode(int mode);
/* leaf depth statistics of every search since the last reset: sum, max, simulations */
void or_depth_stats(long long *out3, int reset);
/* numpy float32 pairwise sum (np.sum order, pinned in tests) */
float or_np_sum_f32(const float *x, int len);

/* Root Dirichlet noise (MCTS.py:141-154, 180-186, 239-250). or_dirichlet: this build's
 * Philox Gamma sampler (counters i*4096 for valid action i), normalised like numpy's
 * Generator.dirichlet. or_root_noise: softmax(ps, temp0) -> 0.75/0.25 mix with dir over the
 * valid actions -> normalise, in place on ps[409]. */
void or_dirichlet(double alpha, uint64_t seed, uint32_t board, uint32_t stream, int count, double *out);
void or_root_noise(float *ps, const uint8_t *vs, const double *dir, double temp0);

/* Sequential MCTS (one tree), fake network. Mirrors MCTS.getActionProb; root noise when
 * or_mcts_set_noise gave alpha > 0 (applied at step 0 of every search). Tree persists
 * across calls until or_mcts_free. */
typedef struct or_mcts or_mcts;
or_mcts *or_mcts_new(int n, int num_sims, double cpuct, double fpu, int forced_playouts);
/* neg_v: the hash network with negated values (a second, different network) */
void     or_mcts_set_net(or_mcts *m, int neg_v);
void     or_mcts_set_noise(or_mcts *m, double alpha, double temp0, uint64_t seed, uint32_t board,
                           uint32_t stream);
void     or_mcts_free(or_mcts *m);
/* runs a full search from root (canonical). counts[409] (int64), qsa[409] (f64),
 * probs[409] (f64, temp=1), q[n] (f64). Returns number of nodes in the table. */
int or_mcts_search(or_mcts *m, const int8_t *root, int64_t *counts, double *qsa,
                   double *probs, double *q);

/* Coach.executeEpisode self-play with the hash network, one simulation per iteration per
 * game (device spl_mcts_commit semantics). Returns the number of finished examples
 * (written up to max_ex). hdr_out: B x 8 (player, episode_step, move_no, game_no,
 * games_done, moves, sims_done, budget). */
int or_selfplay_run(int n, int B, int iters, uint64_t seed, uint32_t board_base, int num_sims,
                    int ratio_full, double prob_full, double cpuct, double fpu, int forced_po,
                    int temp_threshold, double dir_alpha, double dir_temp, int8_t *board_out,
                    int32_t *hdr_out, int max_ex, int8_t *ex_state, float *ex_pi, uint64_t *ex_valid,
                    float *ex_winner, int32_t *ex_scdiff, float *ex_q, int32_t *ex_meta);

/* random-policy rollout loop used as the CPU baseline: B boards, steps steps each,
 * mask -> uniform valid action -> chance step -> end check -> reset on end.
 * Returns total board-steps executed. threads<=0 => 1. */
long long or_random_rollouts(int n, int B, int steps, uint64_t seed, int threads);
/* same loop with traces (spl_rollout_step semantics, include/splendor_amd.h); NULL skips.
 * masks: steps x B x 7 legality words of every move (mask_fold: their per-board fold) */
long long or_rollout_run(int n, int B, int steps, uint64_t seed, uint32_t board_base,
                         int8_t *state_out, int8_t *player_out, int16_t *actions,
                         float *ended, int32_t *games, uint64_t *mask_fold, uint64_t *masks);

#ifdef __cplusplus
}
#endif
#endif
