/* Host sanitizer run of the CPU oracle (test infrastructure): AddressSanitizer +
 * UndefinedBehaviorSanitizer over every entry point the parity tests drive — random
 * rollouts with traces (2-4 players, threaded), sequential MCTS with root noise,
 * self-play episodes with examples, symmetries. Any report aborts (make sanitize:
 * -fno-sanitize-recover=all). Run by tests/test_sanitize.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "splendor_oracle.h"

#define ACT 409

static int run_players(int n) {
    const int R = or_rows(n), S = R * 7, B = 24, T = 400;
    int8_t *st = calloc((size_t)B * S, 1), *pl = calloc(B, 1);
    int16_t *act = calloc((size_t)B * T, sizeof(int16_t));
    float *end = calloc((size_t)B * T * n, sizeof(float));
    int32_t *games = calloc(B, sizeof(int32_t));
    uint64_t *fold = calloc(B, sizeof(uint64_t));
    if (or_rollout_run(n, B, T, 0x5EED + n, 0, st, pl, act, end, games, fold, NULL) <= 0) return 1;
    if (or_random_rollouts(n, 64, 200, 7 + n, 2) <= 0) return 1;

    /* symmetries and MCTS (with root noise) from the rollout's final boards */
    float pi[ACT], *spi = malloc(sizeof(float) * ACT * 64);
    uint8_t vm[ACT], *svm = malloc((size_t)ACT * 64);
    int8_t *sst = malloc((size_t)S * 64);
    int64_t counts[ACT];
    double qsa[ACT], probs[ACT], q[4];
    for (int b = 0; b < 4; b++) {
        int8_t *s = st + (size_t)b * S;
        or_valid_moves(n, s, 0, vm);
        for (int a = 0; a < ACT; a++) pi[a] = vm[a] ? 1.f : 0.f;
        or_symmetries(n, s, pi, vm, sst, spi, svm);
        or_mcts *m = or_mcts_new(n, 48, 2.5, 0.3, b & 1);
        or_mcts_set_noise(m, 0.3, 1.25, 11, (uint32_t)b, 0);
        or_mcts_search(m, s, counts, qsa, probs, q);
        or_mcts_search(m, s, counts, qsa, probs, q);
        or_mcts_free(m);
    }

    /* self-play: a few games to the end, examples assembled */
    const int SB = 3, ITERS = 6000, MAXEX = 4096;
    int8_t *bo = malloc((size_t)SB * S), *exs = malloc((size_t)MAXEX * S);
    int32_t *hdr = malloc(sizeof(int32_t) * SB * 8), *exd = malloc(sizeof(int32_t) * MAXEX * n);
    int32_t *exm = malloc(sizeof(int32_t) * MAXEX * 8);
    float *exp_ = malloc(sizeof(float) * (size_t)MAXEX * ACT), *exw = malloc(sizeof(float) * MAXEX * n);
    float *exq = malloc(sizeof(float) * MAXEX * n);
    uint64_t *exv = malloc(sizeof(uint64_t) * MAXEX * 7);
    const int ex = or_selfplay_run(n, SB, ITERS, 3 + n, 0, 16, 4, 0.25, 2.5, 0.3, 1, 10, 0.3, 1.25, bo, hdr,
                                   MAXEX, exs, exp_, exv, exw, exd, exq, exm);
    printf("%dp: %d examples, %d games\n", n, ex, hdr[4] + hdr[8 + 4] + hdr[16 + 4]);
    free(fold); free(st); free(pl); free(act); free(end); free(games); free(spi); free(svm); free(sst);
    free(bo); free(exs); free(hdr); free(exd); free(exm); free(exp_); free(exw); free(exq); free(exv);
    return ex < 0;
}

int main(void) {
    for (int n = 2; n <= 4; n++)
        if (run_players(n)) { fprintf(stderr, "%dp: oracle call failed\n", n); return 1; }
    printf("sanitize ok\n");
    return 0;
}
