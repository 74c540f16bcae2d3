/*
 * azg_mcts.h -- C-ABI of the native multi-game batched-leaf MCTS (host C++).
 *
 * Reproduces reference mcts/new_mcts_alpha.py:77-197 (PUCT with Q = W/(1+N),
 * leaf queue of batch_size, no virtual loss, prior = p*valid without
 * renormalisation, uniform fallback, root-only Dirichlet, N/W reset on install,
 * tree reuse across moves, key = board bytes + side to move) bit for bit,
 * including numpy's float32/float64 promotion rules in the PUCT score, for
 * Gomoku (games/gomoku.py) and Pente (games/pente.py), over many games at once:
 * every game owns its own tree; `azg_mcts_advance` runs all games (in parallel
 * over host threads) until each one needs its pending leaves evaluated, and hands
 * back ONE contiguous batch of encoded boards for a single GPU forward.
 *
 * Randomness stays with the caller (numpy), so RNG streams match the reference:
 * the Dirichlet mix of a root prior is done by the caller (azg_mcts_noise_request /
 * azg_mcts_set_root_prior), and so is move sampling.
 *
 * All pointers are HOST pointers.  Return 0 = ok, nonzero = error
 * (azg_mcts_last_error).  Not re-entrant per handle.
 */
#ifndef AZG_MCTS_H
#define AZG_MCTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct azg_mcts azg_mcts;

typedef struct {
    int32_t rules;                 /* 0 = Gomoku, 1 = Pente */
    int32_t board;                 /* 15 */
    int32_t n_simulations;
    int32_t batch_size;            /* reference default 32 */
    int32_t apply_dirichlet_n_first_moves;
    int32_t add_dirichlet_noise;
    double cpuct;
    double dirichlet_alpha;        /* informational: the caller draws the noise */
    double epsilon;                /* informational: the caller mixes the noise */
} azg_mcts_config;

/* per-game status after azg_mcts_advance */
enum {
    AZG_MCTS_IDLE = 0,        /* no search in progress                             */
    AZG_MCTS_NEED_EVAL = 1,   /* leaves emitted; call azg_mcts_feed                 */
    AZG_MCTS_DONE = 2         /* this move's search finished; azg_mcts_get_pi       */
};

const char* azg_mcts_last_error(void);
int32_t azg_mcts_create(const azg_mcts_config* cfg, int32_t n_games, azg_mcts** out);
int32_t azg_mcts_destroy(azg_mcts* h);

/* Start the search of one move for game g from this position (reference run():
 * root_key = key(position)).  board: int8 [size*size] (0/1/2); last move (-1,-1)
 * for none; captures only for Pente; move_number = len(move_history) as passed by
 * the reference callers (drives the Dirichlet condition). */
int32_t azg_mcts_set_root(azg_mcts* h, int32_t g, const int8_t* board, int32_t player, int32_t last_r,
                          int32_t last_c, int32_t cap1, int32_t cap2, int32_t move_number);

/* Run every game with a search in progress until it needs an evaluation or its
 * move is done.  Writes the pending leaves of all games, in game order, as
 * float32 [n][3][size][size] (reference get_encoded_state) into `leaves`
 * (capacity n_games*batch_size boards), per-game leaf counts into `counts`
 * [n_games] and per-game status into `status` [n_games]; returns n via *n_out.
 * n_threads <= 0: use all host threads. */
int32_t azg_mcts_advance(azg_mcts* h, float* leaves, int32_t* counts, int32_t* status, int32_t* n_out,
                         int32_t n_threads);

/* Same as azg_mcts_advance, but the leaves are written as int8 boards [n][size*size]
 * (0 empty, 1, 2) and the side to move [n] (1|2), for the on-GPU encoding of
 * azg_pv_forward_boards (capacity n_games*batch_size boards). */
int32_t azg_mcts_advance_boards(azg_mcts* h, int8_t* boards, int8_t* players, int32_t* counts, int32_t* status,
                                int32_t* n_out, int32_t n_threads);

/* Install the evaluation of the last emitted leaves (same order): probs
 * float32 [n][size*size], values float32 [n] (stored, unused by the search,
 * as in the reference). */
int32_t azg_mcts_feed(azg_mcts* h, const float* probs, const float* values);

/* After azg_mcts_feed: if game g's root was just installed under the Dirichlet
 * condition, returns 1 and copies its masked float32 prior into p (size*size);
 * the caller must then call azg_mcts_set_root_prior with the float64 mixed prior
 * ((1-eps)*p + eps*noise, renormalised) before the next azg_mcts_advance. */
int32_t azg_mcts_noise_request(azg_mcts* h, int32_t g, float* p);
int32_t azg_mcts_set_root_prior(azg_mcts* h, int32_t g, const double* p64);

/* pi = N/sum(N) at the root (float32), or the valid mask normalised. */
int32_t azg_mcts_get_pi(azg_mcts* h, int32_t g, float* pi);

/* Forget game g's tree (reference clear_tree). */
int32_t azg_mcts_clear(azg_mcts* h, int32_t g);
int64_t azg_mcts_tree_size(const azg_mcts* h, int32_t g);

/* Rule-engine known-answer hook (the search's own State): from `start` (board*board
 * int8, NULL = empty), side to move `player` and captured pairs (cap1, cap2), play
 * `actions[0..n)` with the Gomoku (rules 0, games/gomoku.py:60-193) or Pente (rules
 * 1, games/pente.py:57-230) rules; after each move k write the board
 * (boards_out[k], may be NULL), the captured-pair counts (caps_out[2k..2k+1]), the
 * winner and the game-over flag.  Fails on an illegal move. */
int32_t azg_mcts_replay(int32_t rules, int32_t board, const int8_t* start, int32_t player, int32_t cap1,
                        int32_t cap2, const int32_t* actions, int32_t n, int8_t* boards_out, int32_t* caps_out,
                        int32_t* winner_out, int32_t* over_out);

#ifdef __cplusplus
}
#endif
#endif /* AZG_MCTS_H */
