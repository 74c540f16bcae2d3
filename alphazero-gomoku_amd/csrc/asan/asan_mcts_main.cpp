// Host AddressSanitizer / UBSan driver of the native search (include/azg_mcts.h,
// csrc/mcts_engine.cpp), SURVEY §5: several games of Gomoku and Pente played to
// the end through the C-ABI with a deterministic stand-in evaluator (both leaf
// formats, Dirichlet root priors, multi-threaded advance, tree reuse and clear),
// the rule-replay hook, and every error path.  Built by `make -C csrc asan`.
#include "../../../include/azg_mcts.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                    \
        }                                                               \
    } while (0)

static void fake_eval(const int8_t* boards, const int8_t* players, int n, int A, std::vector<float>& p,
                      std::vector<float>& v)
{
    p.assign((size_t)n * A, 0.f);
    v.assign(n, 0.f);
    for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int a = 0; a < A; ++a) {
            const int8_t b = boards[(size_t)i * A + a];
            const float x = b == 0 ? 1.f + 0.5f * std::sin(0.37f * a + 0.11f * i) : 0.f;
            p[(size_t)i * A + a] = x;
            s += x;
        }
        for (int a = 0; a < A; ++a) p[(size_t)i * A + a] = (float)(p[(size_t)i * A + a] / (s > 0 ? s : 1));
        v[i] = players[i] == 1 ? 0.1f : -0.1f;
    }
}

static void play(int rules, int games, int sims, bool boards_mode, int threads)
{
    azg_mcts_config cfg{};
    cfg.rules = rules;
    cfg.board = 15;
    cfg.n_simulations = sims;
    cfg.batch_size = 8;
    cfg.apply_dirichlet_n_first_moves = 4;
    cfg.add_dirichlet_noise = 1;
    cfg.cpuct = 1.2;
    cfg.dirichlet_alpha = 0.3;
    cfg.epsilon = 0.25;
    azg_mcts* h = nullptr;
    CHECK(azg_mcts_create(&cfg, games, &h) == 0 && h);
    const int A = 225;
    std::vector<std::vector<int8_t>> board(games, std::vector<int8_t>(A, 0));
    std::vector<int> player(games, 1), moves(games, 0), lastm(games, -1), done(games, 0);
    std::vector<int> caps(2 * games, 0);
    for (int g = 0; g < games; ++g) CHECK(azg_mcts_set_root(h, g, board[g].data(), 1, -1, -1, 0, 0, 0) == 0);
    std::vector<float> leaves((size_t)games * cfg.batch_size * 3 * A), p, v, pi(A);
    std::vector<int8_t> lb((size_t)games * cfg.batch_size * A), lp((size_t)games * cfg.batch_size);
    std::vector<int32_t> counts(games), status(games);
    int live = games, rounds = 0;
    while (live > 0 && rounds < 20000) {
        ++rounds;
        int32_t n = 0;
        if (boards_mode) {
            CHECK(azg_mcts_advance_boards(h, lb.data(), lp.data(), counts.data(), status.data(), &n, threads) == 0);
        } else {
            CHECK(azg_mcts_advance(h, leaves.data(), counts.data(), status.data(), &n, threads) == 0);
            // rebuild int8 boards from the float planes for the stand-in evaluator
            for (int i = 0; i < n; ++i)
                for (int a = 0; a < A; ++a) {
                    const float cur = leaves[((size_t)i * 3 + 0) * A + a], opp = leaves[((size_t)i * 3 + 1) * A + a];
                    lb[(size_t)i * A + a] = cur > 0 ? 1 : (opp > 0 ? 2 : 0);
                    lp[i] = 1;
                }
        }
        for (int g = 0; g < games; ++g) {
            if (done[g] || status[g] != AZG_MCTS_DONE) continue;
            CHECK(azg_mcts_get_pi(h, g, pi.data()) == 0);
            int best = -1;
            for (int a = 0; a < A; ++a)
                if (board[g][a] == 0 && (best < 0 || pi[a] > pi[best])) best = a;
            CHECK(best >= 0);
            // advance the true game with the native rules (replay hook)
            int8_t nb[A];
            int32_t cp[2], w = 0, over = 0;
            const int32_t act = best;
            CHECK(azg_mcts_replay(rules, 15, board[g].data(), player[g], caps[2 * g], caps[2 * g + 1], &act, 1, nb,
                                  cp, &w, &over) == 0);
            std::memcpy(board[g].data(), nb, A);
            caps[2 * g] = cp[0];
            caps[2 * g + 1] = cp[1];
            player[g] = 3 - player[g];
            lastm[g] = best;
            ++moves[g];
            if (over || moves[g] >= 60) {
                done[g] = 1;
                --live;
                CHECK(azg_mcts_tree_size(h, g) > 0);
                CHECK(azg_mcts_clear(h, g) == 0);
                CHECK(azg_mcts_tree_size(h, g) == 0);
            } else {
                CHECK(azg_mcts_set_root(h, g, board[g].data(), player[g], best / 15, best % 15, caps[2 * g],
                                        caps[2 * g + 1], moves[g]) == 0);
            }
        }
        if (n > 0) {
            fake_eval(lb.data(), lp.data(), n, A, p, v);
            CHECK(azg_mcts_feed(h, p.data(), v.data()) == 0);
            for (int g = 0; g < games; ++g) {
                std::vector<float> p32(A);
                if (azg_mcts_noise_request(h, g, p32.data()) == 1) {
                    std::vector<double> mix(A);
                    double s = 0;
                    for (int a = 0; a < A; ++a) s += (mix[a] = 0.75 * p32[a] + 0.25 / A);
                    for (auto& m : mix) m /= s;
                    CHECK(azg_mcts_set_root_prior(h, g, mix.data()) == 0);
                }
            }
        }
    }
    CHECK(live == 0);
    CHECK(azg_mcts_destroy(h) == 0);
    std::printf("rules %d games %d sims %d boards %d threads %d: %d rounds\n", rules, games, sims, (int)boards_mode,
                threads, rounds);
}

int main()
{
    play(0, 4, 48, true, 4);
    play(0, 3, 33, false, 1);
    play(1, 4, 40, true, 3);
    play(1, 2, 24, false, 2);
    // error paths: bad config, bad game index, illegal replay, use before a search
    azg_mcts_config bad{};
    azg_mcts* h = nullptr;
    CHECK(azg_mcts_create(&bad, 1, &h) != 0 && std::strlen(azg_mcts_last_error()) > 0);
    azg_mcts_config cfg{};
    cfg.rules = 0;
    cfg.board = 15;
    cfg.n_simulations = 8;
    cfg.batch_size = 4;
    cfg.cpuct = 1.0;
    CHECK(azg_mcts_create(&cfg, 1, &h) == 0);
    float pi[225];
    CHECK(azg_mcts_get_pi(h, 0, pi) != 0);
    CHECK(azg_mcts_get_pi(h, 5, pi) != 0);
    CHECK(azg_mcts_clear(h, -1) != 0);
    const int32_t twice[2] = {7, 7};
    int32_t cp[4], w[2], o[2];
    CHECK(azg_mcts_replay(0, 15, nullptr, 1, 0, 0, twice, 2, nullptr, cp, w, o) != 0);
    CHECK(azg_mcts_replay(2, 15, nullptr, 1, 0, 0, twice, 1, nullptr, cp, w, o) != 0);
    CHECK(azg_mcts_destroy(h) == 0);
    CHECK(azg_mcts_destroy(nullptr) == 0);
    std::printf("asan_mcts: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
