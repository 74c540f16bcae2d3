// Native multi-game batched-leaf MCTS (include/azg_mcts.h), host C++17.
//
// Semantics are those of reference mcts/new_mcts_alpha.py:77-197 and
// games/gomoku.py / games/pente.py, reproduced bit for bit:
//   * PUCT score exactly as numpy evaluates
//       W/(1+N) + cpuct*P*sqrt(sum N)/(1+N), invalid -> -1e9, first argmax,
//     in float32 (python scalars are weak: cast to float32), or in float64 for a
//     root whose prior became float64 through the Dirichlet mix;
//   * N and W are integer-valued (backed-up values are 0/-1/+1: network values are
//     stored but never read by the reference search), kept as int32 here and
//     converted exactly to float32 for the score;
//   * a simulation that fills the leaf queue is suspended and, after the batch is
//     installed, continues descending from the now-evaluated node;
//   * installing resets N/W and overwrites the prior of every queued key.
// Build with -ffp-contract=off (no FMA contraction: numpy rounds every op).
#include "../../include/azg_mcts.h"

#include <omp.h>

#include <array>
#include <cmath>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;
int32_t fail(const std::string& s) { g_err = s; return 1; }

constexpr int MAXN = 15 * 15;

// numpy pairwise summation (float32 accumulation), contiguous input
float np_pairwise_sum_f32(const float* a, long n)
{
    if (n < 8) {
        float r = 0.f;
        for (long i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum_f32(a, n2) + np_pairwise_sum_f32(a + n2, n - n2);
}

struct Key {
    std::array<int8_t, MAXN + 1> b;   // board bytes + side to move
    bool operator==(const Key& o) const { return b == o.b; }
};

struct KeyHash {
    size_t operator()(const Key& k) const
    {
        uint64_t h = 1469598103934665603ull;
        // 8-byte words through memcpy: the key bytes have no 8-byte alignment (a
        // reinterpret_cast load was undefined behaviour -- found by the UBSan driver)
        for (size_t i = 0; i < (MAXN + 1) / 8; ++i) {
            uint64_t wi;
            std::memcpy(&wi, k.b.data() + 8 * i, sizeof(wi));
            h ^= wi;
            h *= 1099511628211ull;
            h ^= h >> 29;
        }
        for (size_t i = (MAXN + 1) / 8 * 8; i < MAXN + 1; ++i) {
            h ^= (uint8_t)k.b[i];
            h *= 1099511628211ull;
        }
        return (size_t)h;
    }
};

struct State {
    int n = 15;
    int rules = 0;
    std::array<int8_t, MAXN> board{};
    int player = 1;
    int last = -1;          // r*n + c or -1
    int cap[3] = {0, 0, 0};

    Key key() const
    {
        Key k;
        std::memcpy(k.b.data(), board.data(), MAXN);
        k.b[MAXN] = (int8_t)player;
        return k;
    }

    bool five_through(int r, int c, int who) const
    {
        static const int dirs[4][2] = {{1, 0}, {0, 1}, {1, 1}, {1, -1}};
        for (auto& d : dirs) {
            int run = 1;
            for (int sgn = 1; sgn >= -1; sgn -= 2) {
                int rr = r + sgn * d[0], cc = c + sgn * d[1];
                while (rr >= 0 && rr < n && cc >= 0 && cc < n && board[rr * n + cc] == who) {
                    ++run;
                    rr += sgn * d[0];
                    cc += sgn * d[1];
                }
            }
            if (run >= 5) return true;
        }
        return false;
    }

    int winner() const   // gomoku.py:155-193 / pente.py:199-230
    {
        if (last < 0) return 0;
        const int r = last / n, c = last % n;
        const int who = board[last];
        if (who == 0) return 0;
        if (rules == 1 && cap[who] >= 5) return who;
        return five_through(r, c, who) ? who : 0;
    }

    bool has_legal() const
    {
        for (int i = 0; i < n * n; ++i)
            if (board[i] == 0) return true;
        return false;
    }

    bool game_over() const { return winner() != 0 || !has_legal(); }

    void do_move(int a)   // gomoku.py:60-78, pente.py:57-78 (+ captures :114-152)
    {
        const int r = a / n, c = a % n, who = player, opp = 3 - who;
        board[a] = (int8_t)who;
        last = a;
        if (rules == 1) {
            static const int dirs[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {1, -1}, {-1, 1}};
            for (auto& d : dirs) {
                const int r3 = r + 3 * d[0], c3 = c + 3 * d[1];
                if (r3 < 0 || r3 >= n || c3 < 0 || c3 >= n) continue;
                const int i1 = (r + d[0]) * n + c + d[1], i2 = (r + 2 * d[0]) * n + c + 2 * d[1];
                if (board[i1] == opp && board[i2] == opp && board[r3 * n + c3] == who) {
                    board[i1] = 0;
                    board[i2] = 0;
                    cap[who] += 1;
                }
            }
        }
        player = opp;
    }

    void encode(float* out) const   // gomoku.py:130-150
    {
        const int A = n * n;
        for (int i = 0; i < A; ++i) {
            out[i] = board[i] == player ? 1.f : 0.f;
            out[A + i] = board[i] == 3 - player ? 1.f : 0.f;
            out[2 * A + i] = 1.f;
        }
    }
};

struct Node {
    std::array<float, MAXN> P{};
    std::unique_ptr<std::array<double, MAXN>> P64;   // float64 prior (Dirichlet-mixed root)
    std::array<int32_t, MAXN> N{};
    std::array<int32_t, MAXN> W{};
    std::array<uint8_t, MAXN> valid{};
    float V = 0.f;
};

// Node storage in fixed chunks: growing never moves a node.  (A std::vector<Node>
// doubled by reallocation: at 16 k nodes of 2.9 KB that is a 47 MB copy per tree,
// and the trees of one forest cross the doubling sizes in the same round -- the
// self-play timeline showed 140-340 ms stalls of one advance call at those rounds.)
class NodeStore {
    static constexpr int kShift = 8, kChunk = 1 << kShift;   // 256 nodes (~750 KB) per chunk
    std::vector<std::unique_ptr<Node[]>> chunks_;
    size_t n_ = 0;

public:
    size_t size() const { return n_; }
    Node& operator[](size_t i) { return chunks_[i >> kShift][i & (kChunk - 1)]; }
    const Node& operator[](size_t i) const { return chunks_[i >> kShift][i & (kChunk - 1)]; }
    void emplace_back()
    {
        if ((n_ >> kShift) == chunks_.size()) chunks_.emplace_back(new Node[kChunk]());
        ++n_;
    }
};

struct Pending {
    Key key;
    State st;
};

struct GameSearch {
    std::unordered_map<Key, int32_t, KeyHash> index;
    NodeStore nodes;
    // current move
    bool active = false;
    State root;
    Key root_key;
    int move_number = 0;
    int sims_left = 0;
    // current simulation
    bool in_sim = false;
    bool suspended = false;
    State cur;
    Key cur_key;
    std::vector<std::pair<int32_t, int32_t>> path;
    // leaf queue
    std::vector<Pending> queue;
    bool final_flush = false;
    int status = AZG_MCTS_IDLE;
    // noise hand-off
    bool noise_pending = false;
    int32_t noise_node = -1;

    int32_t node_for(const Key& k) const
    {
        auto it = index.find(k);
        return it == index.end() ? -1 : it->second;
    }

    int32_t make_node(const Key& k)
    {
        auto it = index.find(k);
        if (it != index.end()) return it->second;
        const int32_t id = (int32_t)nodes.size();
        nodes.emplace_back();
        index.emplace(k, id);
        return id;
    }
};

}  // namespace

struct azg_mcts {
    azg_mcts_config cfg{};
    int A = 225;
    std::vector<GameSearch> games;
};

namespace {

// PUCT choice at a node (new_mcts_alpha.py:135-140) with numpy's dtype rules.
int choose(const azg_mcts* h, const Node& nd)
{
    const int A = h->A;
    float nsum_arr[MAXN];
    for (int i = 0; i < A; ++i) nsum_arr[i] = (float)nd.N[i];
    const float nsum = np_pairwise_sum_f32(nsum_arr, A);
    const double sq = std::sqrt((double)nsum);
    int best = 0;
    if (!nd.P64) {
        const float cp = (float)h->cfg.cpuct, sqf = (float)sq;
        float bv = 0.f;
        for (int i = 0; i < A; ++i) {
            float s;
            if (nd.valid[i] == 1) {
                const float den = 1.0f + (float)nd.N[i];
                const float q = (float)nd.W[i] / den;
                float u = cp * nd.P[i];
                u = u * sqf;
                u = u / den;
                s = q + u;
            } else {
                s = -1e9f;
            }
            if (i == 0 || s > bv) { bv = s; best = i; }
        }
    } else {
        const double cp = h->cfg.cpuct;
        double bv = 0.0;
        for (int i = 0; i < A; ++i) {
            double s;
            if (nd.valid[i] == 1) {
                const float den = 1.0f + (float)nd.N[i];
                const float q = (float)nd.W[i] / den;
                double u = cp * (*nd.P64)[i];
                u = u * sq;
                u = u / (double)den;
                s = (double)q + u;
            } else {
                s = -1e9;
            }
            if (i == 0 || s > bv) { bv = s; best = i; }
        }
    }
    return best;
}

void backup(GameSearch& gs, int v)
{
    // reference: v = -search(child); W[a] += v; N[a] += 1; return v
    for (int i = (int)gs.path.size() - 1; i >= 0; --i) {
        v = -v;
        Node& nd = gs.nodes[gs.path[i].first];
        nd.W[gs.path[i].second] += v;
        nd.N[gs.path[i].second] += 1;
    }
    gs.path.clear();
    gs.in_sim = false;
}

void install_uniform(GameSearch& gs, const Key& k, const State& st, int A)
{
    Node& nd = gs.nodes[gs.make_node(k)];
    int cnt = 0;
    for (int i = 0; i < A; ++i) {
        nd.valid[i] = st.board[i] == 0;
        cnt += nd.valid[i];
    }
    const float fc = (float)cnt;
    for (int i = 0; i < A; ++i) nd.P[i] = (float)nd.valid[i] / fc;
    nd.P64.reset();
    nd.V = 0.f;
    nd.N.fill(0);
    nd.W.fill(0);
}

// Advance one game until it needs an evaluation or its move is done.
void run_game(const azg_mcts* h, GameSearch& gs)
{
    const int A = h->A, bs = h->cfg.batch_size;
    if (!gs.active) { gs.status = AZG_MCTS_IDLE; return; }
    for (;;) {
        if (!gs.in_sim) {
            if (gs.sims_left == 0) {
                if (!gs.queue.empty() && !gs.final_flush) {   // run(): final _predict_batch
                    gs.final_flush = true;
                    break;
                }
                gs.status = AZG_MCTS_DONE;
                gs.active = false;
                return;
            }
            gs.sims_left -= 1;
            gs.in_sim = true;
            gs.suspended = false;
            gs.cur = gs.root;
            gs.path.clear();
        }
        // descend
        bool emitted = false;
        for (;;) {
            Key k;
            if (gs.suspended) {
                k = gs.cur_key;
                gs.suspended = false;
                const int32_t id = gs.node_for(k);
                if (id < 0) {   // (cannot happen: a flush installs every queued key)
                    install_uniform(gs, k, gs.cur, A);
                    backup(gs, 0);
                    break;
                }
            } else {
                k = gs.cur.key();
                if (gs.cur.game_over()) {
                    backup(gs, gs.cur.winner() == 0 ? 0 : -1);
                    break;
                }
                if (gs.node_for(k) < 0) {
                    gs.queue.push_back(Pending{k, gs.cur});
                    if ((int)gs.queue.size() >= bs) {
                        gs.suspended = true;
                        gs.cur_key = k;
                        emitted = true;
                        break;
                    }
                    install_uniform(gs, k, gs.cur, A);
                    backup(gs, 0);
                    break;
                }
            }
            const int32_t id = gs.node_for(k);
            const int a = choose(h, gs.nodes[id]);
            gs.path.emplace_back(id, a);
            gs.cur.do_move(a);
        }
        if (emitted) break;
    }
    gs.status = AZG_MCTS_NEED_EVAL;   // the queue is emitted by the caller (advance_impl)
}

// Run all games (parallel), then write the pending leaves of every game, in game
// order, either as float32 planes or as int8 boards + side to move (parallel copy
// at prefix offsets).
int32_t advance_impl(azg_mcts* h, float* leaves, int8_t* boards, int8_t* players, int32_t* counts,
                     int32_t* status, int32_t* n_out, int32_t n_threads)
{
    const int G = (int)h->games.size();
    for (int g = 0; g < G; ++g)
        if (h->games[g].noise_pending) return fail("azg_mcts_advance: a root prior awaits azg_mcts_set_root_prior");
    const int nt = n_threads > 0 ? n_threads : omp_get_max_threads();
    std::vector<size_t> off(G + 1, 0);
#pragma omp parallel num_threads(nt)
    {
#pragma omp for schedule(dynamic, 1)
        for (int g = 0; g < G; ++g) {
            GameSearch& gs = h->games[g];
            if (gs.status == AZG_MCTS_NEED_EVAL) continue;   // not fed yet: re-emit the same leaves
            run_game(h, gs);
        }
#pragma omp single
        {
            for (int g = 0; g < G; ++g) {
                const GameSearch& gs = h->games[g];
                status[g] = gs.status;
                const int n = gs.status == AZG_MCTS_NEED_EVAL ? (int)gs.queue.size() : 0;
                counts[g] = n;
                off[g + 1] = off[g] + n;
            }
        }
        const int A = h->A;
#pragma omp for schedule(dynamic, 4)
        for (int g = 0; g < G; ++g) {
            const GameSearch& gs = h->games[g];
            const size_t n = off[g + 1] - off[g];
            for (size_t i = 0; i < n; ++i) {
                const size_t row = off[g] + i;
                const State& st = gs.queue[i].st;
                if (leaves) st.encode(leaves + row * 3 * A);
                if (boards) {
                    std::memcpy(boards + row * A, st.board.data(), A);
                    players[row] = (int8_t)st.player;
                }
            }
        }
    }
    *n_out = (int32_t)off[G];
    return 0;
}

}  // namespace

extern "C" {

const char* azg_mcts_last_error(void) { return g_err.c_str(); }

int32_t azg_mcts_create(const azg_mcts_config* cfg, int32_t n_games, azg_mcts** out)
{
    if (!cfg || !out || n_games <= 0) return fail("azg_mcts_create: bad arguments");
    if (cfg->board != 15) return fail("azg_mcts_create: board must be 15");
    if (cfg->rules != 0 && cfg->rules != 1) return fail("azg_mcts_create: rules must be 0 (gomoku) or 1 (pente)");
    if (cfg->batch_size < 1 || cfg->n_simulations < 0) return fail("azg_mcts_create: bad batch/simulations");
    azg_mcts* h = new (std::nothrow) azg_mcts();
    if (!h) return fail("azg_mcts_create: out of memory");
    h->cfg = *cfg;
    h->A = cfg->board * cfg->board;
    h->games.resize(n_games);
    *out = h;
    return 0;
}

int32_t azg_mcts_destroy(azg_mcts* h)
{
    delete h;
    return 0;
}

int32_t azg_mcts_set_root(azg_mcts* h, int32_t g, const int8_t* board, int32_t player, int32_t last_r,
                          int32_t last_c, int32_t cap1, int32_t cap2, int32_t move_number)
{
    if (!h || g < 0 || g >= (int)h->games.size() || !board) return fail("azg_mcts_set_root: bad arguments");
    GameSearch& gs = h->games[g];
    if (gs.active) return fail("azg_mcts_set_root: a search is already in progress for this game");
    State s;
    s.n = h->cfg.board;
    s.rules = h->cfg.rules;
    std::memcpy(s.board.data(), board, h->A);
    s.player = player;
    s.last = (last_r >= 0 && last_c >= 0) ? last_r * s.n + last_c : -1;
    s.cap[1] = cap1;
    s.cap[2] = cap2;
    gs.root = s;
    gs.root_key = s.key();
    gs.move_number = move_number;
    gs.sims_left = h->cfg.n_simulations;
    gs.in_sim = false;
    gs.suspended = false;
    gs.final_flush = false;
    gs.queue.clear();
    gs.path.clear();
    gs.active = true;
    gs.status = AZG_MCTS_IDLE;
    return 0;
}

int32_t azg_mcts_advance(azg_mcts* h, float* leaves, int32_t* counts, int32_t* status, int32_t* n_out,
                         int32_t n_threads)
{
    if (!h || !leaves || !counts || !status || !n_out) return fail("azg_mcts_advance: null argument");
    return advance_impl(h, leaves, nullptr, nullptr, counts, status, n_out, n_threads);
}

int32_t azg_mcts_advance_boards(azg_mcts* h, int8_t* boards, int8_t* players, int32_t* counts, int32_t* status,
                                int32_t* n_out, int32_t n_threads)
{
    if (!h || !boards || !players || !counts || !status || !n_out) return fail("azg_mcts_advance_boards: null argument");
    return advance_impl(h, nullptr, boards, players, counts, status, n_out, n_threads);
}

int32_t azg_mcts_feed(azg_mcts* h, const float* probs, const float* values)
{
    if (!h || !probs || !values) return fail("azg_mcts_feed: null argument");
    const int A = h->A;
    const bool noise_cfg = h->cfg.add_dirichlet_noise != 0;
    size_t off = 0;
    for (auto& gs : h->games) {
        if (gs.status != AZG_MCTS_NEED_EVAL) continue;
        const bool noise_move = noise_cfg && gs.move_number < h->cfg.apply_dirichlet_n_first_moves;
        for (size_t i = 0; i < gs.queue.size(); ++i, ++off) {
            const Pending& pd = gs.queue[i];
            Node& nd = gs.nodes[gs.make_node(pd.key)];
            float p[MAXN];
            int cnt = 0;
            for (int a = 0; a < A; ++a) {
                nd.valid[a] = pd.st.board[a] == 0;
                cnt += nd.valid[a];
                p[a] = probs[off * A + a] * (float)nd.valid[a];
            }
            if (np_pairwise_sum_f32(p, A) < 1e-8f) {
                const float fc = (float)cnt;
                for (int a = 0; a < A; ++a) p[a] = (float)nd.valid[a] / fc;
            }
            std::memcpy(nd.P.data(), p, sizeof(float) * A);
            nd.P64.reset();
            nd.V = values[off];
            nd.N.fill(0);
            nd.W.fill(0);
            if (noise_move && pd.key == gs.root_key) {
                gs.noise_pending = true;
                gs.noise_node = gs.node_for(pd.key);
            }
        }
        gs.queue.clear();
        gs.status = AZG_MCTS_IDLE;
    }
    return 0;
}

int32_t azg_mcts_noise_request(azg_mcts* h, int32_t g, float* p)
{
    if (!h || g < 0 || g >= (int)h->games.size()) return -1;
    GameSearch& gs = h->games[g];
    if (!gs.noise_pending) return 0;
    if (p) std::memcpy(p, gs.nodes[gs.noise_node].P.data(), sizeof(float) * h->A);
    return 1;
}

int32_t azg_mcts_set_root_prior(azg_mcts* h, int32_t g, const double* p64)
{
    if (!h || g < 0 || g >= (int)h->games.size() || !p64) return fail("azg_mcts_set_root_prior: bad arguments");
    GameSearch& gs = h->games[g];
    if (!gs.noise_pending) return fail("azg_mcts_set_root_prior: no pending noise request");
    Node& nd = gs.nodes[gs.noise_node];
    nd.P64.reset(new std::array<double, MAXN>());
    std::memcpy(nd.P64->data(), p64, sizeof(double) * h->A);
    gs.noise_pending = false;
    gs.noise_node = -1;
    return 0;
}

int32_t azg_mcts_get_pi(azg_mcts* h, int32_t g, float* pi)
{
    if (!h || g < 0 || g >= (int)h->games.size() || !pi) return fail("azg_mcts_get_pi: bad arguments");
    GameSearch& gs = h->games[g];
    const int32_t id = gs.node_for(gs.root_key);
    if (id < 0) return fail("azg_mcts_get_pi: root not in tree");
    const Node& nd = gs.nodes[id];
    const int A = h->A;
    float cnt[MAXN] = {};
    for (int a = 0; a < A; ++a) cnt[a] = (float)nd.N[a];
    const float total = np_pairwise_sum_f32(cnt, A);
    if (total > 0) {
        for (int a = 0; a < A; ++a) pi[a] = cnt[a] / total;
    } else {
        float v[MAXN] = {};
        for (int a = 0; a < A; ++a) v[a] = (float)nd.valid[a];
        const float s = np_pairwise_sum_f32(v, A);
        for (int a = 0; a < A; ++a) pi[a] = v[a] / s;
    }
    return 0;
}

int32_t azg_mcts_clear(azg_mcts* h, int32_t g)
{
    if (!h || g < 0 || g >= (int)h->games.size()) return fail("azg_mcts_clear: bad arguments");
    GameSearch fresh;
    std::swap(h->games[g], fresh);
    return 0;
}

int64_t azg_mcts_tree_size(const azg_mcts* h, int32_t g)
{
    if (!h || g < 0 || g >= (int)h->games.size()) return -1;
    return (int64_t)h->games[g].nodes.size();
}

int32_t azg_mcts_replay(int32_t rules, int32_t board, const int8_t* start, int32_t player, int32_t cap1,
                        int32_t cap2, const int32_t* actions, int32_t n, int8_t* boards_out, int32_t* caps_out,
                        int32_t* winner_out, int32_t* over_out)
{
    if ((rules != 0 && rules != 1) || board < 5 || board * board > MAXN || !actions || n < 0)
        return fail("azg_mcts_replay: bad arguments");
    State s;
    s.n = board;
    s.rules = rules;
    const int A = board * board;
    for (int i = 0; i < A; ++i) s.board[i] = start ? start[i] : 0;
    s.player = player;
    s.cap[1] = cap1;
    s.cap[2] = cap2;
    for (int k = 0; k < n; ++k) {
        const int a = actions[k];
        if (a < 0 || a >= A || s.board[a] != 0) return fail("azg_mcts_replay: illegal move");
        s.do_move(a);
        if (boards_out) std::memcpy(boards_out + (size_t)k * A, s.board.data(), A);
        if (caps_out) {
            caps_out[2 * k] = s.cap[1];
            caps_out[2 * k + 1] = s.cap[2];
        }
        if (winner_out) winner_out[k] = s.winner();
        if (over_out) over_out[k] = s.game_over() ? 1 : 0;
    }
    return 0;
}

}  // extern "C"
