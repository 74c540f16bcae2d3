"""Native (C++) search, libazg_mcts.so (include/azg_mcts.h): bit-exact against the
reference goldens (tests/golden/make_golden_mcts.py, produced by the reference's own
mcts/new_mcts_alpha.py with a deterministic fake model) and against the
reference-semantics Python search on Gomoku and Pente, with Dirichlet noise and
temperature sampling; the multi-game engines equal the games played alone, for any
host thread count.  CPU only (the model is injected)."""
import os
import re
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, GOLDEN)
from fake_model import FakeBoardEvaluator, FakeModel  # noqa: E402

import _native_mcts  # noqa: E402
import selfplay  # noqa: E402
from games.gomoku import Gomoku  # noqa: E402
from games.pente import Pente  # noqa: E402
from mcts.native_mcts import NativeEval, NativeMCTS, NativeSelfPlay  # noqa: E402
from mcts.new_mcts_alpha import MCTS  # noqa: E402

HEADER = os.path.join(REPO, "include", "azg_mcts.h")


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "mcts_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def same_examples(a, b):
    return len(a) == len(b) and all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]
                                    for x, y in zip(a, b))


def test_header_matches_exports():
    txt = open(HEADER).read()
    syms = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\**(azg_mcts_[a-z_]+)\s*\(", txt, re.M))
    assert syms == set(_native_mcts.EXPORTS)
    lib = _native_mcts.load_library()
    for s in syms:
        assert hasattr(lib, s)


@pytest.mark.parametrize("tag,noise,n,sims,seed", [("argmax", False, 14, 60, 0), ("noise", True, 8, 60, 123)])
def test_native_mcts_matches_reference_goldens(gold, tag, noise, n, sims, seed):
    np.random.seed(seed)
    model = FakeModel(seed=1)
    mcts = NativeMCTS(Gomoku, sims, model, cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                      apply_dirichlet_n_first_moves=5, add_dirichlet_noise=noise)
    g = Gomoku(15)
    pis, moves = [], []
    for _ in range(n):
        if g.is_game_over():
            break
        pi = mcts.run(g, len(g.move_history))
        assert pi.dtype == np.float32
        a = int(np.argmax(pi))
        pis.append(np.asarray(pi, dtype=np.float64))
        moves.append(a)
        g.do_move(divmod(a, 15))
    assert np.array_equal(np.array(moves), gold[f"{tag}/moves"])
    assert np.array_equal(np.stack(pis), gold[f"{tag}/pis"])
    assert np.array_equal(np.array(model.calls), gold[f"{tag}/calls"])   # leaf batch sizes
    assert mcts.tree_size() == int(gold[f"{tag}/nkeys"])


def test_native_collect_matches_reference(gold):
    np.random.seed(7)
    model = FakeModel(seed=2)
    mcts = NativeMCTS(Gomoku, 40, model, cpuct=1.2, dirichlet_alpha=0.05, epsilon=0.15,
                      apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True)
    ex, winner = selfplay.play_game_and_collect(mcts, Gomoku(15), lambda n: max(0.0, 1.0 - n / 8))
    assert len(ex) == int(gold["collect/n"]) and winner == int(gold["collect/winner"])
    assert np.array_equal(np.array([e[2] for e in ex]), gold["collect/z"])
    sel = ex[:16] + ex[-8:]
    assert np.array_equal(np.stack([e[0] for e in sel]), gold["collect/states"])
    assert np.array_equal(np.stack([e[1] for e in sel]), gold["collect/pis"])


@pytest.mark.parametrize("mcts_class", [None, MCTS])
def test_player_both_searches_match_reference(gold, mcts_class):
    from players.player_alpha import Player
    p = Player("gomoku", 15, n_simulations=48, model_path=None, nn_model=FakeModel, mcts_class=mcts_class)
    assert isinstance(p.mcts, mcts_class or NativeMCTS)
    for t, b in enumerate(gold["player/boards"]):
        p.mcts.clear_tree()
        last = tuple(int(v) for v in gold["player/last"][t])
        move = p.play(b.tolist(), t, last)
        assert tuple(int(v) for v in move) == tuple(gold["player/moves"][t])


@pytest.mark.parametrize("cls", [Gomoku, Pente])
@pytest.mark.parametrize("cpuct,sims,bs", [(1.1, 50, 32), (2.5, 70, 8), (0.7, 33, 1)])
def test_native_equals_python_search(cls, cpuct, sims, bs):
    """Noise (float64 root prior), sampling, tree reuse, captures, odd batch sizes."""
    res = []
    for M in (MCTS, NativeMCTS):
        m = FakeModel(seed=4)
        mc = M(cls, sims, m, cpuct=cpuct, batch_size=bs, dirichlet_alpha=0.3, epsilon=0.25,
               apply_dirichlet_n_first_moves=6, add_dirichlet_noise=True, rng=np.random.RandomState(5))
        ex, w = selfplay.play_game_and_collect(mc, cls(15), lambda n: 1.0 if n < 10 else 0.0,
                                               max_moves=60 if bs > 1 else 16,
                                               use_symmetries=False)
        res.append((ex, w, m.calls))
    (a, wa, ca), (b, wb, cb) = res
    assert wa == wb and ca == cb and same_examples(a, b)


def test_pente_capture_positions_match():
    """A Pente middlegame with captures on the board and capture counts near the win."""
    rng = np.random.RandomState(3)
    g = Pente(15)
    while len(g.move_history) < 40 and not g.is_game_over():
        v = np.nonzero(g.get_valid_moves())[0]
        g.do_move(divmod(int(rng.choice(v)), 15))
    g.captures = {1: 4, 2: 4}
    pis = []
    for M in (MCTS, NativeMCTS):
        mc = M(Pente, 120, FakeModel(seed=6), cpuct=1.0, add_dirichlet_noise=False)
        pis.append(mc.run(g.clone(), len(g.move_history)))
    assert np.array_equal(pis[0], pis[1])


def test_terminal_root_neighbourhood_and_full_board():
    """Search next to a forced win (terminal leaves dominate) and on a nearly full board."""
    g = Gomoku(15)
    for c in range(4):
        g.do_move((7, c))
        g.do_move((9, c + 5))
    full = Gomoku(15)
    order = np.random.RandomState(1).permutation(225)
    for a in order[:221]:
        full.board.reshape(-1)[a] = 1 + (a % 2)
    full.current_player = 1
    for game in (g, full):
        pis = []
        for M in (MCTS, NativeMCTS):
            mc = M(Gomoku, 64, FakeModel(seed=8), add_dirichlet_noise=False)
            pis.append(mc.run(game.clone(), len(game.move_history)))
        assert np.array_equal(pis[0], pis[1])


@pytest.mark.parametrize("threads", [1, 8])
def test_native_selfplay_equals_games_alone(threads):
    G = 6
    seeds = [11 + i for i in range(G)]
    temp = lambda n: 1.0 if n < 6 else 0.0
    sp = NativeSelfPlay(FakeModel(seed=9).predict, Gomoku, G, 40, cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                        apply_dirichlet_n_first_moves=5, n_threads=threads)
    together = sp.play(temp, max_moves=24, use_symmetries=True, seeds=seeds)
    assert sp.max_batch > 32
    for g in (0, 3, 5):
        mc = MCTS(Gomoku, 40, FakeModel(seed=9), cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                  apply_dirichlet_n_first_moves=5, rng=np.random.RandomState(seeds[g]))
        ex, w = selfplay.play_game_and_collect(mc, Gomoku(15), temp, max_moves=24)
        assert w == together[g][1] and same_examples(ex, together[g][0])


def test_native_eval_equals_python_eval():
    from train import eval_game_gen
    mn_model, mb_model = FakeModel(seed=21), FakeModel(seed=22)
    openings = [(7, 7), (5, 9), (10, 3), (8, 8), (4, 4)]

    def fresh():
        gs = []
        for o in openings:
            g = Gomoku(15)
            g.do_move(o)
            gs.append(g)
        return gs

    starts = [i % 2 == 0 for i in range(len(openings))]
    arena = NativeEval({"new": mn_model.predict, "best": mb_model.predict}, Gomoku, len(openings), 30, cpuct=1.3)
    games_n = fresh()
    w_native = arena.play(games_n, ["new" if s else "best" for s in starts])
    # the pinned int8-board evaluator path (both networks' batches in flight)
    arena_b = NativeEval(None, Gomoku, len(openings), 30, cpuct=1.3,
                         evaluator_factories={"new": lambda c: FakeBoardEvaluator(mn_model, c),
                                              "best": lambda c: FakeBoardEvaluator(mb_model, c)})
    games_b = fresh()
    assert arena_b.play(games_b, ["new" if s else "best" for s in starts]) == w_native
    assert [g.move_history for g in games_b] == [g.move_history for g in games_n]
    gens = []
    games_p = fresh()
    for game, s in zip(games_p, starts):
        mn = MCTS(Gomoku, 30, mn_model, cpuct=1.3, add_dirichlet_noise=False)
        mb = MCTS(Gomoku, 30, mb_model, cpuct=1.3, add_dirichlet_noise=False)
        gens.append(eval_game_gen(mn, mb, game, s))
    w_py = selfplay.BatchedSelfPlay({"new": mn_model, "best": mb_model}).run(gens)
    assert w_native == w_py
    for a, b in zip(games_n, games_p):
        assert a.move_history == b.move_history


def test_errors_are_loud():
    f = _native_mcts.SearchForest(2, 8)
    with pytest.raises(RuntimeError):
        f.get_pi(0)                       # no root searched yet
    g = Gomoku(15)
    f.set_root(0, g, 0)
    with pytest.raises(RuntimeError):
        f.set_root(0, g, 0)               # search in progress
    with pytest.raises(RuntimeError):
        _native_mcts.SearchForest(1, 8, board=9)
    with pytest.raises(RuntimeError):
        _native_mcts.SearchForest(1, 8, batch_size=0)
    # a pending Dirichlet request blocks advance until the prior is supplied
    f2 = _native_mcts.SearchForest(1, 4, add_dirichlet_noise=True, batch_size=1)
    f2.set_root(0, Gomoku(15), 0)
    n = f2.advance()
    assert n == 1 and f2.status[0] == _native_mcts.NEED_EVAL
    p, v = FakeModel().predict(f2.leaves[:n])
    f2.feed(p, v)
    p32 = f2.noise_request(0)
    assert p32 is not None and p32.dtype == np.float32
    with pytest.raises(RuntimeError):
        f2.advance()
    f2.set_root_prior(0, p32.astype(np.float64))
    f2.advance()


@pytest.mark.parametrize("groups", [1, 2, 3])
def test_pipelined_board_selfplay_equals_sync(groups):
    """Board-mode leaves (int8 + side to move), masked priors and the grouped
    search/evaluate pipeline give exactly the synchronous planes-mode games."""
    G = 7
    seeds = [31 + i for i in range(G)]
    temp = lambda n: 1.0 if n < 5 else 0.0
    kw = dict(cpuct=1.1, dirichlet_alpha=0.3, epsilon=0.25, apply_dirichlet_n_first_moves=4)
    sync = NativeSelfPlay(FakeModel(seed=12).predict, Gomoku, G, 36, **kw).play(temp, max_moves=14, seeds=seeds)
    m = FakeModel(seed=12)
    pipe = NativeSelfPlay(None, Gomoku, G, 36, evaluator_factory=lambda cap: FakeBoardEvaluator(m, cap),
                          groups=groups, **kw)
    out = pipe.play(temp, max_moves=14, seeds=seeds)
    assert len(pipe.forests) == groups
    for (ea, wa), (eb, wb) in zip(sync, out):
        assert wa == wb and same_examples(ea, eb)


def test_advance_boards_matches_planes():
    """The int8 leaves encode to exactly the float planes advance() emits."""
    fa = _native_mcts.SearchForest(3, 40, add_dirichlet_noise=False)
    fb = _native_mcts.SearchForest(3, 40, add_dirichlet_noise=False)
    m = FakeModel(seed=2)
    for g in range(3):
        game = Gomoku(15)
        game.do_move((g, 2 * g))
        fa.set_root(g, game, 1)
        fb.set_root(g, game, 1)
    boards = np.zeros((3 * 32, 225), np.int8)
    players = np.zeros(3 * 32, np.int8)
    for _ in range(4):
        na = fa.advance()
        nb = fb.advance_boards(boards, players)
        assert na == nb and np.array_equal(fa.counts, fb.counts) and np.array_equal(fa.status, fb.status)
        if na == 0:
            break
        b = boards[:nb].astype(np.int64)
        pl = players[:nb].astype(np.int64)[:, None]
        x = np.stack([(b == pl), (b == 3 - pl), np.ones_like(b, dtype=bool)], axis=1).astype(np.float32)
        assert np.array_equal(x.reshape(nb, 3, 15, 15), fa.leaves[:na])
        p, v = m.predict(fa.leaves[:na])
        fa.feed(p, v)
        fb.feed(p * (boards[:nb] == 0), v)      # pre-masked priors install identically
