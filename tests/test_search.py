"""Search layer (host side of the hot path's caller): MCTS, self-play collection,
Player API and game rules, pinned bit-exactly against goldens produced by the
reference (tests/golden/make_golden_mcts.py) with a deterministic fake model.
CPU only: the search is host logic; the model is injected."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
from fake_model import FakeModel  # noqa: E402

from games.gomoku import Gomoku  # noqa: E402  (product)
from games.pente import Pente  # noqa: E402
from mcts.new_mcts_alpha import MCTS  # noqa: E402
import selfplay  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "mcts_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def argmax_game(noise, n_moves, sims, seed):
    np.random.seed(seed)
    model = FakeModel(seed=1)
    mcts = MCTS(Gomoku, sims, model, cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                apply_dirichlet_n_first_moves=5, add_dirichlet_noise=noise)
    g = Gomoku(15)
    pis, moves = [], []
    for _ in range(n_moves):
        if g.is_game_over():
            break
        pi = mcts.run(g, len(g.move_history))
        a = int(np.argmax(pi))
        pis.append(np.asarray(pi, dtype=np.float64))
        moves.append(a)
        g.do_move(divmod(a, 15))
    return np.stack(pis), np.array(moves), np.array(model.calls), len(mcts.P)


@pytest.mark.parametrize("tag,noise,n,sims,seed", [("argmax", False, 14, 60, 0), ("noise", True, 8, 60, 123)])
def test_mcts_matches_reference_bit_exact(gold, tag, noise, n, sims, seed):
    pis, moves, calls, nkeys = argmax_game(noise, n, sims, seed)
    assert np.array_equal(moves, gold[f"{tag}/moves"])
    assert np.array_equal(pis, gold[f"{tag}/pis"])
    assert np.array_equal(calls, gold[f"{tag}/calls"])        # leaf batch sizes (32, 32, ..., flush)
    assert nkeys == int(gold[f"{tag}/nkeys"])


def test_play_game_and_collect_matches_reference(gold):
    np.random.seed(7)
    model = FakeModel(seed=2)
    mcts = MCTS(Gomoku, 40, model, cpuct=1.2, dirichlet_alpha=0.05, epsilon=0.15,
                apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True)
    ex, winner = selfplay.play_game_and_collect(mcts, Gomoku(15), lambda n: max(0.0, 1.0 - n / 8))
    assert len(ex) == int(gold["collect/n"]) and winner == int(gold["collect/winner"])
    assert np.array_equal(np.array([e[2] for e in ex]), gold["collect/z"])
    sel = ex[:16] + ex[-8:]
    assert np.array_equal(np.stack([e[0] for e in sel]), gold["collect/states"])
    assert np.array_equal(np.stack([e[1] for e in sel]), gold["collect/pis"])


def test_player_api_matches_reference(gold):
    from players.player_alpha import Player
    p = Player("gomoku", 15, n_simulations=48, model_path=None, nn_model=FakeModel)
    for t, b in enumerate(gold["player/boards"]):
        p.mcts.clear_tree()
        last = tuple(int(v) for v in gold["player/last"][t])
        move = p.play(b.tolist(), t, last)
        assert tuple(int(v) for v in move) == tuple(gold["player/moves"][t])


def test_batched_driver_equals_independent_games():
    """Many games advanced together (one batched evaluate per round) give exactly
    the trees/results of each game alone (batch-independent model, no RNG use)."""
    temp0 = lambda n: 0.0

    def one(seed_game):
        m = FakeModel(seed=3)
        mc = MCTS(Gomoku, 24, m, add_dirichlet_noise=False)
        g = Gomoku(15)
        g.do_move(divmod(seed_game * 17 % 225, 15))
        return selfplay.play_game_and_collect(mc, g, temp0, max_moves=12, use_symmetries=False)

    alone = [one(i) for i in range(5)]
    model = FakeModel(seed=3)
    gens = []
    for i in range(5):
        mc = MCTS(Gomoku, 24, model, add_dirichlet_noise=False)
        g = Gomoku(15)
        g.do_move(divmod(i * 17 % 225, 15))
        gens.append(selfplay.play_game_gen(mc, g, temp0, max_moves=12, use_symmetries=False))
    drv = selfplay.BatchedSelfPlay(model)
    together = drv.run(gens)
    assert drv.max_batch > 32
    for (ea, wa), (eb, wb) in zip(alone, together):
        assert wa == wb and len(ea) == len(eb)
        for x, y in zip(ea, eb):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]


def test_symmetries_are_dihedral():
    mc = MCTS(Gomoku, 1, FakeModel())
    s = np.random.default_rng(0).random((3, 15, 15)).astype(np.float32)
    pi = np.arange(225, dtype=np.float32)
    imgs = mc.symmetries(s, pi)
    assert len(imgs) == 8
    for si, pii in imgs:
        # the pi image must move with plane 0's image
        src = np.argwhere(si[0] == s[0, 3, 4])[0]
        assert pii.reshape(15, 15)[tuple(src)] == pi[3 * 15 + 4]


# ---------------------------------------------------------------- rules KATs
@pytest.mark.parametrize("dr,dc", [(0, 1), (1, 0), (1, 1), (1, -1)])
def test_gomoku_five_in_row(dr, dc):
    g = Gomoku(15)
    r0, c0 = 5, 7
    for i in range(5):
        g.board[r0 + i * dr, c0 + i * dc] = 1
    g.last_move = (r0 + 2 * dr, c0 + 2 * dc)
    assert g.check_winner() == 1 and g.is_game_over()
    g.board[r0 + 4 * dr, c0 + 4 * dc] = 0
    assert g.check_winner() == 0


def test_gomoku_play_and_encoding():
    g = Gomoku(15)
    assert g.do_move((7, 7)) and not g.do_move((7, 7)) and not g.do_move((15, 0))
    assert g.current_player == 2 and g.last_move == (7, 7)
    e = g.get_encoded_state()
    assert e[1, 7, 7] == 1 and e[0].sum() == 0 and np.all(e[2] == 1)
    assert g.get_valid_moves().sum() == 224
    g.undo_move()
    assert g.current_player == 1 and g.last_move is None and g.board.sum() == 0


def test_pente_capture_and_capture_win():
    g = Pente(15)
    # X O O X horizontally: player 1 at (7,4), player 2 at (7,5),(7,6); player 1 plays (7,7)
    g.board[7, 4] = 1
    g.board[7, 5] = 2
    g.board[7, 6] = 2
    g.current_player = 1
    g.do_move((7, 7))
    assert g.board[7, 5] == 0 and g.board[7, 6] == 0 and g.captures[1] == 1
    g.captures[1] = 4
    g.board[3, 3] = 1
    g.board[3, 4] = 2
    g.board[3, 5] = 2
    g.current_player = 1
    g.do_move((3, 6))
    assert g.captures[1] == 5 and g.check_winner() == 1
