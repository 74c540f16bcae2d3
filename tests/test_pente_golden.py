"""Pente pinned to the REFERENCE (tests/golden/pente_golden.npz, written by
tests/golden/make_golden_pente.py importing /root/reference/games/pente.py and
mcts/new_mcts_alpha.py): capture known answers in all 8 directions, double capture,
edge non-capture, capture win at 5 pairs (pente.py:114-152,199-233), undo_move with
its colour quirk, encoding and legal mask; 64 random games move by move; reference
MCTS pi per move from a capture-rich mid-game (noise off / on); the reference
play_game_and_collect.  Checked against the builder's Python Pente, the native C++
rule engine (azg_mcts_replay) and both searches (Python and native).  CPU only."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
from fake_model import FakeModel  # noqa: E402

import _native_mcts  # noqa: E402
import selfplay  # noqa: E402
from games.pente import Pente  # noqa: E402
from mcts.native_mcts import NativeMCTS  # noqa: E402
from mcts.new_mcts_alpha import MCTS  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "pente_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _setup(gold, i):
    g = Pente(15)
    g.board[:] = gold["kat/setup"][i]
    g.captures = {1: int(gold["kat/setup_caps"][i][0]), 2: int(gold["kat/setup_caps"][i][1])}
    g.current_player = int(gold["kat/setup_player"][i])
    return g, tuple(int(v) for v in gold["kat/move"][i])


def test_capture_known_answers_python(gold):
    for i in range(len(gold["kat/move"])):
        g, mv = _setup(gold, i)
        assert g.do_move(mv)
        assert np.array_equal(g.board, gold["kat/board"][i]), i
        assert [g.captures[1], g.captures[2]] == list(gold["kat/caps"][i]), i
        assert g.get_winner() == gold["kat/winner"][i] and g.is_game_over() == bool(gold["kat/over"][i]), i
        assert np.array_equal(g.get_encoded_state(), gold["kat/enc"][i]), i
        assert np.array_equal(g.get_valid_moves(), gold["kat/mask"][i]), i
        g.undo_move()
        assert np.array_equal(g.board, gold["kat/undo_board"][i]), i          # reference colour quirk
        assert [g.captures[1], g.captures[2]] == list(gold["kat/undo_caps"][i]), i


def test_capture_known_answers_native(gold):
    for i in range(len(gold["kat/move"])):
        mv = gold["kat/move"][i]
        b, cap, win, over = _native_mcts.replay(1, [int(mv[0]) * 15 + int(mv[1])], start=gold["kat/setup"][i],
                                                player=int(gold["kat/setup_player"][i]), caps=gold["kat/setup_caps"][i])
        assert np.array_equal(b[0].reshape(15, 15), gold["kat/board"][i]), i
        assert list(cap[0]) == list(gold["kat/caps"][i]), i
        assert win[0] == gold["kat/winner"][i] and over[0] == bool(gold["kat/over"][i]), i


def test_random_games_python_and_native(gold):
    for gi in range(len(gold["play/n"])):
        n = int(gold["play/n"][gi])
        acts = gold["play/moves"][gi][:n].astype(np.int64)
        g = Pente(15)
        for k, a in enumerate(acts):
            assert g.do_move(divmod(int(a), 15))
            assert (g.captures[1], g.captures[2]) == tuple(gold["play/caps"][gi][k]), (gi, k)
        assert np.array_equal(g.board, gold["play/final"][gi])
        assert g.get_winner() == gold["play/winner"][gi] and g.is_game_over() == bool(gold["play/over"][gi])
        b, cap, win, over = _native_mcts.replay(1, acts)
        assert np.array_equal(cap, gold["play/caps"][gi][:n]), gi
        assert np.array_equal(b[-1].reshape(15, 15), gold["play/final"][gi]), gi
        assert win[-1] == gold["play/winner"][gi] and over[-1] == bool(gold["play/over"][gi]), gi
        assert not over[:-1].any()                        # the playout stopped at the first game over


def test_undo_replays_reference(gold):
    n = int(gold["play/n"][0])
    g = Pente(15)
    for a in gold["play/moves"][0][:n]:
        g.do_move(divmod(int(a), 15))
    for k in range(n):
        g.undo_move()
        assert np.array_equal(g.board, gold["undo/boards"][k]), k


def _midgame(gold, tag):
    g = Pente(15)
    for r, c in gold[f"{tag}/start_moves"]:
        g.do_move((int(r), int(c)))
    return g


@pytest.mark.parametrize("search", [MCTS, NativeMCTS])
@pytest.mark.parametrize("tag,noise,n,seed", [("mcts_argmax", False, 12, 0), ("mcts_noise", True, 8, 123)])
def test_search_matches_reference(gold, search, tag, noise, n, seed):
    np.random.seed(seed)
    model = FakeModel(seed=1)
    mcts = search(Pente, 60, model, cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                  apply_dirichlet_n_first_moves=40, add_dirichlet_noise=noise)
    g = _midgame(gold, tag)
    pis, moves, caps = [], [], []
    for _ in range(n):
        if g.is_game_over():
            break
        pi = mcts.run(g, len(g.move_history))
        a = int(np.argmax(pi))
        pis.append(np.asarray(pi, dtype=np.float64))
        moves.append(a)
        g.do_move(divmod(a, 15))
        caps.append((g.captures[1], g.captures[2]))
    assert np.array_equal(np.array(moves), gold[f"{tag}/moves"])
    assert np.array_equal(np.stack(pis), gold[f"{tag}/pis"])
    assert np.array_equal(np.array(caps), gold[f"{tag}/caps"])
    assert np.array_equal(np.array(model.calls), gold[f"{tag}/calls"])
    size = mcts.tree_size() if hasattr(mcts, "tree_size") else len(mcts.P)
    assert size == int(gold[f"{tag}/nkeys"])


@pytest.mark.parametrize("search", [MCTS, NativeMCTS])
def test_collect_matches_reference(gold, search):
    np.random.seed(7)
    model = FakeModel(seed=2)
    mcts = search(Pente, 40, model, cpuct=1.2, dirichlet_alpha=0.05, epsilon=0.15,
                  apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True)
    ex, winner = selfplay.play_game_and_collect(mcts, Pente(15), lambda n: max(0.0, 1.0 - n / 8))
    assert len(ex) == int(gold["collect/n"]) and winner == int(gold["collect/winner"])
    assert np.array_equal(np.array([e[2] for e in ex]), gold["collect/z"])
    sel = ex[:16] + ex[-8:]
    assert np.array_equal(np.stack([e[0] for e in sel]), gold["collect/states"])
    assert np.array_equal(np.stack([e[1] for e in sel]), gold["collect/pis"])
