"""The loop around the hot path pinned to the REFERENCE (tests/golden/loop_golden.npz,
written by tests/golden/make_golden_loop.py importing /root/reference):
  * f3 replay-buffer interop: the reference's save_replay_buffer pickle (train.py:
    302-319) loads through selfplay.load_replay_buffer with identical examples, and
    selfplay.save_replay_buffer writes byte-for-byte the pickle the reference's
    load_replay_buffer (train.py:322-354) was shown to read back;
  * f4 evaluation: train.evaluate_models (native C++ searches and the Python ones)
    equals the reference game body (train.py:418-487): same results, same moves;
  * f4 arena: play_loop.change_starting_player with this framework's player_alpha /
    player_alpha2 plays the reference play_loop.py:36-112 games move for move.
CPU only (fake models, tests/golden/fake_model.py)."""
import io
import os
import random
import sys
from contextlib import redirect_stdout

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
from fake_model import FakeModel  # noqa: E402

import selfplay  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLDEN, "loop_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _examples(gold):
    return [(gold["buffer/states"][i], gold["buffer/pis"][i], float(gold["buffer/z"][i]))
            for i in range(len(gold["buffer/z"]))]


def test_reference_buffer_pickle_loads(gold, tmp_path):
    p = tmp_path / "ref.pkl"
    p.write_bytes(gold["buffer/ref_pickle"].tobytes())
    with redirect_stdout(io.StringIO()):
        buf = selfplay.load_replay_buffer(str(p), capacity=50)
    assert buf is not None and buf.capacity == 50 and len(buf) == len(gold["buffer/z"])
    for (s, pi, z), (s0, pi0, z0) in zip(buf.buffer, _examples(gold)):
        assert s.dtype == np.float32 and np.array_equal(s, s0) and np.array_equal(pi, pi0) and z == z0
    st, ps, zs = buf.sample(4)
    assert st.shape == (4, 3, 15, 15) and ps.shape == (4, 225) and zs.shape == (4, 1)


def test_buffer_pickle_is_what_the_reference_reads(gold, tmp_path):
    buf = selfplay.ReplayBuffer(capacity=50)
    buf.add(_examples(gold))
    p = tmp_path / "azg.pkl"
    with redirect_stdout(io.StringIO()):
        assert selfplay.save_replay_buffer(buf, str(p))
    assert p.read_bytes() == gold["buffer/azg_pickle"].tobytes()
    # ... and what the reference's loader read from those bytes (recorded at generation)
    assert int(gold["buffer/ref_read_capacity"]) == 50
    assert np.array_equal(gold["buffer/ref_read_states"], gold["buffer/states"])
    assert np.array_equal(gold["buffer/ref_read_pis"], gold["buffer/pis"])
    assert np.array_equal(gold["buffer/ref_read_z"], gold["buffer/z"])


@pytest.mark.parametrize("native", [True, False])
def test_evaluate_models_matches_reference(gold, native):
    import train
    random.seed(11)
    games = []
    nw, rate, draws = train.evaluate_models(FakeModel(seed=3), FakeModel(seed=4), "gomoku",
                                            n_games=int(gold["eval/n_games"]), n_simulations=int(gold["eval/sims"]),
                                            cpuct=1.0, native=native, record=games)
    assert (nw, draws) == (int(gold["eval/new_wins"]), int(gold["eval/draws"]))
    assert rate == float(gold["eval/win_rate"])
    for g, want in zip(games, gold["eval/moves"]):
        got = [r * 15 + c for r, c in g.move_history]
        assert got == [int(v) for v in want if v >= 0]


@pytest.mark.parametrize("mcts_class", [None, "python"])
def test_arena_matches_reference_play_loop(gold, mcts_class):
    import play_loop
    import players.player_alpha as pa
    import players.player_alpha2 as pa2
    from games.gomoku import Gomoku
    from mcts.new_mcts_alpha import MCTS
    sims = int(gold["arena/sims"])
    seeds = {"player_alpha": 5, "player_alpha2": 6}

    def loader(name, rules, size):
        mod = {"player_alpha": pa, "player_alpha2": pa2}[name]
        return mod.Player(rules, size, n_simulations=sims, model_path=None,
                          nn_model=lambda board_size: FakeModel(board_size, seed=seeds[name]),
                          mcts_class=MCTS if mcts_class == "python" else None)

    names = ("player_alpha", "player_alpha2")
    with redirect_stdout(io.StringIO()):
        p1, p2 = loader(names[0], "gomoku", 15), loader(names[1], "gomoku", 15)
        metrics = play_loop.initiate_metrics(names[0], names[1], p1, p2, "gomoku", 2)
        random.seed(21)
        w1 = play_loop.change_starting_player(names[0], names[1], Gomoku(15), "gomoku", 15, metrics, 1,
                                              loader=loader)
        w2 = play_loop.change_starting_player(names[1], names[0], Gomoku(15), "gomoku", 15, metrics, 2,
                                              loader=loader)
    assert [w or "" for w in (w1, w2)] == list(gold["arena/winners"])
    for g in (1, 2):
        for n in names:
            got = [int(r) * 15 + int(c) for r, c in metrics["move_made"][n][f"game_{g}"]]
            assert got == [int(v) for v in gold[f"arena/game{g}/{n}"]], (g, n)
