"""§8(f)4 on the GPU: gating (train.evaluate_models, reference train.py:418-487) and
the arena (play_loop.change_starting_player, reference play_loop.py:36-112) with the
HIP engine behind both players.  The CPU tests (test_loop_golden.py) pin these game
bodies to the reference with fake models; here the SAME bodies run on real HIP
models through every search / evaluation path the product has, and must agree move
for move (the forward is bitwise batch-independent, so batching never changes a
prior):

  * evaluate_models(native=True) with two HIP models -> NativeEval with both nets'
    int8 board evaluators in flight (train.py's path), vs
  * evaluate_models(native=True) over the models' float `predict` (NativeEval
    without board evaluators), vs
  * evaluate_models(native=False): the reference-semantics Python searches under
    BatchedSelfPlay on the same HIP models;
  * play_loop.change_starting_player with players.player_alpha / player_alpha2 on
    HIP models: native search vs the Python MCTS.
"""
import io
import random
from contextlib import redirect_stdout

import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def _model(seed, blocks=3, ch=64):
    from network import PyTorchModel
    torch.manual_seed(seed)
    m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=blocks, channels=ch)
    m.net.eval()
    return m


class _PredictOnly:
    """A HIP model seen through `predict` only (no board_evaluator): NativeEval then
    feeds float planes through PyTorchModel.predict instead of int8 boards."""

    def __init__(self, m):
        self._m = m
        self.board_size = m.board_size
        self.engine = m.engine

    def predict(self, x):
        return self._m.predict(x)


@pytest.mark.timeout(600)
def test_evaluate_models_gpu_paths_agree():
    import train
    new, best = _model(31), _model(32)
    runs = {}
    for name, a, b, native in (("native_boards", new, best, True),
                               ("native_predict", _PredictOnly(new), _PredictOnly(best), True),
                               ("python", new, best, False)):
        random.seed(11)
        games = []
        res = train.evaluate_models(a, b, "gomoku", n_games=4, n_simulations=24, cpuct=1.0, native=native,
                                    record=games)
        runs[name] = (res, [list(g.move_history) for g in games])
        new.engine.check_status()
        best.engine.check_status()
    ref = runs["native_boards"]
    assert sum(len(mv) for mv in ref[1]) > 4 * 8          # real games, not openings only
    for name, got in runs.items():
        assert got[0] == ref[0], (name, got[0], ref[0])
        assert got[1] == ref[1], name


@pytest.mark.timeout(600)
def test_arena_player_alpha_on_hip_models_native_vs_python():
    import play_loop
    import players.player_alpha as pa
    import players.player_alpha2 as pa2
    from games.gomoku import Gomoku
    from mcts.new_mcts_alpha import MCTS
    seeds = {"player_alpha": 41, "player_alpha2": 42}
    names = ("player_alpha", "player_alpha2")
    out = {}
    for impl in ("native", "python"):
        def loader(name, rules, size, impl=impl):
            mod = {"player_alpha": pa, "player_alpha2": pa2}[name]
            return mod.Player(rules, size, n_simulations=32, model_path=None,
                              nn_model=lambda board_size: _model(seeds[name]),
                              mcts_class=MCTS if impl == "python" else None)
        with redirect_stdout(io.StringIO()):
            p1, p2 = loader(names[0], "gomoku", 15), loader(names[1], "gomoku", 15)
            metrics = play_loop.initiate_metrics(names[0], names[1], p1, p2, "gomoku", 2)
            random.seed(21)
            w1 = play_loop.change_starting_player(names[0], names[1], Gomoku(15), "gomoku", 15, metrics, 1,
                                                  verbose=False, loader=loader)
            w2 = play_loop.change_starting_player(names[1], names[0], Gomoku(15), "gomoku", 15, metrics, 2,
                                                  verbose=False, loader=loader)
        out[impl] = ((w1, w2), {n: {g: [tuple(int(v) for v in mv) for mv in metrics["move_made"][n][g]]
                                    for g in ("game_1", "game_2")} for n in names})
    assert out["native"][0] == out["python"][0]
    assert out["native"][1] == out["python"][1]
    assert sum(len(v) for d in out["native"][1].values() for v in d.values()) > 10
