"""End-to-end on the GPU: batched self-play through the HIP engine, the training
loop entry point, and checkpoint interop with the reference format
(network.py:240-258) via the oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import golden_state, has_gpu, load_golden
from oracle.boards import encode_batch, synth_positions
from oracle.ref_net import RefModel, load_numpy_state, state_to_numpy

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def test_batched_selfplay_on_gpu_matches_sequential():
    from games.gomoku import Gomoku
    from mcts.new_mcts_alpha import MCTS
    from network import PyTorchModel
    import selfplay

    g = load_golden("3x64")
    m = PyTorchModel(device="cuda")
    m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state(g).items()})
    temp0 = lambda n: 0.0

    def gen(i):
        mc = MCTS(Gomoku, 40, m, add_dirichlet_noise=False)
        game = Gomoku(15)
        game.do_move(divmod((i * 37 + 11) % 225, 15))
        return selfplay.play_game_gen(mc, game, temp0, max_moves=10, use_symmetries=True)

    drv = selfplay.BatchedSelfPlay(m)
    together = drv.run([gen(i) for i in range(6)])
    assert drv.max_batch > 32 and drv.boards > 6 * 10 * 40 * 0.9
    for i in (0, 5):
        mc_gen = gen(i)
        alone = MCTS(Gomoku, 1, m).drive(mc_gen)
        ea, wa = alone
        eb, wb = together[i]
        assert wa == wb and len(ea) == len(eb) == 80
        for x, y in zip(ea, eb):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]


def test_checkpoint_roundtrip_with_reference_format(tmp_path):
    from network import PyTorchModel
    g = load_golden("3x64")
    st = golden_state(g)
    # a reference-format checkpoint written by the oracle (== reference network.py:240-248)
    ref = RefModel(3, 64)
    load_numpy_state(ref.net, st)
    b, p = synth_positions(16, seed=3)
    x = encode_batch(b, p)
    ref.train_batch(x, np.full((16, 225), 1 / 225, np.float32), np.zeros((16, 1), np.float32))
    path = str(tmp_path / "ref.pt")
    torch.save({"net": ref.net.state_dict(), "opt": ref.optimizer.state_dict(), "board_size": 15,
                "action_size": 225}, path)
    m = PyTorchModel(device="cuda")
    m.load(path)
    rp, rv = ref.predict(x)
    gp, gv = m.predict(x)
    np.testing.assert_allclose(gp, rp, atol=1e-5)
    np.testing.assert_allclose(gv, rv, atol=1e-5)
    # optimizer state carried over into the flat moment buffers
    st0 = m.optimizer.state[next(iter(m.net.parameters()))]
    assert float(st0["step"]) == 1.0
    np.testing.assert_allclose(st0["exp_avg"].cpu().numpy(),
                               ref.optimizer.state[next(iter(ref.net.parameters()))]["exp_avg"].numpy(), atol=1e-7)
    # and back: our checkpoint loads into the oracle (reference) module
    out = str(tmp_path / "ours.pt")
    m.save(out)
    d = torch.load(out, map_location="cpu", weights_only=True)
    assert set(d) == {"net", "opt", "board_size", "action_size"}
    ref2 = RefModel(3, 64)
    ref2.net.load_state_dict(d["net"])
    ref2.optimizer.load_state_dict(d["opt"])
    np.testing.assert_allclose(ref2.predict(x)[0], gp, atol=1e-5)


def test_train_alphazero_smoke(tmp_path):
    import train
    best = train.train_alphazero(num_iterations=1, games_per_iteration=3, n_simulations=12, batch_size=64,
                                 epochs_per_iter=1, eval_games=2, eval_mcts_simulations=8, model_dir=str(tmp_path),
                                 n_res_blocks=1, channels=64, max_moves=20)
    files = os.listdir(tmp_path)
    assert any(f.startswith("snapshot_iter1_") for f in files) and "replay_buffer_latest.pkl" in files
    assert best.engine is not None


def test_native_selfplay_on_gpu_matches_python_search():
    """The C++ multi-game search fed by the HIP forward gives, per game, exactly the
    reference-semantics Python search run alone on the same model (noise + sampling
    from the game's own RandomState)."""
    from games.gomoku import Gomoku
    from mcts.native_mcts import NativeSelfPlay
    from mcts.new_mcts_alpha import MCTS
    from network import PyTorchModel
    import selfplay

    g = load_golden("3x64")
    m = PyTorchModel(device="cuda")
    m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state(g).items()})
    temp = lambda n: 1.0 if n < 4 else 0.0
    seeds = [101, 202, 303, 404, 505, 606, 707, 808]
    kw = dict(cpuct=1.2, dirichlet_alpha=0.3, epsilon=0.25, apply_dirichlet_n_first_moves=3)
    sp = NativeSelfPlay(m.predict, Gomoku, len(seeds), 48, **kw)
    together = sp.play(temp, max_moves=8, use_symmetries=False, seeds=seeds)
    assert sp.max_batch > 32
    # int8 leaves + on-GPU encode + pinned async evaluation in 2 pipelined groups
    pipe = NativeSelfPlay(None, Gomoku, len(seeds), 48, evaluator_factory=m.board_evaluator, groups=2, **kw)
    piped = pipe.play(temp, max_moves=8, use_symmetries=False, seeds=seeds)
    for (ea, wa), (eb, wb) in zip(together, piped):
        assert wa == wb and len(ea) == len(eb)
        for x, y in zip(ea, eb):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]
    for i in (0, 7):
        mc = MCTS(Gomoku, 48, m, cpuct=1.2, dirichlet_alpha=0.3, epsilon=0.25, apply_dirichlet_n_first_moves=3,
                  rng=np.random.RandomState(seeds[i]))
        ea, wa = selfplay.play_game_and_collect(mc, Gomoku(15), temp, max_moves=8, use_symmetries=False)
        eb, wb = together[i]
        assert wa == wb and len(ea) == len(eb)
        for x, y in zip(ea, eb):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]


def test_native_pente_10x256_selfplay_on_gpu():
    """BASELINE configs[4] shape at toy scale: Pente rules (captures) in the native
    search, 10-block/256-filter net on the GPU, pipelined int8-board evaluation ==
    the Python search played alone."""
    from games.pente import Pente
    from mcts.native_mcts import NativeSelfPlay
    from mcts.new_mcts_alpha import MCTS
    from network import PyTorchModel
    import selfplay

    torch.manual_seed(3)
    m = PyTorchModel(device="cuda", n_res_blocks=10, channels=256)
    temp = lambda n: 1.0 if n < 3 else 0.0
    seeds = [5, 6, 7, 8]
    kw = dict(cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25, apply_dirichlet_n_first_moves=2)
    sp = NativeSelfPlay(None, Pente, len(seeds), 40, evaluator_factory=m.board_evaluator, groups=2, **kw)
    out = sp.play(temp, max_moves=6, use_symmetries=False, seeds=seeds)
    mc = MCTS(Pente, 40, m, rng=np.random.RandomState(seeds[1]), **kw)
    ea, wa = selfplay.play_game_and_collect(mc, Pente(15), temp, max_moves=6, use_symmetries=False)
    eb, wb = out[1]
    assert wa == wb and len(ea) == len(eb)
    for x, y in zip(ea, eb):
        assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]
