"""Game-level parity of the HIP path with the oracle.

The forward is checked against the oracle board by board elsewhere (<= 1e-5); here
whole games are: the SAME games (same seeds, openings, search code) are played once
with the product's HIP evaluation and once with the oracle's CPU `predict`
(oracle/ref_net.py, same weights: the reference's 20-step goldens), and must agree
move for move.  Two fp32 implementations of the net agree to ~1e-6, so a search can
only take another branch where two PUCT scores tie within that; such a flip moves a
visit or two, and a game diverges only where that changes the played move.  A
divergence is therefore exempt only when it is explained by a near-tie: both
searches' root visit counts at that move differ by at most TIE_VISITS per action, and
the move was sampled (temperature > 0) or the root's top-2 visit gap is at most
TIE_VISITS.  Any other divergence fails, and the exempt games are gated too: at most
MAX_EXEMPT_FRAC of a case's games may diverge, and the moves played identically before
any divergence must be at least MIN_MATCHED_FRAC of all moves.  The
headline case runs configs[2]'s settings: 6x128, 400 sims/move, every game to its end.

  * self-play: NativeSelfPlay over the HIP int8 board evaluators (train.py's path,
    reference train.py:360-412) vs NativeSelfPlay over the oracle's predict, Gomoku and
    Pente (reference games/pente.py, captures);
  * gating: the reference evaluation game body (train.eval_game_gen, reference
    train.py:418-487; argmax moves, no noise) in lockstep on both evaluators, and the
    product's train.evaluate_models (NativeEval, both HIP nets' board evaluators in
    flight) must reproduce the HIP lockstep games exactly.
"""
import random

import numpy as np
import pytest
import torch

from conftest import golden_state, has_gpu, load_golden

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

TIE_VISITS = 2
MAX_EXEMPT_FRAC = 0.34
MIN_MATCHED_FRAC = 0.6


def off_grid(st: dict, rel: float = 3e-4, seed: int = 17) -> dict:
    """The golden weights are fp16-representable (tests/golden/make_golden.py rounds them),
    so the split-fp16 products' lo halves of every weight are 0.  This
    moves every float parameter off the fp16 grid by a deterministic fp32 perturbation
    (w * (1 + rel * u), u ~ U(-1, 1) from a seeded generator), applied identically to the
    HIP model and the oracle."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, v in st.items():
        a = np.asarray(v)
        if a.dtype == np.float32 and not k.endswith(("running_mean", "running_var")):
            u = rng.uniform(-1.0, 1.0, a.shape).astype(np.float32)
            a = (a * (np.float32(1.0) + np.float32(rel) * u)).astype(np.float32)
        out[k] = a
    return out


def _pair(tag, blocks, ch, perturb=False):
    from network import PyTorchModel
    from oracle.ref_net import RefModel, load_numpy_state
    st = golden_state(load_golden(tag))
    if perturb:
        st = off_grid(st)
        conv = np.asarray(st["res_blocks.0.conv1.weight"])
        assert np.mean(conv.astype(np.float16).astype(np.float32) != conv) > 0.9   # lo halves nonzero
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=blocks, channels=ch)
    m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    m.net.eval()
    ref = RefModel(blocks, ch)
    load_numpy_state(ref.net, st)
    ref.net.eval()
    return m, ref


def _top2_gap(visits):
    v = np.sort(visits)[::-1]
    return float(v[0] - v[1])


def _compare(moves_h, moves_o, pis_h, pis_o, sims, sampled):
    """(identical, exempt, max visit difference before the games part, moves matched)"""
    n = min(len(moves_h), len(moves_o))
    maxdv = 0.0
    for k in range(n):
        dv = float(np.abs(np.asarray(pis_h[k]) - np.asarray(pis_o[k])).max()) * sims
        if moves_h[k] != moves_o[k]:
            vh, vo = np.asarray(pis_h[k]) * sims, np.asarray(pis_o[k]) * sims
            tie = dv <= TIE_VISITS and (sampled(k) or min(_top2_gap(vh), _top2_gap(vo)) <= TIE_VISITS)
            assert tie, f"divergence at move {k} not explained by a near-tie: visit diff {dv}, " \
                        f"top-2 gaps {_top2_gap(vh)} / {_top2_gap(vo)}"
            return False, True, max(maxdv, dv), k
        maxdv = max(maxdv, dv)
    assert len(moves_h) == len(moves_o), "one game ended before the other without a divergence"
    return True, False, maxdv, n


@pytest.mark.timeout(900)
@pytest.mark.parametrize("game,tag,blocks,ch,games,sims,moves", [
    ("gomoku", "3x64", 3, 64, 8, 100, 60), ("gomoku", "6x128", 6, 128, 4, 100, 30),
    ("gomoku", "6x128", 6, 128, 3, 400, 225),
    # the headline settings again on weights moved off the fp16 grid (every split-fp16
    # product term nonzero: VERDICT r5 next 1)
    ("gomoku", "6x128/off-grid", 6, 128, 3, 400, 225),
    # Pente (captures, reference games/pente.py) to game end: same encoding, so the 6x128 goldens
    ("pente", "6x128", 6, 128, 4, 100, 225)])
def test_selfplay_games_match_oracle(game, tag, blocks, ch, games, sims, moves):
    from games.gomoku import Gomoku
    from games.pente import Pente
    from mcts.native_mcts import NativeSelfPlay
    Game = Pente if game == "pente" else Gomoku
    m, ref = _pair(tag.split("/")[0], blocks, ch, perturb=tag.endswith("/off-grid"))
    temp = lambda n: max(0.0, 1.0 - n / 10)          # train.py:647-648
    seeds = [700 + g for g in range(games)]

    def play(**ev):
        sp = NativeSelfPlay(game_class=Game, n_games=games, n_simulations=sims, cpuct=1.0, dirichlet_alpha=0.05,
                            epsilon=0.15, **ev)
        gs = []
        for _ in range(games):
            g = Game(size=15)
            g.current_player = 1
            gs.append(g)
        res = sp.play(temp, max_moves=moves, use_symmetries=False, seeds=seeds, games=gs)
        return gs, res

    hip_games, hip_res = play(evaluate=None, evaluator_factory=m.board_evaluator)
    m.engine.check_status()
    ora_games, ora_res = play(evaluate=ref.predict)
    same = exempt = matched = 0
    worst = 0.0
    for g in range(games):
        pis_h = [pi for _, pi, _ in hip_res[g][0]]
        pis_o = [pi for _, pi, _ in ora_res[g][0]]
        ident, ex, dv, nm = _compare(hip_games[g].move_history, ora_games[g].move_history, pis_h, pis_o, sims,
                                     lambda k: temp(k) > 0)
        worst = max(worst, dv)
        matched += nm
        same += ident
        exempt += ex
        if ident:
            assert hip_res[g][1] == ora_res[g][1]
            assert all(np.array_equal(a[2], b[2]) for a, b in zip(hip_res[g][0], ora_res[g][0]))
    nmoves = sum(len(g.move_history) for g in hip_games)
    print(f"{game} {tag}: {games} self-play games x {sims} sims, {nmoves} moves: {same} identical to the oracle's, "
          f"{exempt} diverged at a near-tie (exempt), {matched} moves matched before any divergence; "
          f"max root visit difference before a divergence {worst:.0f}")
    assert same + exempt == games
    assert nmoves > games * 10
    assert exempt <= MAX_EXEMPT_FRAC * games, f"{exempt} of {games} games exempt"
    assert matched >= MIN_MATCHED_FRAC * nmoves, f"only {matched} of {nmoves} moves matched"
    if moves == 225:                       # to game end: every identical game finished on both sides
        assert all(g.is_game_over() for g in hip_games)


class _Predict:
    def __init__(self, f, board_size=15):
        self.predict = f
        self.board_size = board_size


def _eval_lockstep(ev_new, ev_best, game, new_starts, sims):
    """train.eval_game_gen on native searches, recording every root pi."""
    from games.gomoku import Gomoku
    from mcts.native_mcts import NativeMCTS
    mn = NativeMCTS(Gomoku, sims, _Predict(ev_new), cpuct=1.0, add_dirichlet_noise=False)
    mb = NativeMCTS(Gomoku, sims, _Predict(ev_best), cpuct=1.0, add_dirichlet_noise=False)
    pis = []
    move_number = 1
    while not game.is_game_over():
        if (game.current_player == 1 and new_starts) or (game.current_player == 2 and not new_starts):
            pi = mn.run(game, len(game.move_history))
        else:
            pi = mb.run(game, len(game.move_history))
        pis.append(np.asarray(pi).copy())
        game.do_move(divmod(int(np.argmax(pi)), game.size))
        move_number += 1
        if move_number > game.size * game.size:
            break
    return pis


@pytest.mark.timeout(900)
def test_gating_games_match_oracle():
    import train
    from games.gomoku import Gomoku
    sims, n = 64, 4
    new, ref_new = _pair("3x64", 3, 64)
    best, ref_best = _pair("6x128", 6, 128)
    # the product's gating (NativeEval, both nets' int8 board evaluators in flight)
    random.seed(5)
    played = []
    train.evaluate_models(new, best, "gomoku", n_games=n, n_simulations=sims, cpuct=1.0, native=True, record=played)
    openings = [g.move_history[0] for g in played]
    same = exempt = matched = total = 0
    for i, op in enumerate(openings):
        runs = {}
        for name, en, eb in (("hip", new.predict, best.predict), ("oracle", ref_new.predict, ref_best.predict)):
            g = Gomoku(size=15)
            g.do_move(op)
            pis = _eval_lockstep(en, eb, g, i % 2 == 0, sims)
            runs[name] = (g, pis)
        (gh, ph), (go, po) = runs["hip"], runs["oracle"]
        # the product path is the HIP lockstep game, move for move
        assert list(gh.move_history) == list(played[i].move_history), i
        ident, ex, _, nm = _compare(gh.move_history[1:], go.move_history[1:], ph, po, sims, lambda k: False)
        matched += nm
        total += len(gh.move_history) - 1
        same += ident
        exempt += ex
    print(f"gating: {n} games (3x64 vs 6x128, {sims} sims): {same} identical to the oracle's, {exempt} exempt")
    assert same + exempt == n
    assert exempt <= MAX_EXEMPT_FRAC * n, f"{exempt} of {n} games exempt"
    assert matched >= MIN_MATCHED_FRAC * total, f"only {matched} of {total} moves matched"
