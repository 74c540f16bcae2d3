"""Golden vectors for the search layer from the REFERENCE (read-only import of
/root/reference in this container), driven by tests/golden/fake_model.py:
  * mcts_argmax: reference MCTS.run pi per move of a temp-0 game, noise off
    (mcts/new_mcts_alpha.py:77-197), plus the per-move predict batch sizes;
  * mcts_noise: same with Dirichlet noise on (np.random.seed fixed);
  * collect: reference train.play_game_and_collect (train.py:360-412) with
    temperature sampling + symmetries: example count, z labels, first/last pis;
  * player: reference players/player_alpha.Player.play moves for fixed inputs.
Run: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mcts.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
sys.path.insert(0, HERE)

from fake_model import FakeModel  # noqa: E402
from games.gomoku import Gomoku  # noqa: E402  (reference)
from mcts.new_mcts_alpha import MCTS  # noqa: E402  (reference)


def argmax_game(noise: bool, n_moves: int, sims: int, seed: int):
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


def main():
    out = {}
    pis, moves, calls, nkeys = argmax_game(False, 14, 60, 0)
    out.update({"argmax/pis": pis, "argmax/moves": moves, "argmax/calls": calls, "argmax/nkeys": nkeys})
    pis, moves, calls, nkeys = argmax_game(True, 8, 60, 123)
    out.update({"noise/pis": pis, "noise/moves": moves, "noise/calls": calls, "noise/nkeys": nkeys})

    import train as ref_train  # reference train.py (play_game_and_collect)
    np.random.seed(7)
    model = FakeModel(seed=2)
    mcts = MCTS(Gomoku, 40, model, cpuct=1.2, dirichlet_alpha=0.05, epsilon=0.15,
                apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True)
    temp_fn = lambda n: max(0.0, 1.0 - n / 8)
    ex, winner = ref_train.play_game_and_collect(mcts, Gomoku(15), temp_fn, max_moves=225, use_symmetries=True)
    out["collect/n"] = len(ex)
    out["collect/winner"] = winner
    out["collect/z"] = np.array([e[2] for e in ex], dtype=np.float64)
    out["collect/states"] = np.stack([e[0] for e in ex[:16]] + [e[0] for e in ex[-8:]])
    out["collect/pis"] = np.stack([e[1] for e in ex[:16]] + [e[1] for e in ex[-8:]])

    from players.player_alpha import Player
    moves = []
    rng = np.random.default_rng(5)
    p = Player("gomoku", 15, n_simulations=48, model_path=None, nn_model=FakeModel)
    boards, lasts = [], []
    for t in range(4):
        b = np.zeros((15, 15), dtype=int)
        k = 2 * t + 1
        cells = rng.permutation(225)[:k]
        b.reshape(-1)[cells[0::2]] = 1
        b.reshape(-1)[cells[1::2]] = 2
        last = divmod(int(cells[-1]), 15)
        boards.append(b)
        lasts.append(last)
        p.mcts.clear_tree()
        moves.append(p.play(b.tolist(), t, last))
    out["player/boards"] = np.stack(boards)
    out["player/moves"] = np.array(moves)
    out["player/last"] = np.array(lasts)
    np.savez_compressed(os.path.join(HERE, "mcts_golden.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})


if __name__ == "__main__":
    main()
