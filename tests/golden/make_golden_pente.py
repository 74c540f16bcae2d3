"""Golden vectors for Pente from the REFERENCE (read-only import of /root/reference
in this container): games/pente.py rules and mcts/new_mcts_alpha.py search on Pente,
driven by tests/golden/fake_model.py.
  * kat/*: custodian captures in all 8 directions (pente.py:114-152), a double
    capture, an edge pattern that must NOT capture, the capture win at 5 pairs
    (pente.py:209), undo_move after a capture (pente.py:84-111, its colour quirk
    included), the encoding (pente.py:180-194) and legal mask after captures;
  * play/*: 64 seeded random games (until game over or 120 moves): moves, capture
    counts after every move, final board / winner / game-over flag;
  * undo/*: every board while undoing game 0 move by move;
  * mcts_argmax/*, mcts_noise/*: reference MCTS.run pi per move from a mid-game
    position with captures available (noise off / on), leaf batch sizes, tree size;
  * collect/*: reference train.play_game_and_collect on Pente (sampling + symmetries).
Run: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_pente.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
sys.path.insert(0, HERE)

from fake_model import FakeModel  # noqa: E402
from games.pente import Pente  # noqa: E402  (reference)
from mcts.new_mcts_alpha import MCTS  # noqa: E402  (reference)

DIRS = [(1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, -1), (1, -1), (-1, 1)]


def snap(g):
    return (g.board.astype(np.int8).copy(), np.array([g.captures[1], g.captures[2]], np.int64),
            int(g.get_winner()), bool(g.is_game_over()))


def kat(out):
    boards, caps, winners, over, after_undo, caps_undo, encs, masks = [], [], [], [], [], [], [], []
    setups = []
    for dr, dc in DIRS:                                   # single capture per direction
        g = Pente(15)
        r, c = 7, 7
        g.board[r + dr, c + dc] = 2
        g.board[r + 2 * dr, c + 2 * dc] = 2
        g.board[r + 3 * dr, c + 3 * dc] = 1
        g.current_player = 1
        setups.append((g, (r, c)))
    g = Pente(15)                                         # double capture: (1,0) and (0,1)
    for dr, dc in ((1, 0), (0, 1)):
        g.board[7 + dr, 7 + dc] = 2
        g.board[7 + 2 * dr, 7 + 2 * dc] = 2
        g.board[7 + 3 * dr, 7 + 3 * dc] = 1
    g.current_player = 1
    setups.append((g, (7, 7)))
    g = Pente(15)                                         # edge: X O O off-board -> no capture
    g.board[0, 1] = 2
    g.board[0, 2] = 2
    g.current_player = 1
    setups.append((g, (0, 0)))
    g = Pente(15)                                         # player 2 captures
    g.board[3, 4] = 1
    g.board[3, 5] = 1
    g.board[3, 6] = 2
    g.current_player = 2
    setups.append((g, (3, 3)))
    g = Pente(15)                                         # capture win: 4 pairs + 1
    g.captures[1] = 4
    g.board[10, 11] = 2
    g.board[10, 12] = 2
    g.board[10, 13] = 1
    g.current_player = 1
    setups.append((g, (10, 10)))
    for g, mv in setups:
        g0 = g.board.copy()
        setup_caps = np.array([g.captures[1], g.captures[2]], np.int64)
        g.do_move(mv)
        b, cp, w, o = snap(g)
        boards.append(b)
        caps.append(cp)
        winners.append(w)
        over.append(o)
        encs.append(g.get_encoded_state())
        masks.append(g.get_valid_moves())
        g.undo_move()
        after_undo.append(g.board.astype(np.int8).copy())
        caps_undo.append(np.array([g.captures[1], g.captures[2]], np.int64))
        out.setdefault("kat/setup", []).append(g0.astype(np.int8))
        out.setdefault("kat/setup_caps", []).append(setup_caps)
        out.setdefault("kat/move", []).append(np.array(mv))
        out.setdefault("kat/setup_player", []).append(1 if mv != (3, 3) else 2)
    out["kat/board"] = np.stack(boards)
    out["kat/caps"] = np.stack(caps)
    out["kat/winner"] = np.array(winners)
    out["kat/over"] = np.array(over)
    out["kat/enc"] = np.stack(encs)
    out["kat/mask"] = np.stack(masks)
    out["kat/undo_board"] = np.stack(after_undo)
    out["kat/undo_caps"] = np.stack(caps_undo)
    for k in ("kat/setup", "kat/setup_caps", "kat/move", "kat/setup_player"):
        out[k] = np.stack(out[k]) if k != "kat/setup_player" else np.array(out[k])


def playouts(out, n_games=64, max_moves=120):
    moves = np.full((n_games, max_moves), -1, np.int16)
    caps = np.zeros((n_games, max_moves, 2), np.int8)
    nmoves = np.zeros(n_games, np.int16)
    final = np.zeros((n_games, 15, 15), np.int8)
    winner = np.zeros(n_games, np.int8)
    over = np.zeros(n_games, bool)
    undo_boards = None
    for gi in range(n_games):
        rng = np.random.RandomState(1000 + gi)
        g = Pente(15)
        k = 0
        while k < max_moves and not g.is_game_over():
            v = np.nonzero(g.get_valid_moves())[0]
            a = int(rng.choice(v))
            g.do_move(divmod(a, 15))
            moves[gi, k] = a
            caps[gi, k] = (g.captures[1], g.captures[2])
            k += 1
        nmoves[gi] = k
        final[gi] = g.board
        winner[gi] = g.get_winner()
        over[gi] = g.is_game_over()
        if gi == 0:
            ub = []
            while g.move_history:
                g.undo_move()
                ub.append(g.board.astype(np.int8).copy())
            undo_boards = np.stack(ub)
    out.update({"play/moves": moves, "play/caps": caps, "play/n": nmoves, "play/final": final,
                "play/winner": winner, "play/over": over, "undo/boards": undo_boards})


def midgame(seed=37, n=70):   # both sides have a captured pair; 5 capturing moves open
    rng = np.random.RandomState(seed)
    g = Pente(15)
    while len(g.move_history) < n and not g.is_game_over():
        v = np.nonzero(g.get_valid_moves())[0]
        g.do_move(divmod(int(rng.choice(v)), 15))
    return g


def mcts_game(out, tag, noise, n_moves, sims, seed):
    np.random.seed(seed)
    model = FakeModel(seed=1)
    mcts = MCTS(Pente, sims, model, cpuct=1.0, dirichlet_alpha=0.3, epsilon=0.25,
                apply_dirichlet_n_first_moves=40, add_dirichlet_noise=noise)
    g = midgame()
    out[f"{tag}/start_moves"] = np.array(g.move_history)
    pis, moves, caps = [], [], []
    for _ in range(n_moves):
        if g.is_game_over():
            break
        pi = mcts.run(g, len(g.move_history))
        a = int(np.argmax(pi))
        pis.append(np.asarray(pi, dtype=np.float64))
        moves.append(a)
        g.do_move(divmod(a, 15))
        caps.append((g.captures[1], g.captures[2]))
    out[f"{tag}/pis"] = np.stack(pis)
    out[f"{tag}/moves"] = np.array(moves)
    out[f"{tag}/caps"] = np.array(caps)
    out[f"{tag}/calls"] = np.array(model.calls)
    out[f"{tag}/nkeys"] = len(mcts.P)


def main():
    out = {}
    kat(out)
    playouts(out)
    mcts_game(out, "mcts_argmax", False, 12, 60, 0)
    mcts_game(out, "mcts_noise", True, 8, 60, 123)
    import train as ref_train  # reference train.py (play_game_and_collect)
    np.random.seed(7)
    model = FakeModel(seed=2)
    mcts = MCTS(Pente, 40, model, cpuct=1.2, dirichlet_alpha=0.05, epsilon=0.15,
                apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True)
    ex, winner = ref_train.play_game_and_collect(mcts, Pente(15), lambda n: max(0.0, 1.0 - n / 8), max_moves=225,
                                                 use_symmetries=True)
    out["collect/n"] = len(ex)
    out["collect/winner"] = winner
    out["collect/z"] = np.array([e[2] for e in ex], dtype=np.float64)
    out["collect/states"] = np.stack([e[0] for e in ex[:16]] + [e[0] for e in ex[-8:]])
    out["collect/pis"] = np.stack([e[1] for e in ex[:16]] + [e[1] for e in ex[-8:]])
    np.savez_compressed(os.path.join(HERE, "pente_golden.npz"), **out)
    print({k: np.asarray(v).shape for k, v in out.items()})
    print("play: winners", np.bincount(out["play/winner"], minlength=3), "captures max",
          out["play/caps"].max(), "mcts caps", out["mcts_argmax/caps"][-1], out["mcts_noise/caps"][-1],
          "collect", len(ex), winner)


if __name__ == "__main__":
    main()
