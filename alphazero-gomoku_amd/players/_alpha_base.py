"""AlphaZero player over the HIP policy/value engine, with the reference's
``Player(rules, board_size, ...).play(board, turn_number, last_opponent_move)``
plug-in API (reference players/player_alpha.py:7-77; loaded by play_loop.py:18-29,
play.py:19-30, gui.py:20-31 as ``module.Player(rules, size)``).

Kept from the reference on purpose: the side to move is inferred from
``turn_number % 2`` (player_alpha.py:65), a list board becomes an int (int64)
array (player_alpha.py:59-62), the search tree persists across calls, and the
move is argmax(pi) (first index on ties).

The search is the native one (mcts/native_mcts.py, bit-identical to the reference
search); ``mcts_class`` selects another implementation with the same interface
(e.g. the pure-Python mcts.new_mcts_alpha.MCTS).
"""
from __future__ import annotations

import numpy as np

from games.gomoku import Gomoku
from mcts.native_mcts import NativeMCTS


class AlphaPlayer:
    def __init__(self, rules="gomoku", board_size=15, n_simulations=5000, c_puct=1.0, model_path=None,
                 nn_model=None, mcts_kwargs=None, mcts_class=None):
        if nn_model is None:
            from network import PyTorchModel
            nn_model = PyTorchModel
        self.rules = rules.lower()
        self.board_size = board_size
        self.n_simulations = n_simulations
        self.c_puct = c_puct
        self.model_path = model_path
        self.net = nn_model(board_size=self.board_size)
        if model_path is not None:
            print(f"[PlayerAlpha] loading model: {model_path}")
            self.net.load(model_path)
        else:
            print("[PlayerAlpha] WARNING: no model given, using random weights")
        self.net.net.eval()
        if self.rules != "gomoku":
            raise ValueError(f"Unsupported rules: {self.rules}. Only 'gomoku' is supported.")
        self.game_class = Gomoku
        mcts_class = mcts_class or NativeMCTS
        self.mcts = mcts_class(game_class=self.game_class, n_simulations=self.n_simulations, nn_model=self.net,
                         cpuct=self.c_puct, add_dirichlet_noise=False, **(mcts_kwargs or {}))

    def play(self, board, turn_number, last_opponent_move):
        game = self.game_class(size=self.board_size)
        game.board = np.array(board, dtype=int) if isinstance(board, list) else np.copy(board.board)
        game.current_player = 1 if turn_number % 2 == 0 else 2
        game.last_move = last_opponent_move
        pi = self.mcts.run(game, turn_number)
        action = np.argmax(pi)
        return divmod(action, self.board_size)
