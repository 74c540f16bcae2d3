"""15x15 Gomoku state with the reference's interface and semantics
(reference games/gomoku.py:5-234).

Semantics kept exactly (they define the hot path's input contract):
  * board int8 [size, size], 0 empty / 1 / 2; ``current_player`` 1 or 2;
    ``move_history`` list of (r, c); ``last_move``;
  * action index = r * size + c (gomoku.py:46-55);
  * ``get_valid_moves``: float32 [size*size], 1.0 on empty cells (gomoku.py:109-121);
  * ``get_encoded_state``: float32 [3, size, size] = (side-to-move stones,
    opponent stones, all ones) (gomoku.py:130-150);
  * winner only from ``last_move``: five or more in a row through it
    (gomoku.py:155-193); game over = winner or no empty cell (gomoku.py:195-197).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

_DIRS = ((1, 0), (0, 1), (1, 1), (1, -1))


class Gomoku:
    def __init__(self, size: int = 15):
        self.size = size
        self.board = np.zeros((size, size), dtype=np.int8)
        self.current_player = 1
        self.move_history: List[Tuple[int, int]] = []
        self.last_move: Optional[Tuple[int, int]] = None

    # -- copies / actions -------------------------------------------------
    def clone(self) -> "Gomoku":
        g = self.__class__.__new__(self.__class__)
        g.size = self.size
        g.board = self.board.copy()
        g.current_player = int(self.current_player)
        g.move_history = list(self.move_history)
        g.last_move = None if self.last_move is None else tuple(self.last_move)
        return g

    @property
    def action_size(self) -> int:
        return self.size * self.size

    def action_to_move(self, action: int) -> Tuple[int, int]:
        return divmod(int(action), self.size)

    def move_to_action(self, move: Tuple[int, int]) -> int:
        return int(move[0] * self.size + move[1])

    # -- moves --------------------------------------------------------------
    def do_move(self, move: Tuple[int, int]) -> bool:
        r, c = move
        if not (0 <= r < self.size and 0 <= c < self.size) or self.board[r, c] != 0:
            return False
        self.board[r, c] = self.current_player
        self.move_history.append((r, c))
        self.last_move = (r, c)
        self.current_player = 3 - self.current_player
        return True

    def undo_move(self) -> None:
        if not self.move_history:
            return
        r, c = self.move_history.pop()
        self.board[r, c] = 0
        self.current_player = 3 - self.current_player
        self.last_move = self.move_history[-1] if self.move_history else None

    def get_legal_moves(self) -> List[Tuple[int, int]]:
        rs, cs = np.nonzero(self.board == 0)
        return list(zip(rs.tolist(), cs.tolist()))

    def has_legal_moves(self) -> bool:
        return bool((self.board == 0).any())

    def get_valid_moves(self) -> np.ndarray:
        return (self.board.reshape(-1) == 0).astype(np.float32)

    # -- encoding -----------------------------------------------------------
    def get_state(self) -> np.ndarray:
        return self.board.copy()

    def get_encoded_state(self) -> np.ndarray:
        out = np.empty((3, self.size, self.size), dtype=np.float32)
        out[0] = self.board == self.current_player
        out[1] = self.board == 3 - self.current_player
        out[2] = 1.0
        return out

    # -- result ---------------------------------------------------------------
    def _line_through(self, r: int, c: int, who: int) -> bool:
        b, n = self.board, self.size
        for dr, dc in _DIRS:
            run = 1
            for sgn in (1, -1):
                rr, cc = r + sgn * dr, c + sgn * dc
                while 0 <= rr < n and 0 <= cc < n and b[rr, cc] == who:
                    run += 1
                    rr += sgn * dr
                    cc += sgn * dc
            if run >= 5:
                return True
        return False

    def check_winner(self) -> int:
        if self.last_move is None:
            return 0
        r, c = self.last_move
        who = int(self.board[r, c])
        if who == 0:
            return 0
        return who if self._line_through(r, c, who) else 0

    def is_game_over(self) -> bool:
        return self.check_winner() != 0 or not self.has_legal_moves()

    def get_winner(self) -> int:
        return self.check_winner()

    def display(self) -> None:
        marks = {0: " - ", 1: " X ", 2: " O "}
        print("    " + " ".join(f"{i + 1:2}" for i in range(self.size)))
        for r in range(self.size):
            print(f"{r + 1:2}  " + "".join(marks[int(v)] for v in self.board[r]))
        print(f"to move: player {self.current_player}")
