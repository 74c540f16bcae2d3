"""15x15 Pente with custodian pair captures, reference interface and semantics
(reference games/pente.py:5-267).

  * placing at p captures an opponent pair X O O X along any of 8 directions
    (both O removed, +1 pair for the mover) (pente.py:114-152);
  * winner from ``last_move``: 5 captured pairs, or 5 in a row through it
    (pente.py:199-230);
  * encoding identical to Gomoku: capture counts are NOT encoded (pente.py:180-194);
  * ``undo_move`` restores captured stones with the colour of the player who made
    the undone move -- the reference's behaviour (pente.py:91-108), kept as is.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from games.gomoku import Gomoku

_CAPTURE_DIRS = ((1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, -1), (1, -1), (-1, 1))


class Pente(Gomoku):
    def __init__(self, size: int = 15):
        super().__init__(size)
        self.captures = {1: 0, 2: 0}
        self.capture_history: List[List[Tuple[int, int]]] = []

    def clone(self) -> "Pente":
        g = super().clone()
        g.captures = dict(self.captures)
        g.capture_history = [list(x) for x in self.capture_history]
        return g

    def _captures_at(self, r: int, c: int, who: int) -> List[Tuple[int, int]]:
        b, n, opp = self.board, self.size, 3 - who
        taken: List[Tuple[int, int]] = []
        for dr, dc in _CAPTURE_DIRS:
            r3, c3 = r + 3 * dr, c + 3 * dc
            if not (0 <= r3 < n and 0 <= c3 < n):
                continue
            r1, c1, r2, c2 = r + dr, c + dc, r + 2 * dr, c + 2 * dc
            if b[r1, c1] == opp and b[r2, c2] == opp and b[r3, c3] == who:
                b[r1, c1] = 0
                b[r2, c2] = 0
                self.captures[who] += 1
                taken += [(r1, c1), (r2, c2)]
        return taken

    def do_move(self, move: Tuple[int, int]) -> bool:
        r, c = move
        if not (0 <= r < self.size and 0 <= c < self.size) or self.board[r, c] != 0:
            return False
        who = self.current_player
        self.board[r, c] = who
        self.last_move = (r, c)
        self.move_history.append((r, c))
        self.capture_history.append(self._captures_at(r, c, who))
        self.current_player = 3 - who
        return True

    def undo_move(self) -> None:
        if not self.move_history:
            return
        self.current_player = 3 - self.current_player
        r, c = self.move_history.pop()
        taken = self.capture_history.pop()
        self.board[r, c] = 0
        if taken:
            for rr, cc in taken:
                self.board[rr, cc] = self.current_player
            self.captures[self.current_player] -= len(taken) // 2
        self.last_move = self.move_history[-1] if self.move_history else None

    def check_winner(self) -> int:
        if self.last_move is None:
            return 0
        r, c = self.last_move
        who = int(self.board[r, c])
        if who == 0:
            return 0
        if self.captures[who] >= 5:
            return who
        return who if self._line_through(r, c, who) else 0

    def display(self) -> None:
        super().display()
        print(f"captures: 1={self.captures[1]} 2={self.captures[2]}")
