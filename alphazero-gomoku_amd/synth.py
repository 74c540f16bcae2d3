"""Seeded synthetic positions for benchmarks: k ~ U[0,120)
stones on a random permutation of cells, colours alternating from player 1,
side to move = 1 if k is even else 2; encoded as games/gomoku.py:146-150
(plane0 = side to move, plane1 = opponent, plane2 = ones)."""
from __future__ import annotations

import numpy as np


def synth_boards(n: int, seed: int = 0, size: int = 15, max_stones: int = 120):
    rng = np.random.default_rng(seed)
    boards = np.zeros((n, size, size), dtype=np.int8)
    players = np.zeros(n, dtype=np.int8)
    for i in range(n):
        k = int(rng.integers(0, max_stones))
        cells = rng.permutation(size * size)[:k]
        flat = boards[i].reshape(-1)
        flat[cells[0::2]] = 1
        flat[cells[1::2]] = 2
        players[i] = 1 if k % 2 == 0 else 2
    return boards, players


def encode_boards(boards: np.ndarray, players: np.ndarray) -> np.ndarray:
    """[B,15,15] int8 + [B] side to move -> [B,3,15,15] float32."""
    b = np.asarray(boards)
    p = np.asarray(players).reshape(-1, 1, 1)
    out = np.empty((b.shape[0], 3) + b.shape[1:], dtype=np.float32)
    out[:, 0] = (b == p)
    out[:, 1] = (b == 3 - p)
    out[:, 2] = 1.0
    return out


def synth_encoded(n: int, seed: int = 0) -> np.ndarray:
    return encode_boards(*synth_boards(n, seed))
