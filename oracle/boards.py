"""Oracle: board encoding / legal mask restated from the reference, plus the
seeded synthetic-position generator of SURVEY.md §8(d).  TEST INFRASTRUCTURE ONLY.

* ``encode``      -- reference ``games/gomoku.py:130-150`` (Pente: ``games/pente.py:180-194``):
                     plane0 = side-to-move stones, plane1 = opponent stones, plane2 = all ones.
* ``valid_mask``  -- reference ``games/gomoku.py:109-121``: float32 (board == 0), flattened r*size+c.
"""
from __future__ import annotations

import numpy as np


def encode(board: np.ndarray, player: int) -> np.ndarray:
    board = np.asarray(board)
    n = board.shape[0]
    out = np.empty((3, n, n), dtype=np.float32)
    out[0] = (board == player)
    out[1] = (board == 3 - player)
    out[2] = 1.0
    return out


def valid_mask(board: np.ndarray) -> np.ndarray:
    return (np.asarray(board).reshape(-1) == 0).astype(np.float32)


def synth_positions(n: int, seed: int = 0, size: int = 15, max_stones: int = 120):
    """Legal-looking positions: k ~ U[0, max_stones) stones on a random permutation of
    cells, colours alternating from player 1; side to move = 1 if k even else 2."""
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


def encode_batch(boards: np.ndarray, players: np.ndarray) -> np.ndarray:
    return np.stack([encode(b, int(p)) for b, p in zip(boards, players)], axis=0)


def synth_targets(n: int, seed: int = 1, actions: int = 225):
    """Training targets: pi ~ normalised U[0,1)^A, z in {-1, 0, 1}."""
    rng = np.random.default_rng(seed)
    pi = rng.random((n, actions)).astype(np.float32)
    pi /= pi.sum(axis=1, keepdims=True)
    z = rng.integers(-1, 2, size=(n, 1)).astype(np.float32)
    return pi.astype(np.float32), z
