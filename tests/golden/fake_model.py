"""Deterministic stand-in for PyTorchModel used to pin the search layer (MCTS,
self-play collection, Player) against the reference: outputs depend only on each
board (computed row by row in float64, rounded to float32), so any batching gives
identical results.  Test infrastructure only."""
import numpy as np


class _Net:
    def eval(self):
        return self

    def train(self, mode=True):
        return self


class FakeModel:
    def __init__(self, board_size=15, action_size=None, device=None, seed=0, **kw):
        rng = np.random.default_rng(seed)
        n = 3 * board_size * board_size
        self.W = rng.standard_normal((n, board_size * board_size)) * 0.35
        self.wv = rng.standard_normal(n) * 0.05
        self.board_size = board_size
        self.net = _Net()
        self.calls = []

    def load(self, path, map_location=None):
        return None

    def predict(self, X):
        X = np.asarray(X, dtype=np.float64).reshape(len(X), -1)
        logits = np.stack([row @ self.W for row in X])
        logits -= logits.max(axis=1, keepdims=True)
        p = np.exp(logits)
        p /= p.sum(axis=1, keepdims=True)
        v = np.tanh(np.array([row @ self.wv for row in X]) - 0.5)
        self.calls.append(len(X))
        return p.astype(np.float32), v.reshape(-1, 1).astype(np.float32)


class FakeBoardEvaluator:
    """Test double of network.BoardEvaluator: int8 board staging, deferred
    evaluation, masked priors (probs * valid) -- drives the pipelined native
    self-play on CPU."""

    def __init__(self, model, capacity, board_size=15):
        self.model = model
        self.boards = np.zeros((capacity, board_size * board_size), np.int8)
        self.players = np.zeros((capacity,), np.int8)
        self.n = 0
        self.out = None

    def submit(self, n):
        self.n = n
        b = self.boards[:n].astype(np.int64)
        pl = self.players[:n].astype(np.int64)[:, None]
        x = np.stack([(b == pl), (b == 3 - pl), np.ones_like(b, dtype=bool)], axis=1).astype(np.float32)
        x = x.reshape(n, 3, int(np.sqrt(b.shape[1])), -1)
        probs, values = self.model.predict(x)
        self.out = (probs * (self.boards[:n] == 0).astype(np.float32), values)

    def wait(self):
        return self.out
