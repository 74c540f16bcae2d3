"""Batched-leaf PUCT search with the reference's semantics
(reference mcts/new_mcts_alpha.py:4-197), restructured so that the point where
the reference calls ``nn_model.predict`` is a generator yield: one search can run
standalone (``run``), or many searches (one per concurrent game) can be advanced
together by a driver that evaluates all their pending leaves in ONE batched GPU
forward (selfplay.py).  Because the HIP forward is bitwise batch-independent,
both ways give identical trees.

Reference behaviour reproduced on purpose:
  * tree = dicts P, V, N, W, children keyed by board.tobytes() + bytes([player]);
  * new leaf: queued, given a uniform prior over valid moves, V = 0, and the
    simulation returns 0 at once (no virtual loss);
  * when the queue reaches ``batch_size`` (32), every queued key is (re)installed:
    p = prior * valid (NOT renormalised), uniform fallback if sum < 1e-8, root-only
    Dirichlet mix + renormalise, N = W = 0 (also resets a key visited meanwhile);
    the simulation that filled the queue then continues from the now-evaluated node;
  * PUCT: Q = W / (1 + N), U = cpuct * P * sqrt(sum N) / (1 + N), invalid -1e9,
    first index on ties; float32 N / W;
  * terminal: 0 for a draw, -1 for the side to move (the previous mover won);
  * pi = N / sum N at the root, or the valid-move mask normalised if N is all 0.
"""
from __future__ import annotations

import math

import numpy as np


class MCTS:
    def __init__(self, game_class, n_simulations, nn_model, cpuct=1.0, batch_size=32, dirichlet_alpha=0.03,
                 epsilon=0.03, apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True, rng=None):
        self.game_class = game_class
        # Dirichlet draws come from numpy's global RandomState (the reference's
        # np.random.dirichlet) unless a per-search RandomState is given.
        self.rng = np.random if rng is None else rng
        self.n_simulations = n_simulations
        self.nn_model = nn_model
        self.cpuct = cpuct
        self.batch_size = batch_size
        self.dirichlet_alpha = dirichlet_alpha
        self.epsilon = epsilon
        self.apply_dirichlet_n_first_moves = apply_dirichlet_n_first_moves
        self.add_dirichlet_noise = add_dirichlet_noise
        self.action_size = game_class().size ** 2
        self.clear_tree()

    # ---------------------------------------------------------------- utilities
    def symmetries(self, state, pi):
        """8 dihedral images of (state [C,H,W], pi [H*W]) in the reference's order:
        rotation k = 0..3 (np.rot90 over the board axes), then its horizontal flip."""
        n = state.shape[1]
        board_pi = pi.reshape(n, n)
        images = []
        for k in range(4):
            s_k = np.rot90(state, k, axes=(1, 2))
            p_k = np.rot90(board_pi, k)
            images.append((s_k, p_k.flatten()))
            images.append((np.flip(s_k, axis=2), np.flip(p_k, axis=1).flatten()))
        return images

    def clear_tree(self):
        self.P, self.V, self.N, self.W, self.children = {}, {}, {}, {}, {}
        self.pending_states, self.pending_keys, self.pending_game_states = [], [], []
        self.root_key = None

    @staticmethod
    def _state_key(game_state):
        return game_state.board.tobytes() + bytes([game_state.current_player])

    # ------------------------------------------------------------- entry points
    def run(self, game_state, move_number):
        """pi [action_size] after n_simulations (reference run, :77-97)."""
        return self.drive(self.run_gen(game_state, move_number))

    def search(self, game_state, move_number):
        return self.drive(self._search(game_state, move_number))

    def _predict_batch(self, move_number):
        self.drive(self._flush(move_number))

    def drive(self, gen):
        """Run a search generator to completion, answering each leaf batch with
        nn_model.predict (the standalone / reference-compatible mode)."""
        try:
            req = next(gen)
            while True:
                req = gen.send(self.nn_model.predict(req))
        except StopIteration as stop:
            return stop.value

    # ------------------------------------------------------------- generators
    def run_gen(self, game_state, move_number):
        """Generator form of run(): yields leaf batches X [b,3,H,W] float32, expects
        (probs [b,A], values [b,1]) to be sent back; returns pi."""
        self.root_key = self._state_key(game_state)
        for _ in range(self.n_simulations):
            yield from self._search(game_state.clone(), move_number)
        yield from self._flush(move_number)
        root = self._state_key(game_state)
        counts = self.N[root]
        total = np.sum(counts)
        if total > 0:
            return counts / total
        valid = self.children[root]
        return valid / np.sum(valid)

    def _search(self, game, move_number):
        key = self._state_key(game)
        if game.is_game_over():
            return 0 if game.get_winner() == 0 else -1
        if key not in self.P:
            self.pending_states.append(game.get_encoded_state())
            self.pending_keys.append(key)
            self.pending_game_states.append(game.clone())
            if len(self.pending_states) >= self.batch_size:
                yield from self._flush(move_number)
            if key not in self.P:
                valid = game.get_valid_moves()
                self.P[key] = valid / np.sum(valid)
                self.V[key] = 0
                self.N[key] = np.zeros_like(valid, dtype=np.float32)
                self.W[key] = np.zeros_like(valid, dtype=np.float32)
                self.children[key] = valid
                return self.V[key]
        n_visits = self.N[key]
        scale = math.sqrt(np.sum(n_visits))
        denom = 1 + n_visits
        score = self.W[key] / denom + self.cpuct * self.P[key] * scale / denom
        score = np.where(self.children[key] == 1, score, -1e9)
        action = np.argmax(score)
        game.do_move(divmod(action, game.size))
        value = -(yield from self._search(game, move_number))
        self.W[key][action] += value
        self.N[key][action] += 1
        return value

    def _flush(self, move_number):
        if not self.pending_states:
            return
        X = np.stack(self.pending_states, axis=0).astype(np.float32)
        policies, values = yield X
        use_noise = self.add_dirichlet_noise and move_number < self.apply_dirichlet_n_first_moves
        for key, p, v, gs in zip(self.pending_keys, policies, values, self.pending_game_states):
            p = p.flatten()
            valid = gs.get_valid_moves()
            p = p * valid
            if np.sum(p) < 1e-8:
                p = valid / np.sum(valid)
            if use_noise and key == self.root_key:
                noise = self.rng.dirichlet([self.dirichlet_alpha] * len(p))
                p = (1 - self.epsilon) * p + self.epsilon * noise
                p /= np.sum(p)
            self.P[key] = p
            self.V[key] = v[0] if hasattr(v, "__len__") else v
            self.N[key] = np.zeros_like(p, dtype=np.float32)
            self.W[key] = np.zeros_like(p, dtype=np.float32)
            self.children[key] = valid
        self.pending_states, self.pending_keys, self.pending_game_states = [], [], []
