"""Native (C++) search behind the reference MCTS interface
(reference mcts/new_mcts_alpha.py:21-97), and the multi-game self-play engine
built on it.

``NativeMCTS`` is a drop-in for ``mcts.new_mcts_alpha.MCTS``: same constructor,
``run(game, move_number) -> pi``, ``run_gen`` (leaf batches as generator yields),
``clear_tree``, ``symmetries``.  The tree walk, PUCT, backup, leaf queue and
prior installation run in libazg_mcts.so with the reference's exact float32 /
float64 arithmetic; only the Dirichlet draw (numpy, same call as the reference)
and the noise mix stay in Python, so RNG streams are the reference's.

``NativeSelfPlay`` plays many games at once: every round one ``advance`` call runs
all games' searches in parallel on host threads (OpenMP) up to their next leaf
flush, one batched forward evaluates every pending leaf, one ``feed`` installs
them.  Each game owns a ``numpy.random.RandomState`` (Dirichlet noise and move
sampling), so a game's result does not depend on which other games share its
batches or on thread scheduling -- it equals that game played alone through the
reference-semantics Python search with the same RandomState.
"""
from __future__ import annotations

import time
from typing import Callable, List, Optional, Sequence

import numpy as np

from _native_mcts import DONE, NEED_EVAL, SearchForest
from mcts.new_mcts_alpha import MCTS as _PyMCTS


def _rules_of(game_class) -> int:
    return 1 if hasattr(game_class(), "captures") else 0


def _mix_noise(p32: np.ndarray, rng, alpha: float, eps: float) -> np.ndarray:
    """new_mcts_alpha.py:176-179 verbatim in numpy: float32 prior, float64 noise."""
    noise = rng.dirichlet([alpha] * len(p32))
    p = (1 - eps) * p32 + eps * noise
    p /= np.sum(p)
    return p


class NativeMCTS:
    symmetries = _PyMCTS.symmetries
    drive = _PyMCTS.drive

    def __init__(self, game_class, n_simulations, nn_model, cpuct=1.0, batch_size=32, dirichlet_alpha=0.03,
                 epsilon=0.03, apply_dirichlet_n_first_moves=10, add_dirichlet_noise=True, rng=None, n_threads=1):
        self.game_class = game_class
        self.n_simulations = n_simulations
        self.nn_model = nn_model
        self.cpuct = cpuct
        self.batch_size = batch_size
        self.dirichlet_alpha = dirichlet_alpha
        self.epsilon = epsilon
        self.apply_dirichlet_n_first_moves = apply_dirichlet_n_first_moves
        self.add_dirichlet_noise = add_dirichlet_noise
        self.rng = np.random if rng is None else rng
        g0 = game_class()
        self.action_size = g0.size ** 2
        self.forest = SearchForest(1, n_simulations, rules=_rules_of(game_class), board=g0.size, cpuct=cpuct,
                                   batch_size=batch_size, dirichlet_alpha=dirichlet_alpha, epsilon=epsilon,
                                   apply_dirichlet_n_first_moves=apply_dirichlet_n_first_moves,
                                   add_dirichlet_noise=add_dirichlet_noise, n_threads=n_threads)

    def clear_tree(self):
        self.forest.clear(0)

    def tree_size(self) -> int:
        return self.forest.tree_size(0)

    def run(self, game_state, move_number):
        return self.drive(self.run_gen(game_state, move_number))

    def run_gen(self, game_state, move_number):
        f = self.forest
        f.set_root(0, game_state, move_number)
        while True:
            n = f.advance()
            if f.status[0] != NEED_EVAL:
                break
            probs, values = yield f.leaves[:n].copy()
            f.feed(probs, values)
            p32 = f.noise_request(0)
            if p32 is not None:
                f.set_root_prior(0, _mix_noise(p32, self.rng, self.dirichlet_alpha, self.epsilon))
        return f.get_pi(0)


class PlanesEvaluator:
    """Synchronous adapter: the search emits float32 planes, ``evaluate(X)`` returns
    (probs, values) -- e.g. PyTorchModel.predict or a test double."""

    def __init__(self, evaluate: Callable, forest: SearchForest):
        self.evaluate, self.forest, self.result = evaluate, forest, None

    def advance(self) -> int:
        return self.forest.advance()

    def submit(self, n: int) -> None:
        self.result = self.evaluate(self.forest.leaves[:n])

    def wait(self):
        return self.result


class _BoardsAdapter:
    """Board-mode adapter around an evaluator with pinned ``boards``/``players``
    staging and asynchronous ``submit(n)`` / ``wait()`` (network.BoardEvaluator)."""

    def __init__(self, ev, forest: SearchForest):
        self.ev, self.forest = ev, forest

    def advance(self) -> int:
        return self.forest.advance_boards(self.ev.boards, self.ev.players)

    def submit(self, n: int) -> None:
        self.ev.submit(n)

    def wait(self):
        return self.ev.wait()


class NativeSelfPlay:
    """Concurrent self-play games over native search forests (train.py:360-412 per game).

    Evaluation, one of:
      * ``evaluate(X float32 [n,3,H,W]) -> (probs, values)``: synchronous, one forest;
      * ``evaluator_factory(capacity) -> evaluator`` with pinned ``boards``/``players``
        staging and async ``submit(n)``/``wait()`` (PyTorchModel.board_evaluator): the
        games are split into ``groups`` forests and the host searches one group while
        the GPU evaluates another (leaves cross PCIe as int8 boards, encoded on the GPU).
    Every game draws from its own RandomState, so results are identical in both modes
    and for any grouping.  Statistics: boards, forwards, nn_seconds (host time waiting
    for / inside evaluation), search_seconds, max_batch."""

    def __init__(self, evaluate: Optional[Callable], game_class, n_games: int, n_simulations: int,
                 cpuct: float = 1.0, batch_size: int = 32, dirichlet_alpha: float = 0.03, epsilon: float = 0.03,
                 apply_dirichlet_n_first_moves: int = 10, add_dirichlet_noise: bool = True, n_threads: int = 0,
                 evaluator_factory: Optional[Callable] = None, groups: int = 2):
        if (evaluate is None) == (evaluator_factory is None):
            raise ValueError("give exactly one of evaluate / evaluator_factory")
        self.game_class = game_class
        self.n_games = n_games
        self.alpha, self.eps = dirichlet_alpha, epsilon
        g0 = game_class()
        self.board = g0.size
        K = 1 if evaluate is not None else max(1, min(groups, n_games))
        bounds = [n_games * k // K for k in range(K + 1)]
        self.slices = [(bounds[k], bounds[k + 1]) for k in range(K)]
        self.forests, self.evals = [], []
        for lo, hi in self.slices:
            f = SearchForest(hi - lo, n_simulations, rules=_rules_of(game_class), board=g0.size, cpuct=cpuct,
                             batch_size=batch_size, dirichlet_alpha=dirichlet_alpha, epsilon=epsilon,
                             apply_dirichlet_n_first_moves=apply_dirichlet_n_first_moves,
                             add_dirichlet_noise=add_dirichlet_noise, n_threads=n_threads)
            self.forests.append(f)
            if evaluate is not None:
                self.evals.append(PlanesEvaluator(evaluate, f))
            else:
                self.evals.append(_BoardsAdapter(evaluator_factory((hi - lo) * batch_size), f))
        self.forest = self.forests[0]
        self.boards = self.forwards = self.max_batch = 0
        self.moves = self.rounds = 0
        self.game_lengths: List[int] = []
        self.nn_seconds = self.search_seconds = 0.0

    def play(self, temp_fn: Callable[[int], float], max_moves: int = 225, use_symmetries: bool = True,
             seeds: Optional[Sequence[int]] = None, games: Optional[list] = None,
             progress: Optional[Callable[[int], None]] = None):
        """Play one game per slot to the end; returns [(examples, winner)] in slot
        order.  ``seeds`` seed each game's RandomState (default: drawn from numpy's
        global RNG); ``games`` optionally gives the starting positions; ``progress``
        (optional) is called with the number of live games once per round."""
        G = self.n_games
        if seeds is None:
            seeds = np.random.randint(0, 2 ** 31 - 1, size=G)
        rngs = [np.random.RandomState(int(s)) for s in seeds]
        if games is None:
            games = []
            for _ in range(G):
                g = self.game_class(size=self.board)
                g.current_player = 1
                games.append(g)
        hist: List[list] = [[] for _ in range(G)]
        moves = [0] * G
        results = [None] * G
        live = [0] * len(self.forests)
        for k, (lo, hi) in enumerate(self.slices):
            f = self.forests[k]
            for g in range(lo, hi):
                f.clear(g - lo)          # a fresh tree per game, reused across its moves
                f.set_root(g - lo, games[g], len(games[g].move_history))
            live[k] = hi - lo
        pending = [False] * len(self.forests)
        while any(live) or any(pending):
            if progress is not None:
                progress(sum(live))
            for k, (lo, hi) in enumerate(self.slices):
                f, ev = self.forests[k], self.evals[k]
                t0 = time.perf_counter()
                if pending[k]:
                    probs, values = ev.wait()
                    t1 = time.perf_counter()
                    self.nn_seconds += t1 - t0
                    t0 = t1
                    f.feed(probs, values)
                    for i in np.nonzero(f.status == NEED_EVAL)[0]:
                        p32 = f.noise_request(int(i))
                        if p32 is not None:
                            f.set_root_prior(int(i), _mix_noise(p32, rngs[lo + i], self.alpha, self.eps))
                    pending[k] = False
                if not live[k]:
                    self.search_seconds += time.perf_counter() - t0
                    continue
                # advance; if no leaf came out (every live game of the group finished its move
                # search this round) play the moves and advance again at once, so the group's
                # next forward is submitted before the host turns to the other group (the GPU
                # would otherwise idle through a whole group's move processing)
                while True:
                    n = ev.advance()
                    done = np.nonzero(f.status == DONE)[0]
                    if n:
                        # the leaves are staged: the GPU starts on them while the host plays
                        # the finished games' moves (their trees hold no pending leaves, so
                        # this order changes no result)
                        t1 = time.perf_counter()
                        ev.submit(n)
                        dt = time.perf_counter() - t1
                        self.nn_seconds += dt
                        t0 += dt            # search_seconds excludes the submit
                        pending[k] = True
                        self.boards += n
                        self.forwards += 1
                        self.max_batch = max(self.max_batch, n)
                    self._play_done(f, done, lo, games, hist, moves, results, live, k, rngs, temp_fn, max_moves,
                                    use_symmetries)
                    if pending[k] or not live[k] or not len(done):
                        break
                self.search_seconds += time.perf_counter() - t0
        self.rounds = max(self.rounds, max(moves) if moves else 0)
        return results

    def _play_done(self, f, done, lo, games, hist, moves, results, live, k, rngs, temp_fn, max_moves,
                   use_symmetries):
        """Games whose move search finished: sample (per-game RNG), play, restart."""
        from selfplay import sample_action_from_pi
        for i in done:
            i = int(i)
            g = lo + i
            game = games[g]
            pi = f.get_pi(i)
            state_enc = game.get_encoded_state()
            action = sample_action_from_pi(pi, temp_fn(moves[g]), rngs[g])
            if game.get_valid_moves()[action] != 1.0:
                action = int(np.argmax(pi))
            hist[g].append((state_enc, pi.copy(), int(game.current_player)))
            game.do_move(divmod(action, game.size))
            moves[g] += 1
            self.moves += 1
            if game.is_game_over() or moves[g] >= max_moves:
                results[g] = self._finish(hist[g], game.get_winner(), use_symmetries)
                self.game_lengths.append(moves[g])
                live[k] -= 1
            else:
                f.set_root(i, game, len(game.move_history))

    @staticmethod
    def _finish(history, winner, use_symmetries):
        """A finished game's examples: per position (in order) its 8 dihedral images in
        _PyMCTS.symmetries' order (rotation k, then its horizontal flip) with the outcome
        from the mover's view.  The images are formed for the whole game at once (8 array
        ops instead of 8 per position: the per-position form stalled the GPU for tens of ms
        when many games ended in one round); the values are the same permutations."""
        if not history:
            return [], winner
        zs = [0.0 if winner == 0 else (1.0 if winner == who else -1.0) for _, _, who in history]
        S = np.stack([h[0] for h in history]).astype(np.float32)          # [T, C, n, n]
        n = S.shape[2]
        P = np.stack([h[1] for h in history]).astype(np.float32).reshape(len(history), n, n)
        if not use_symmetries:
            return [(S[t], P[t].reshape(-1), zs[t]) for t in range(len(history))], winner
        imgs = []
        for k in range(4):
            s_k = np.rot90(S, k, axes=(2, 3))
            p_k = np.rot90(P, k, axes=(1, 2))
            imgs.append((np.ascontiguousarray(s_k), np.ascontiguousarray(p_k).reshape(len(history), -1)))
            imgs.append((np.ascontiguousarray(np.flip(s_k, axis=3)),
                         np.ascontiguousarray(np.flip(p_k, axis=2)).reshape(len(history), -1)))
        out = [(si[t], pi[t], zs[t]) for t in range(len(history)) for si, pi in imgs]
        return out, winner


class NativeEval:
    """Evaluation games between two networks (reference train.py:418-487 game body,
    = train.eval_game_gen): every game keeps one native tree per network; the side to
    move searches its own tree and plays argmax(pi).  Each round the pending leaves
    of all games are evaluated with ONE forward per network.

    ``evaluators`` {tag: evaluate(X float planes) -> (probs, values)} (synchronous), or
    ``evaluator_factories`` {tag: factory(capacity)} giving pinned int8-board
    evaluators (PyTorchModel.board_evaluator): the leaves leave the search as int8
    boards, are encoded on the GPU, both networks' batches are submitted before
    either is waited on, and the masked priors come back (same results: the
    search's own masking of an already-masked prior is the identity)."""

    def __init__(self, evaluators: Optional[dict], game_class, n_games: int, n_simulations: int,
                 cpuct: float = 1.0, batch_size: int = 32, n_threads: int = 0,
                 evaluator_factories: Optional[dict] = None):
        if (evaluators is None) == (evaluator_factories is None):
            raise ValueError("give exactly one of evaluators / evaluator_factories")
        self.tags = list(evaluators if evaluators is not None else evaluator_factories)
        self.evaluators = evaluators
        self.boards_ev = None if evaluator_factories is None else \
            {t: f(n_games * batch_size) for t, f in evaluator_factories.items()}
        self.n_games = n_games
        g0 = game_class()
        self.forests = {t: SearchForest(n_games, n_simulations, rules=_rules_of(game_class), board=g0.size,
                                        cpuct=cpuct, batch_size=batch_size, add_dirichlet_noise=False,
                                        n_threads=n_threads) for t in self.tags}
        self.boards = self.forwards = self.max_batch = 0
        self.nn_seconds = self.search_seconds = 0.0

    def play(self, games: list, first_tag: list) -> list:
        """games[g] already opened; first_tag[g] = tag of the network playing
        player 1.  Returns the winners (0 draw, 1, 2) in slot order."""
        G = len(games)
        assert G == self.n_games and len(first_tag) == G
        other = {self.tags[0]: self.tags[1], self.tags[1]: self.tags[0]}
        winners = [None] * G
        move_no = [1] * G
        to_move = {}

        def start(g):
            game = games[g]
            tag = first_tag[g] if game.current_player == 1 else other[first_tag[g]]
            to_move[g] = tag
            self.forests[tag].set_root(g, game, len(game.move_history))

        for f in self.forests.values():
            for g in range(G):
                f.clear(g)
        for g in range(G):
            if games[g].is_game_over():
                winners[g] = games[g].get_winner()
            else:
                start(g)
        while to_move:
            t0 = time.perf_counter()
            if self.boards_ev is None:
                ns = {t: f.advance() for t, f in self.forests.items()}
            else:
                ns = {t: f.advance_boards(self.boards_ev[t].boards, self.boards_ev[t].players)
                      for t, f in self.forests.items()}
            self.search_seconds += time.perf_counter() - t0
            t0 = time.perf_counter()
            if self.boards_ev is not None:     # both networks' batches in flight, then the moves
                for t, n in ns.items():        # (finished trees hold no pending leaves)
                    if n:
                        self.boards_ev[t].submit(n)
            self.nn_seconds += time.perf_counter() - t0
            for g in sorted(to_move):
                f = self.forests[to_move[g]]
                if f.status[g] != DONE:
                    continue
                game = games[g]
                action = int(np.argmax(f.get_pi(g)))
                game.do_move(divmod(action, game.size))
                move_no[g] += 1
                if game.is_game_over() or move_no[g] > game.size * game.size:
                    winners[g] = game.get_winner()
                    del to_move[g]
                else:
                    start(g)
            t0 = time.perf_counter()
            for t, n in ns.items():
                if not n:
                    continue
                f = self.forests[t]
                if self.boards_ev is None:
                    probs, values = self.evaluators[t](f.leaves[:n])
                else:
                    probs, values = self.boards_ev[t].wait()
                self.boards += n
                self.forwards += 1
                self.max_batch = max(self.max_batch, n)
                f.feed(probs, values)
            self.nn_seconds += time.perf_counter() - t0
        return winners
