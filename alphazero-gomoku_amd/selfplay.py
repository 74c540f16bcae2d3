"""Self-play data generation over the HIP engine.

Reference semantics (train.py) restated:
  * ``softmax_temperature`` / ``sample_action_from_pi``    -- train.py:252-266
  * ``play_game_and_collect``                              -- train.py:360-412
  * ``ReplayBuffer`` + pickle persistence                  -- train.py:272-354

MI355X-first part: ``BatchedSelfPlay`` advances many games at once.  Each game
owns a reference-semantics MCTS (mcts/new_mcts_alpha.py) whose leaf evaluation is
a generator yield; every round the driver concatenates the pending leaf batches
of all live games (<= 32 boards each) into one device-resident forward of up to
32 x n_games boards (BASELINE configs[2]).  The forward is bitwise
batch-independent, so every game's tree is exactly what it would be alone.
"""
from __future__ import annotations

import os
import pickle
import random
import time
from collections import deque
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch

Example = Tuple[np.ndarray, np.ndarray, float]


def softmax_temperature(pi: np.ndarray, temp: float) -> np.ndarray:
    if temp <= 0:
        return pi
    logits = np.log(pi + 1e-15) / temp
    e = np.exp(logits - np.max(logits))
    return e / np.sum(e)


def sample_action_from_pi(pi: np.ndarray, temp: float, rng=None) -> int:
    if temp == 0:
        return int(np.argmax(pi))
    p = softmax_temperature(pi, temp)
    return int((np.random if rng is None else rng).choice(len(p), p=p))


def play_game_gen(mcts, game, temp_fn: Callable[[int], float], max_moves: int = 225,
                  use_symmetries: bool = True):
    """Generator form of train.py:360-412: yields leaf batches, returns
    (examples [(state, pi, z)], winner)."""
    history = []
    move_number = 0
    while True:
        state_enc = game.get_encoded_state()
        pi = yield from mcts.run_gen(game, len(game.move_history))
        stored_pi = pi.copy()
        action = sample_action_from_pi(pi, temp_fn(move_number), getattr(mcts, "rng", None))
        if game.get_valid_moves()[action] != 1.0:       # safety fallback, train.py:380-383
            action = int(np.argmax(pi))
        history.append((state_enc, stored_pi, int(game.current_player)))
        game.do_move(divmod(action, game.size))
        move_number += 1
        if game.is_game_over() or move_number >= max_moves:
            break
    winner = game.get_winner()
    out: List[Example] = []
    for state_enc, pi_vec, who in history:
        z = 0.0 if winner == 0 else (1.0 if winner == who else -1.0)
        if use_symmetries:
            for s_aug, pi_aug in mcts.symmetries(state_enc, pi_vec):
                out.append((s_aug.astype(np.float32), pi_aug.astype(np.float32), z))
        else:
            out.append((state_enc.astype(np.float32), pi_vec.astype(np.float32), z))
    return out, winner


def play_game_and_collect(mcts, game, temp_fn, max_moves=225, use_symmetries=True):
    return mcts.drive(play_game_gen(mcts, game, temp_fn, max_moves, use_symmetries))


class BatchedSelfPlay:
    """Advance many search generators together, one device forward per round.

    ``model`` is a PyTorchModel (HIP engine), or a dict {tag: model} when the
    generators yield tagged requests (tag, X) -- e.g. evaluation games where two
    networks play each other; requests are then batched per tag.
    Statistics: ``boards`` (leaf boards evaluated), ``forwards`` (device calls),
    ``nn_seconds`` (time inside forward incl. H2D/D2H), ``max_batch``."""

    def __init__(self, model):
        self.models = model if isinstance(model, dict) else {None: model}
        self.boards = 0
        self.forwards = 0
        self.nn_seconds = 0.0
        self.max_batch = 0

    def _evaluate(self, tag, X: np.ndarray):
        t0 = time.perf_counter()
        probs, values = self.models[tag].predict(X)
        self.nn_seconds += time.perf_counter() - t0
        self.boards += len(X)
        self.forwards += 1
        self.max_batch = max(self.max_batch, len(X))
        return probs, values

    def run(self, gens: list) -> list:
        tagged = None not in self.models
        results = [None] * len(gens)
        pending = {}
        for i, g in enumerate(gens):
            try:
                pending[i] = next(g)
            except StopIteration as stop:
                results[i] = stop.value
        while pending:
            groups = {}
            for i, req in pending.items():
                tag, X = req if tagged else (None, req)
                groups.setdefault(tag, []).append((i, X))
            replies = {}
            for tag, items in groups.items():
                probs, values = self._evaluate(tag, np.concatenate([X for _, X in items], axis=0))
                off = 0
                for i, X in items:
                    n = len(X)
                    replies[i] = (probs[off:off + n], values[off:off + n])
                    off += n
            for i, reply in replies.items():
                try:
                    pending[i] = gens[i].send(reply)
                except StopIteration as stop:
                    results[i] = stop.value
                    del pending[i]
        return results


def selfplay_games(model, game_class, n_games: int, n_simulations: int, cpuct: float, temp_fn,
                   dirichlet_alpha: float, dirichlet_epsilon: float, dirichlet_n_moves: int,
                   add_dirichlet_noise: bool = True, max_moves: int = 225, use_symmetries: bool = True,
                   board_size: int = 15, driver: Optional[BatchedSelfPlay] = None, native: bool = True,
                   seeds=None):
    """n_games concurrent self-play games (train.py:671-742 semantics per game).
    Returns (examples, winners {0,1,2: count}, driver).

    native=True (default): the C++ search (mcts/native_mcts.NativeSelfPlay), every
    game with its own RandomState seeded from numpy's global RNG (or ``seeds``).
    native=False: reference-semantics Python searches advanced by BatchedSelfPlay,
    drawing from numpy's global RNG."""
    examples: List[Example] = []
    winners = {0: 0, 1: 0, 2: 0}
    if native:
        from mcts.native_mcts import NativeSelfPlay
        kw = dict(cpuct=cpuct, dirichlet_alpha=dirichlet_alpha, epsilon=dirichlet_epsilon,
                  apply_dirichlet_n_first_moves=dirichlet_n_moves, add_dirichlet_noise=add_dirichlet_noise)
        if hasattr(model, "board_evaluator"):      # HIP model: int8 leaves, GPU encode, pipelined groups
            driver = NativeSelfPlay(None, game_class, n_games, n_simulations,
                                    evaluator_factory=model.board_evaluator, groups=2 if n_games > 1 else 1, **kw)
        else:
            driver = NativeSelfPlay(model.predict, game_class, n_games, n_simulations, **kw)
        games = [game_class(size=board_size) for _ in range(n_games)]
        results = driver.play(temp_fn, max_moves=max_moves, use_symmetries=use_symmetries, seeds=seeds,
                              games=games)
    else:
        from mcts.new_mcts_alpha import MCTS
        driver = driver or BatchedSelfPlay(model)
        gens = []
        for _ in range(n_games):
            mcts = MCTS(game_class=game_class, n_simulations=n_simulations, nn_model=model, cpuct=cpuct,
                        dirichlet_alpha=dirichlet_alpha, epsilon=dirichlet_epsilon,
                        apply_dirichlet_n_first_moves=dirichlet_n_moves, add_dirichlet_noise=add_dirichlet_noise)
            game = game_class(size=board_size)
            game.current_player = 1
            gens.append(play_game_gen(mcts, game, temp_fn, max_moves=max_moves, use_symmetries=use_symmetries))
        results = driver.run(gens)
    for ex, w in results:
        examples.extend(ex)
        winners[w] = winners.get(w, 0) + 1
    return examples, winners, driver


# ---------------------------------------------------------------- replay buffer
class ReplayBuffer:
    """train.py:272-297: deque of (state [C,H,W], pi [A], z); uniform sample."""

    def __init__(self, capacity: int = 20000):
        self.capacity = capacity
        self.buffer = deque(maxlen=capacity)

    def add(self, examples):
        self.buffer.extend(examples)

    def sample(self, batch_size: int):
        batch = random.sample(self.buffer, k=batch_size)
        states, pis, zs = zip(*batch)
        return (np.stack(states, axis=0).astype(np.float32), np.stack(pis, axis=0).astype(np.float32),
                np.array(zs, dtype=np.float32).reshape(-1, 1))

    def __len__(self):
        return len(self.buffer)


def save_replay_buffer(buffer: ReplayBuffer, filepath: str) -> bool:
    """train.py:302-319 format: pickle of {'buffer': list, 'capacity': int}."""
    try:
        with open(filepath, "wb") as f:
            pickle.dump({"buffer": list(buffer.buffer), "capacity": buffer.capacity}, f,
                        protocol=pickle.HIGHEST_PROTOCOL)
        print(f"[Buffer] saved: {filepath} ({len(buffer)} samples)")
        return True
    except Exception as e:  # reference swallows errors
        print(f"[Buffer] save failed: {e}")
        return False


def load_replay_buffer(filepath: str, capacity: int) -> Optional[ReplayBuffer]:
    """train.py:322-354.  Only load buffer files this framework (or the reference
    run of the same user) wrote: pickle executes code from untrusted files."""
    if not os.path.exists(filepath):
        print(f"[Buffer] no saved buffer at {filepath}")
        return None
    try:
        with open(filepath, "rb") as f:
            data = pickle.load(f)
        buf = ReplayBuffer(capacity=capacity)
        if data.get("capacity", capacity) != capacity:
            print(f"[Buffer] warning: saved capacity {data.get('capacity')} != {capacity}")
        buf.buffer.extend(data["buffer"])
        print(f"[Buffer] loaded {filepath} ({len(buf)} samples)")
        return buf
    except Exception as e:
        print(f"[Buffer] load failed: {e}")
        return None


def examples_to_device(examples: List[Example], device) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    s = torch.from_numpy(np.stack([e[0] for e in examples]).astype(np.float32)).to(device)
    p = torch.from_numpy(np.stack([e[1] for e in examples]).astype(np.float32)).to(device)
    z = torch.tensor([e[2] for e in examples], dtype=torch.float32, device=device).reshape(-1, 1)
    return s, p, z
