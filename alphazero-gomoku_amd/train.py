"""Self-play -> train -> evaluate loop with the reference's entry point and
semantics (reference train.py:575-845), running on the HIP engine:

  * ``train_alphazero(**kwargs)`` takes every reference keyword (worker / device
    keywords are accepted and ignored: self-play and evaluation run as batched
    concurrent games on the GPU instead of CPU process pools) plus
    ``n_res_blocks`` / ``channels`` (reference default net 3x64, network.py:145-146);
  * candidate self-play (train.py:656-751), ``len(buffer)//batch_size`` train
    steps per epoch (train.py:754-765), gating by win rate (train.py:767-827) with
    the reference's optimiser-state hand-over, per-iteration snapshot + buffer
    pickle (train.py:829-840);
  * under torchrun (one process per GPU): games shard across ranks, the train
    step is data-parallel with one RCCL all-reduce of the flat gradient,
    evaluation wins are summed across ranks, BN stats averaged per iteration.
"""
from __future__ import annotations

import os
import random
import time
from datetime import datetime
from typing import Optional, Tuple

import numpy as np
import torch

import distributed as D
from games.gomoku import Gomoku as GameClass
from mcts.new_mcts_alpha import MCTS
from engine import TowerFault
from network import PyTorchModel
from selfplay import (BatchedSelfPlay, ReplayBuffer, load_replay_buffer, play_game_and_collect,  # noqa: F401
                      sample_action_from_pi, save_replay_buffer, selfplay_games, softmax_temperature)


def _tagged(gen, tag):
    """Re-label a search generator's leaf requests as (tag, X)."""
    try:
        req = next(gen)
        while True:
            req = gen.send((yield (tag, req)))
    except StopIteration as stop:
        return stop.value


def eval_game_gen(mcts_new, mcts_best, game, new_starts: bool):
    """train.py:165-245 / :418-487 game body: alternate the two searches, argmax moves."""
    move_number = 1
    while not game.is_game_over():
        if (game.current_player == 1 and new_starts) or (game.current_player == 2 and not new_starts):
            pi = yield from _tagged(mcts_new.run_gen(game, len(game.move_history)), "new")
        else:
            pi = yield from _tagged(mcts_best.run_gen(game, len(game.move_history)), "best")
        action = int(np.argmax(pi))
        game.do_move(divmod(action, game.size))
        move_number += 1
        if move_number > game.size * game.size:
            break
    return game.get_winner()


def evaluate_models(model_new: PyTorchModel, model_best: PyTorchModel, game_name: str = "gomoku",
                    n_games: int = 20, n_simulations: int = 100, cpuct: float = 1.0,
                    native: bool = True, record: Optional[list] = None) -> Tuple[int, float, int]:
    """(new_wins, win_rate, draws) over n_games (sharded across ranks), each opened
    by one random move in the centre 9x9 (train.py:440-445), new model first on
    even game indices.  native=True: both searches in C++ (mcts/native_mcts.NativeEval);
    native=False: Python searches under BatchedSelfPlay.  ``record`` (optional list)
    receives this rank's finished games."""
    size = model_new.board_size
    center, radius = size // 2, 4
    games, starts, winners, failure = [], [], [], None
    for i in D.shard(n_games):
        game = GameClass(size=size)
        game.do_move((random.randint(center - radius, center + radius), random.randint(center - radius, center + radius)))
        games.append(game)
        starts.append(i % 2 == 0)
    try:
        winners = _play_eval_games(model_new, model_best, games, starts, n_simulations, cpuct, native)
    except Exception as e:   # every rank must still reach the collective below
        failure, winners = e, []
    fault = isinstance(failure, TowerFault)
    if record is not None:
        record.extend(games)
    new_wins = sum(1 for w, s in zip(winners, starts) if (w == 1 and s) or (w == 2 and not s))
    draws = sum(1 for w in winners if w == 0)
    eng = getattr(model_new, "engine", None)
    dev = eng.device if eng is not None else "cpu"
    tot = torch.tensor([new_wins, draws, int(failure is not None), int(fault)], dtype=torch.int64, device=dev)
    D.allreduce_sum_(tot)
    new_wins, draws, failed, faults = (int(v) for v in tot.tolist())
    if faults:   # an engine fault is never a lost game: every rank re-raises it
        raise TowerFault(f"evaluation: engine fault on {faults} rank(s)" + (f": {failure}" if failure else ""))
    if failed:   # all ranks agree; the caller counts it as a loss (reference train.py:803-805)
        raise RuntimeError(f"evaluation failed on {failed} rank(s)" + (f": {failure}" if failure else ""))
    return new_wins, new_wins / float(n_games), draws


def _play_eval_games(model_new, model_best, games, starts, n_simulations, cpuct, native):
    if not games:
        winners = []
    elif native:
        from mcts.native_mcts import NativeEval
        if hasattr(model_new, "board_evaluator") and hasattr(model_best, "board_evaluator"):
            # HIP models: int8 leaves, on-GPU encoding, both networks' batches in flight
            arena = NativeEval(None, GameClass, len(games), n_simulations, cpuct=cpuct,
                               evaluator_factories={"new": model_new.board_evaluator,
                                                    "best": model_best.board_evaluator})
        else:
            arena = NativeEval({"new": model_new.predict, "best": model_best.predict}, GameClass, len(games),
                               n_simulations, cpuct=cpuct)
        winners = arena.play(games, ["new" if s else "best" for s in starts])
    else:
        gens = []
        for game, new_starts in zip(games, starts):
            mn = MCTS(GameClass, n_simulations, model_new, cpuct=cpuct, add_dirichlet_noise=False)
            mb = MCTS(GameClass, n_simulations, model_best, cpuct=cpuct, add_dirichlet_noise=False)
            gens.append(eval_game_gen(mn, mb, game, new_starts))
        winners = BatchedSelfPlay({"new": model_new, "best": model_best}).run(gens)
    return winners


def evaluate_models_mp(model_new, model_best, board_size, action_size, n_games, n_simulations, cpuct, **_ignored):
    """Reference train.py:492-569 signature; runs the batched GPU evaluation."""
    return evaluate_models(model_new, model_best, "gomoku", n_games=n_games, n_simulations=n_simulations, cpuct=cpuct)


def _new_model(board_size, action_size, device, blocks, channels, like: Optional[PyTorchModel] = None,
               with_opt: bool = False) -> PyTorchModel:
    m = PyTorchModel(board_size=board_size, action_size=action_size, device=device, n_res_blocks=blocks,
                     channels=channels)
    if like is not None:
        m.net.load_state_dict(like.net.state_dict())
        if with_opt:
            m.optimizer.load_state_dict(like.optimizer.state_dict())
    if D.world() > 1:
        m.grad_hook = D.grad_hook()
    return m


def train_alphazero(game_name: str = "gomoku", board_size: int = 15, num_iterations: int = 5,
                    games_per_iteration: int = 8, n_simulations: int = 50, buffer_size: int = 10000,
                    batch_size: int = 128, epochs_per_iter: int = 2, temp_threshold: int = 8, eval_games: int = 12,
                    eval_mcts_simulations: int = 200, win_rate_threshold: float = 0.55, cpuct: float = 1.2,
                    model_dir: str = "models", save_every: int = 1, pretrained_model_path: Optional[str] = None,
                    next_iteration_continuation: int = 1, dirichlet_alpha: float = 0.03,
                    dirichlet_epsilon: float = 0.25, dirichlet_n_moves: int = 30, n_res_blocks: int = 3,
                    channels: int = 64, device: Optional[str] = None, max_moves: Optional[int] = None,
                    **reference_worker_kwargs):
    """Reference train.py:575-845.  `reference_worker_kwargs` (selfplay_num_workers,
    selfplay_device, ..., eval_torch_threads) are accepted for drop-in use and
    ignored: concurrency comes from batching games on the GPU."""
    r, w, _, dev = D.init_from_env()
    device = device or str(dev)
    main = r == 0
    os.makedirs(model_dir, exist_ok=True)
    action_size = board_size * board_size
    if pretrained_model_path and os.path.exists(pretrained_model_path):
        if main:
            print(f"loading pretrained model: {pretrained_model_path}")
        model_best = _new_model(board_size, action_size, device, n_res_blocks, channels)
        model_best.load(pretrained_model_path)
    else:
        if main:
            print("no pretrained model: initialising a new one")
        model_best = _new_model(board_size, action_size, device, n_res_blocks, channels)
    D.broadcast_model(model_best)
    model_candidate = _new_model(board_size, action_size, device, n_res_blocks, channels, like=model_best)

    suffix = "" if r == 0 else f"_rank{r}"
    buffer_path = os.path.join(model_dir, f"replay_buffer_latest{suffix}.pkl")
    buffer = load_replay_buffer(buffer_path, capacity=buffer_size) or ReplayBuffer(capacity=buffer_size)
    temp_fn = lambda n: max(0.0, 1.0 - n / temp_threshold)
    max_moves = max_moves or board_size * board_size
    last = next_iteration_continuation + num_iterations - 1
    for it in range(next_iteration_continuation, last + 1):
        t0 = time.time()
        if main:
            print(f"\n=== ITER {it}/{last}: self-play (games={games_per_iteration}, sims={n_simulations}, "
                  f"ranks={w}) {datetime.now():%Y-%m-%d %H:%M:%S} ===")
        n_local = len(D.shard(games_per_iteration))
        examples, winners, drv = selfplay_games(model_candidate, GameClass, n_local, n_simulations, cpuct, temp_fn,
                                                dirichlet_alpha, dirichlet_epsilon, dirichlet_n_moves,
                                                max_moves=max_moves, board_size=board_size)
        buffer.add(examples)
        t_sp = time.time() - t0
        if main:
            print(f"self-play done: {t_sp / 60:.2f} min, winners={winners}, buffer={len(buffer)}, "
                  f"leaf boards={drv.boards} ({drv.boards / max(t_sp, 1e-9):.0f} boards/s, "
                  f"max batch {drv.max_batch})")

        n_batches = D.allreduce_min_int(len(buffer) // batch_size, model_candidate.engine.device)
        if n_batches >= 1:
            loss_info = None
            for epoch in range(epochs_per_iter):
                te = time.time()
                for _ in range(n_batches):
                    s, p, z = buffer.sample(batch_size)
                    loss_info = model_candidate.train_batch(s, p, z, epochs=1)
                if main:
                    print(f"  epoch {epoch + 1}/{epochs_per_iter} {time.time() - te:.1f}s last_loss={loss_info}")
            D.sync_bn_stats(model_candidate)
        elif main:
            print(f"not enough samples (buffer={len(buffer)}, need {batch_size}): skip training")

        te = time.time()
        try:
            new_wins, win_rate, draws = evaluate_models(model_candidate, model_best, game_name, n_games=eval_games,
                                                        n_simulations=eval_mcts_simulations, cpuct=cpuct)
        except TowerFault:
            # a forward that computed on stale inputs and could not be recomputed: an
            # engine fault, not a lost evaluation -- never counted as a rejection
            raise
        except Exception as e:  # reference: evaluation failure counts as a loss (train.py:803-805)
            print(f"evaluation failed: {e}")
            new_wins, win_rate, draws = 0, 0.0, 0
        if main:
            print(f"eval done: {(time.time() - te) / 60:.2f} min, win_rate={win_rate:.3f} "
                  f"({new_wins}/{eval_games}), draws={draws}")
        if win_rate >= win_rate_threshold:
            if main:
                print(" candidate accepted -> best")
            model_best.net.load_state_dict(model_candidate.net.state_dict())
            model_best.optimizer.load_state_dict(model_candidate.optimizer.state_dict())
        elif main:
            print(" candidate rejected -> restore from best")
        model_candidate = _new_model(board_size, action_size, device, n_res_blocks, channels, like=model_best,
                                     with_opt=True)
        if main and it % save_every == 0:
            path = os.path.join(model_dir, f"snapshot_iter{it}_{datetime.now():%Y%m%d_%H%M%S}.pt")
            model_best.save(path)
            print(f" saved snapshot: {path}")
        save_replay_buffer(buffer, buffer_path)
        if main:
            print(f"iteration {it} done in {(time.time() - t0) / 60:.2f} min; winners {winners}")
    if main:
        print("\n=== training done ===")
    return model_best


if __name__ == "__main__":
    train_alphazero(game_name="gomoku", board_size=15, num_iterations=300, games_per_iteration=70,
                    n_simulations=1600, cpuct=1.0, buffer_size=60000, batch_size=128, epochs_per_iter=5,
                    temp_threshold=10, eval_games=60, eval_mcts_simulations=1600, win_rate_threshold=0.5,
                    dirichlet_alpha=0.05, dirichlet_epsilon=0.15, dirichlet_n_moves=10, model_dir="models",
                    save_every=1, pretrained_model_path=None, next_iteration_continuation=1)
