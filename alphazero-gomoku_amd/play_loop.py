"""N-game arena between two player plug-ins (reference play_loop.py, which drives
the hot path through ``players.<name>.Player(rules, size).play``).

    python play_loop.py <player1> <player2> <n_games>

Semantics kept from the reference (play_loop.py:18-245): players are loaded by
module name as ``players.<name>.Player(rules, size)``; each game opens with ONE
uniformly random move (``random.randint(0, 14)`` twice) made for player 1 and
recorded as its move; ``turn_number`` starts at 0 after that opening and counts the
moves played since (so the AlphaZero player infers the side to move from it exactly
as in the reference, quirk included); the starting player alternates between games;
a move that raises or is illegal is retried; metrics (moves, think times, wins,
draws, starting player per game) go to ``metrics/<p1>_<sims>_<p2>_<sims>_3.json``.
Board printing is behind ``verbose``.
"""
from __future__ import annotations

import importlib
import json
import os
import random
import sys
import time
from pathlib import Path

import numpy as np

from games.gomoku import Gomoku

METRICS = Path("metrics")


def load_player(module_name: str, rules: str, size: int):
    name = module_name.replace(".py", "").strip()
    if not name.startswith("players."):
        name = "players." + name
    module = importlib.import_module(name)
    if not hasattr(module, "Player"):
        raise ValueError(f"no Player class in {name}")
    return module.Player(rules, size)


def choose_game() -> str:
    return "gomoku"


def _sims(p):
    for attr in ("n_simulations", "n_playout"):
        if hasattr(p, attr):
            return getattr(p, attr)
    return None


def initiate_metrics(name1, name2, p1, p2, game_name, n_games) -> dict:
    names = (name1, name2)
    games = [f"game_{i}" for i in range(1, n_games + 1)]
    return {
        "total_duration": 0,
        "player1": (name1, _sims(p1), getattr(p1, "model_path", None)),
        "player2": (name2, _sims(p2), getattr(p2, "model_path", None)),
        "game": game_name, "n_games": n_games, "total_duration_minutes": 0,
        "move_made": {n: {g: [] for g in games} for n in names},
        "time_for_each_move": {n: {g: [] for g in games} for n in names},
        "game_duration_seconds": {g: 0 for g in games},
        "wins": {}, "draws": 0,
        "starting_player_per_game": {g: None for g in games},
    }


def change_starting_player(name1, name2, game, game_name, size, metrics, game_iter, verbose=True,
                           loader=None):
    """One game, `name1` moving first (player 1).  Returns the winner's name or None."""
    loader = loader or load_player
    key = f"game_{game_iter}"
    seat = {1: (name1, loader(name1, game_name, size)), 2: (name2, loader(name2, game_name, size))}
    metrics["starting_player_per_game"][key] = name1
    opening = (random.randint(0, 14), random.randint(0, 14))
    game.do_move(opening)
    metrics["move_made"][name1][key].append(opening)
    metrics["time_for_each_move"][name1][key].append(0)
    if verbose:
        game.display()
    turn_number = 0
    while not game.is_game_over():
        name, player = seat[game.current_player]
        while True:
            t0 = time.time()
            try:
                move = player.play(game.clone(), turn_number, game.last_move)
            except Exception as e:   # the reference retries a player that raises
                print(f"player {game.current_player} error: {e}")
                continue
            dt = time.time() - t0
            metrics["move_made"][name][key].append(move)
            metrics["time_for_each_move"][name][key].append(dt)
            if move is None:
                continue
            try:
                game.do_move(move)
            except ValueError as e:
                print(f"invalid move: {e}")
                continue
            turn_number += 1
            break
        if verbose:
            game.display()
    w = game.get_winner()
    return None if w == 0 else seat[w][0]


def to_json_safe(obj):
    if isinstance(obj, dict):
        return {k: to_json_safe(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [to_json_safe(v) for v in obj]
    if isinstance(obj, np.integer):
        return int(obj)
    if isinstance(obj, np.floating):
        return float(obj)
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    return obj


def loop_for_n_games(name1: str, name2: str, n_games: int, size: int = 15, verbose: bool = True,
                     loader=None, pause: float = 3.0) -> dict:
    loader = loader or load_player
    game_name = choose_game()
    p1, p2 = loader(name1, game_name, size), loader(name2, game_name, size)
    wins = {name1: 0, name2: 0}
    metrics = initiate_metrics(name1, name2, p1, p2, game_name, n_games)
    t_start = time.time()
    for i in range(n_games):
        first, second = (name1, name2) if i % 2 == 0 else (name2, name1)
        t0 = time.time()
        winner = change_starting_player(first, second, Gomoku(size), game_name, size, metrics, i + 1,
                                        verbose=verbose, loader=loader)
        metrics["game_duration_seconds"][f"game_{i + 1}"] = time.time() - t0
        if winner:
            wins[winner] += 1
        print(f"Finished game: {i + 1}/{n_games}")
        time.sleep(pause)
    metrics["total_duration_minutes"] = (time.time() - t_start) // 60
    metrics["wins"] = wins
    metrics["draws"] = n_games - sum(wins.values())
    return metrics


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 3:
        print("usage: python play_loop.py <player1> <player2> <n_games>")
        sys.exit(1)
    name1, name2, n = argv[0], argv[1], int(argv[2])
    os.makedirs(METRICS, exist_ok=True)
    m = loop_for_n_games(name1, name2, n)
    for k, v in m["wins"].items():
        print(f"{k} won {v} times")
    fname = f"{name1}_{m['player1'][1]}_{name2}_{m['player2'][1]}_3.json"
    with open(METRICS / fname, "w") as f:
        json.dump(to_json_safe(m), f, indent=4)


if __name__ == "__main__":
    main()
